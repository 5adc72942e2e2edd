#!/bin/bash
# r02 session 2: Gram-solver sensitivity to the LDS-resident deltaW columns (diag build, COCOA_GRAM_HOT caps them)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
python3 -c "
import sys; sys.path.insert(0,'.')
from cocoa_amd import Engine, configs
sh=configs.share('c2'); e=Engine(); e.set_train(sh.train); e.init('cocoa+', sh.n_glob, 10, sh.H, sh.lam); print(e.plan())" || exit 1
for h in 100000 256 64 0; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_HOT=$h timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap --steps 10 > gpurun_out/bench_hot$h.json 2> gpurun_out/bench_hot$h.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_hot$h.json').readlines()[-1]);print($h, round(d['ms_per_step'],4), round(d['kernel_ms']['solver'],4), round(d['kernel_ms']['gram'],4))"
done
