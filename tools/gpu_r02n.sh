#!/bin/bash
# r02 session 2: eval tile A/B (diag build): 4096 vs 2048-entry tiles under the Gram side stream
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 4096 2048 4096 2048; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_EVAL_TILE=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap > gpurun_out/bench_t$v.json 2> gpurun_out/bench_t$v.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_t$v.json').readlines()[-1]);print($v, round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['kernel_ms'].items()}, round(d['roofline_eval']['frac'],3))"
done
