#!/bin/bash
# r02 session 2: dense solver rows-in-flight A/B on C3 (diag build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 8 0 8 0; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_DENSE_P=$p timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline --no-gap --steps 10 > gpurun_out/bench_dp$p.json 2> gpurun_out/bench_dp$p.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_dp$p.json').readlines()[-1]);print($p, round(d['ms_per_step'],4), round(d['kernel_ms']['solver'],4), round(d['kernel_ms']['eval'],4))"
done
