#!/bin/bash
# r02 session 2: Gram solver with / without LDS deltaW columns (diag build A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for h in 1 0 1 0; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_HOTLDS=$h timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap --steps 10 > gpurun_out/bench_hl$h.json 2> gpurun_out/bench_hl$h.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_hl$h.json').readlines()[-1]);print($h, round(d['ms_per_step'],4), round(d['kernel_ms']['solver'],4), round(d['kernel_ms']['gram'],4), round(d['kernel_ms']['eval'],4))"
done
