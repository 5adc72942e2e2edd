#!/bin/bash
# r02 session 2: split-gather eval: parity tests, then A/B (diag build) against v4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_gram.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_z.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_z.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_EVAL_SPLIT=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap --steps 10 > gpurun_out/bench_sp$v.json 2> gpurun_out/bench_sp$v.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_sp$v.json').readlines()[-1]);print($v, round(d['ms_per_step'],4), round(d['kernel_ms']['eval'],4), round(d['roofline_eval']['frac'],3))"
done
