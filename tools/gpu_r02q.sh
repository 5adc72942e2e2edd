#!/bin/bash
# r02 session 2: eval with hot w in LDS -- parity tests, then A/B (diag build) of the variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_q.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_q.log; [ $rc -ne 0 ] && exit $rc
for v in 0 8192 4096 0 8192 4096; do
COCOA_LIB=build/diag/libcocoa_hip.so COCOA_EVAL_HOTW=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-gap > gpurun_out/bench_h$v.json 2> gpurun_out/bench_h$v.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_h$v.json').readlines()[-1]);print($v, round(d['ms_per_step'],4), round(d['kernel_ms']['eval'],4), round(d['kernel_ms']['solver'],4), round(d['roofline_eval']['frac'],3))"
done
