#!/bin/bash
# r02 session 2: Gram kernel v2 (warm updater image + per-partner walk): tests, bench, phase profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_configs.py tests/test_gpu_compact.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_p.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_p.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_p.json').readlines()[-1]);print(d['ms_per_step'], d['value'], d['time_to_gap_s'], d['kernel_ms'], d['roofline_eval']['frac'])"
COCOA_LIB=build/diag/libcocoa_hip.so timeout -k 10 300 python3 tools/prof_gram.py cocoa+ > gpurun_out/prof_gram_v2.json 2> gpurun_out/prof_gram_v2.err || exit $?
cat gpurun_out/prof_gram_v2.json
