#!/bin/bash
# r02 session 2: driver test + gram/dense/compact tests, C2 bench (stream priorities)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_driver.py tests/test_gpu_gram.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_m.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_m.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/bench_m$i.json 2> gpurun_out/bench_m$i.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_m$i.json').readlines()[-1]);print(d['ms_per_step'], d['value'], d['time_to_gap_s'], d['kernel_ms'], d['roofline_eval']['frac'])"
done
