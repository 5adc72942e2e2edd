#!/bin/bash
# r02 session 2: dense-row and compact-deltaW tests, C3/C4 config tests, C3/C4 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_compact.py tests/test_gpu_configs.py -k "dense or compact or c3 or c4" -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_dense.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_dense.log; [ $rc -ne 0 ] && exit $rc
for c in c3 c4; do
timeout -k 10 600 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_$c.json').readlines()[-1]);print('$c', d['ms_per_step'], d['time_to_gap_s'], d['rounds_to_gap'], d['kernel_ms'], d['plan']['solver'], d['plan'].get('dw_compact'))"
done
