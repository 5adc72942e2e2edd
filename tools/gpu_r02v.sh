#!/bin/bash
# r02 session 2: dense solver with one wave per SIMD: tests + C3 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py tests/test_gpu_configs.py tests/test_gpu_multirank.py -k "dense or c3" -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_v.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_v.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3v.json 2> gpurun_out/bench_c3v.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench_c3v.json').readlines()[-1]);print(d['ms_per_step'], d['time_to_gap_s'], d['rounds_to_gap'], d['kernel_ms'])"
