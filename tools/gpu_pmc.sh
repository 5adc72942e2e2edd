#!/bin/bash
# GPU tests, the full default bench line, rocprofv3 kernel stats and PMC traffic passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit $?
tail -1 gpurun_out/bench_full.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- $B > gpurun_out/rocprof_bench.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- $B > gpurun_out/pmc_$c.log 2>&1 || exit $?
  timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/calib_$c -o run --output-format csv -- tools/ubench/calib > gpurun_out/calib_$c.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_TCC -o run --output-format csv -- $B > gpurun_out/pmc_TCC.log 2>&1 || exit $?
echo pmc done
