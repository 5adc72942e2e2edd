#!/bin/bash
# Headline bench (driver's default invocation) + rocprofv3 kernel stats of the same command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
tail -1 gpurun_out/bench_final.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof_final -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gap > gpurun_out/rocprof_final.log 2>&1 || exit $?
find gpurun_out/rocprof_final -name "*kernel_stats*"
