#!/bin/bash
# r02 session 2: full GPU suite, C2 bench line with rocprof stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench.json').readlines()[-1]);print(d['ms_per_step'], d['value'], d['time_to_gap_s'], d['kernel_ms'], d['roofline_eval']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-gap > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
python3 tools/rocpd_summary.py gpurun_out/prof gpurun_out/kernel_stats.csv && head -n 8 gpurun_out/kernel_stats.csv
