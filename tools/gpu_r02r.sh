#!/bin/bash
# r02 session 2: full GPU suite, smoke, default bench line, rocprof kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -n 1 gpurun_out/smoke.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/bench.json').readlines()[-1]);print(d['ms_per_step'], d['value'], d['time_to_gap_s'], d['kernel_ms'], d['roofline']['frac'], d['roofline_eval']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-gap > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
python3 tools/rocpd_summary.py gpurun_out/prof gpurun_out/kernel_stats.csv && head -n 8 gpurun_out/kernel_stats.csv
