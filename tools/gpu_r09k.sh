#!/bin/bash
# warm tier opt-in: tests; C4 kernel times with the warm tier on / off (rocprof)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09k}
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_split.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
for wv in 1 0; do
  COCOA_EVAL_WARM=$wv timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_${T}_w$wv -o run -- python3 bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-gap > $O/bench_${T}_w$wv.log 2>&1 || exit $?
  f=$(find $O/prof_${T}_w$wv -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/rocprof_c4_${T}_w$wv.csv
  python3 -c "
import csv
for r in csv.DictReader(open('$O/rocprof_c4_${T}_w$wv.csv')):
    if 'eval' in r['Name']: print('warm $wv', r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3, 1), 'us')"
done
