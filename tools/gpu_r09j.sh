#!/bin/bash
# warm eval tier (C4): tests, C4 A/B warm on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09j}
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_split.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=10 REPS=2 TAG=ab_${T}c4 tools/benchab.sh "-- --config c4" "COCOA_EVAL_WARM=0 -- --config c4" || exit $?
