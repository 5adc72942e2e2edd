#!/bin/bash
# MbCD / local SGD mirrored: tests, then the C5 lines of those methods
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_configs.py -k "mirror or c5" -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests_r08g.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r08g.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=50 REPS=2 TAG=ab8g tools/benchab.sh "-- --method mbcd" "COCOA_GRAM_MIRROR=0 -- --method mbcd" "-- --method localsgd" \
  "COCOA_GRAM_MIRROR=0 -- --method localsgd" || exit $?
