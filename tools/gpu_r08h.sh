#!/bin/bash
# mb-SGD pull form: tests, then the C5 mb-SGD line A/B (pull / scatter)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mbsgd.py tests/test_gpu_configs.py tests/test_gpu_multirank.py \
  tests/test_gpu_multidevice.py -k "mbsgd or sgd" -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_r08h.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r08h.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=50 REPS=2 TAG=ab8h tools/benchab.sh "-- --method mbsgd" "COCOA_MBSGD_PULL=0 -- --method mbsgd" || exit $?
