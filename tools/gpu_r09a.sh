#!/bin/bash
# eval passes: next-tile bounds loaded during the current tile (vs build/v_old)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_eval_split.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/gpu_tests_r09a.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r09a.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=50 REPS=2 TAG=ab9a tools/benchab.sh " --" "COCOA_LIB=build/v_old/libcocoa_hip.so --" || exit $?
STEPS=10 REPS=2 TAG=ab9ac4 tools/benchab.sh "-- --config c4" "COCOA_LIB=build/v_old/libcocoa_hip.so -- --config c4" || exit $?
