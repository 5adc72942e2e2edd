#!/bin/bash
# eight runs (default layout / memory waves on four SIMDs) against four, now that the Gram rows are faster
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
T=${TAG:-r09h}
COCOA_LIB=build/v_r8s/libcocoa_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mirror.py tests/test_gpu_gram.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/gpu_tests_$T.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_$T.log | tail -3; [ $rc -eq 0 ] || exit $rc
STEPS=100 REPS=2 TAG=ab_$T tools/benchab.sh " --" "COCOA_LIB=build/v_r8/libcocoa_hip.so --" "COCOA_LIB=build/v_r8s/libcocoa_hip.so --" || exit $?
