#!/bin/bash
# the 4-member d = 3 case (tests/test_gpu_multidevice.py) in fresh processes, per setting
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "X=0" "COCOA_LIB=build/v_prev/libcocoa_hip.so" "COCOA_XW_PRODUCER=0" "COCOA_GRAM_MIRROR=0" "X=0" "COCOA_LIB=build/v_prev/libcocoa_hip.so"; do
  echo "== $v"
  env $v timeout -k 10 120 python3 tools/diag_fewfeat.py 2>&1 | tail -6 || exit $?
done
