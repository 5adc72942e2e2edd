#!/bin/bash
# split-eval pass shapes (build/v_*), C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 REPS=2 TAG=ab8k tools/benchab.sh " --" "COCOA_LIB=build/v_h4kb1024/libcocoa_hip.so --" \
  "COCOA_LIB=build/v_h2kb512/libcocoa_hip.so --" "COCOA_LIB=build/v_h2kb1024/libcocoa_hip.so --" \
  "COCOA_LIB=build/v_c2kb512/libcocoa_hip.so --" "COCOA_EVAL_SPLIT=0 --" || exit $?
