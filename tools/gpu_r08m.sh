#!/bin/bash
# does the mirrored solver tolerate a 32-step (2-batch) window?  (per-window Gram rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 REPS=2 TAG=ab8m tools/benchab.sh "COCOA_GRAM_SEQ=0 --" "COCOA_LIB=build/v_gw32/libcocoa_hip.so --" " --" || exit $?
