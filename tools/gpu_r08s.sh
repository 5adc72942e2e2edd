#!/bin/bash
# how the mirrored solver scales with the memory waves' units per batch (diag bit 4: half of them; timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 REPS=2 TAG=ab8s tools/benchab.sh "COCOA_LIB=build/diag/libcocoa_hip.so -- --no-gap" \
  "COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_DIAG=4 --" || exit $?
