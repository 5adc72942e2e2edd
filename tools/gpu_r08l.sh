#!/bin/bash
# what the mirrored solver's memory waves cost: diag build with the scatter
# atomics (1), the base gathers (2) or both (3) skipped (timing only, results invalid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 REPS=2 TAG=ab8l tools/benchab.sh "COCOA_LIB=build/diag/libcocoa_hip.so -- --no-gap" \
  "COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_DIAG=1 --" "COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_DIAG=2 --" \
  "COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_DIAG=3 --" "COCOA_LIB=build/diag/libcocoa_hip.so COCOA_GRAM_SERIAL=1 --" || exit $?
