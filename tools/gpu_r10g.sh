#!/bin/bash
# launch-gap A/B on C2: e_w marked before the x.w gather (COCOA_EW_EARLY=1), and
# the bench's HIP events on the solver only (their own cost in the timed region)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r10g}
STEPS=100 REPS=3 TAG=ab_${T} tools/benchab.sh " --" "COCOA_EW_EARLY=1 --" "-- --stats-kernels solver" \
  "COCOA_EW_EARLY=1 -- --stats-kernels solver" || exit $?
