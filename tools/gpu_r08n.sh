#!/bin/bash
# the pipelined flow (evaluation beside the next round) on the round-6 tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=50 REPS=2 TAG=ab8n tools/benchab.sh " --" "-- --pipeline" "COCOA_GRAM_CHUNKS=3 -- --pipeline" || exit $?
