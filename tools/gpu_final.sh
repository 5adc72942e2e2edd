#!/bin/bash
# round 6, final tree.  PART=1: GPU tests, smoke, the headline bench, rocprof,
# PMC.  PART=2: the four-way A/B with clocks (mirror / gram_seq on and off) and
# the config lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-fin}
if [ "${PART:-1}" = 1 ]; then
  TAG=$T tools/gpu_run.sh tests smoke bench prof pmc || exit $?
else
  STEPS=100 REPS=3 TAG=abfin_$T tools/benchab.sh " --" "COCOA_GRAM_MIRROR=0 --" "COCOA_GRAM_SEQ=0 --" \
    "COCOA_GRAM_MIRROR=0 COCOA_GRAM_SEQ=0 --" || exit $?
  python3 tools/ab_summary.py abfin_$T gpurun_out/ab_final_tree_$T.json "as shipped" "COCOA_GRAM_MIRROR=0" \
    "COCOA_GRAM_SEQ=0" "COCOA_GRAM_MIRROR=0 COCOA_GRAM_SEQ=0" || exit $?
  TAG=$T tools/gpu_run.sh lines || exit $?
fi
