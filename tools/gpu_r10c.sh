#!/bin/bash
# test rows split into the hot / cold passes: GPU tests, same-box A/B against
# COCOA_EVAL_TEST_SPLIT=0 (C2, C4), then the final-tree rocprof of the bench window
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r10c}
TAG=$T TESTS="tests/test_gpu_eval_split.py tests/test_gpu_parity.py tests/test_gpu_configs.py" tools/gpu_run.sh tests || exit $?
STEPS=100 REPS=3 TAG=ab_${T} tools/benchab.sh " --" "COCOA_EVAL_TEST_SPLIT=0 --" || exit $?
STEPS=10 REPS=2 TAG=ab_${T}c4 tools/benchab.sh "-- --config c4" "COCOA_EVAL_TEST_SPLIT=0 -- --config c4" || exit $?
TAG=$T tools/gpu_run.sh prof || exit $?
