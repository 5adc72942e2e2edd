#!/bin/bash
# the side stream's Gram rows gated on the last evaluation's e_inl (COCOA_GATE_INL=1)
# instead of an e_w record behind the x.w gather: C2 tests with it on, same-box A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r10j}
COCOA_GATE_INL=1 TAG=$T TESTS="tests/test_gpu_configs.py tests/test_gpu_mirror.py tests/test_gpu_eval_split.py" \
  tools/gpu_run.sh tests || exit $?
STEPS=100 REPS=3 TAG=ab_${T} tools/benchab.sh " --" "COCOA_GATE_INL=1 --" || exit $?
