#!/bin/bash
# look-back from the plan: Gram/mirror/gram_seq/config tests, the loader profile,
# then an A/B of mirror on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_mirror.py tests/test_gpu_gram_seq.py \
  tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests_r08d.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/gpu_tests_r08d.log | tail -3; [ $rc -eq 0 ] || exit $rc
MIRRORS="1 0" TAG=r08d tools/gpu_r08c.sh || exit $?
STEPS=100 REPS=2 TAG=ab8d tools/benchab.sh " --" "COCOA_GRAM_MIRROR=0 --" || exit $?
