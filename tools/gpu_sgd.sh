#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error|FAIL" gpurun_out/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
METHODS="mbsgd localsgd" bash tools/gpu_configs.sh
