#!/bin/bash
# r02: full GPU suite, then gram vs chain bench (C2 cocoa+/mbcd)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error|FAILED" gpurun_out/gpu_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r02g.sh
