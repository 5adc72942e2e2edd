#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 env COCOA_CHAIN=${TESTCHAIN:-v5} python -u -m pytest tests -m gpu -x -q -k "fast or c2" --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_chain.log 2>&1
rc=$?; echo "chain tests rc=$rc"; tail -3 gpurun_out/gpu_tests_chain.log; [ $rc -ne 0 ] && exit $rc
CHAINS="${CHAINS:-v3 v5}" bash tools/gpu_chain.sh
