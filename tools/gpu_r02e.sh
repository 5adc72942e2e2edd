#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py -q --timeout 120 --timeout-method thread > gpurun_out/gpu_gram.log 2>&1
echo "default rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/gpu_gram.log | tail -12
COCOA_LIB=build/drain/libcocoa_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py -q --timeout 120 --timeout-method thread > gpurun_out/gpu_gram_drain.log 2>&1
echo "drain rc=$?"; grep -E "FAILED|passed|failed" gpurun_out/gpu_gram_drain.log | tail -12
