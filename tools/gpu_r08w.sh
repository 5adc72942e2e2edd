#!/bin/bash
# kernel stats: 8 runs vs 4 runs (rocprofv3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r08w8 tools/gpu_run.sh prof || exit $?
COCOA_LIB=build/v_runs4/libcocoa_hip.so TAG=r08w4 tools/gpu_run.sh prof || exit $?
