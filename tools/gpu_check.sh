#!/bin/bash
# One GPU session: smoke, GPU parity tests, a short bench.  Stops at the first
# timeout / abort / segfault (exit 124, 134, 137, 139) so no GPU step follows a hang.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
fatal $rc && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -v --maxfail=8 --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -5
fatal $rc && exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > gpurun_out/bench.log 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.err; tail -c 3000 gpurun_out/bench.log
fi
