#!/bin/bash
# v2 solver bring-up: parity tests, then the solver diagnostics, then a short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error|Error" gpurun_out/gpu_tests.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 python -u tools/prof_solver.py > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err || exit $?
timeout -k 10 180 env COCOA_LIB=build/diag/libcocoa_hip.so python -u tools/prof_solver.py > gpurun_out/prof_diag.json 2> gpurun_out/prof_diag.err || exit $?
cat gpurun_out/prof_default.json gpurun_out/prof_diag.json
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; tail -c 2500 gpurun_out/bench.log
