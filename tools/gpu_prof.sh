#!/bin/bash
# Solver diagnostics + rocprofv3 kernel stats of the bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u tools/prof_solver.py > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err || exit $?
timeout -k 10 180 env COCOA_LIB=build/diag/libcocoa_hip.so python -u tools/prof_solver.py > gpurun_out/prof_diag.json 2> gpurun_out/prof_diag.err || exit $?
timeout -k 10 180 env COCOA_LIB=build/diag/libcocoa_hip.so python -u tools/prof_solver.py --strict > gpurun_out/prof_diag_strict.json 2>> gpurun_out/prof_diag.err || exit $?
cat gpurun_out/prof_default.json gpurun_out/prof_diag.json gpurun_out/prof_diag_strict.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-gap > gpurun_out/rocprof_bench.log 2>&1 || exit $?
find gpurun_out/rocprof -name "*stats*" | head
