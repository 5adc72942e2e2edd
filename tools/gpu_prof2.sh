#!/bin/bash
# solver diagnostics: default, serialized loader, diag (phase stamps) x {overlap, serial}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { timeout -k 10 180 env "$@" python -u tools/prof_solver.py --rounds 2 ${PROF_ARGS}; }
{ run X=1 && run COCOA_DBG_SERIAL=1 && run COCOA_LIB=build/diag/libcocoa_hip.so && run COCOA_LIB=build/diag/libcocoa_hip.so COCOA_DBG_SERIAL=1; } > gpurun_out/prof2.jsonl 2> gpurun_out/prof2.err
rc=$?; echo "prof rc=$rc"; tail -2 gpurun_out/prof2.err
