#!/bin/bash
# C2 headline with the register-chunk count of the CoCoA+ chain at 4 (shipped), 3 and 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-gap"
timeout -k 10 300 env COCOA_LIB=build/rc2/libcocoa_hip.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rc2_tests.log 2>&1 || { tail -20 gpurun_out/rc2_tests.log; exit 1; }
tail -1 gpurun_out/rc2_tests.log
timeout -k 10 300 $B > gpurun_out/rc4.json 2> gpurun_out/rc4.err || exit $?
timeout -k 10 300 env COCOA_LIB=build/rc3/libcocoa_hip.so $B > gpurun_out/rc3.json 2> gpurun_out/rc3.err || exit $?
timeout -k 10 300 env COCOA_LIB=build/rc2/libcocoa_hip.so $B > gpurun_out/rc2.json 2> gpurun_out/rc2.err || exit $?
python3 - <<'PY'
import json
for f in ["rc4", "rc3", "rc2"]:
    j = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, "ms/round %.3f" % j["ms_per_step"], "solver %.3f" % j["kernel_ms"]["solver"])
PY
