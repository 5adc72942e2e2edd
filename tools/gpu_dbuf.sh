#!/bin/bash
# GPU tests, then the C4 line with double-buffered deltaW slices (default for
# C4) against single-buffered (COCOA_DW_DBUF=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_dbuf.log 2>&1 || { tail -30 gpurun_out/gpu_tests_dbuf.log; exit 1; }
tail -1 gpurun_out/gpu_tests_dbuf.log
B="python3 -u bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-gap"
timeout -k 10 400 $B > gpurun_out/c4_dbuf.json 2> gpurun_out/c4_dbuf.err || exit $?
for zb in 32 128 0; do timeout -k 10 400 env COCOA_ZERO_WGS=$zb $B > gpurun_out/c4_z$zb.json 2> gpurun_out/c4_z$zb.err || exit $?; done
python3 - <<'PY'
import json
for f in ["dbuf", "z32", "z128", "z0"]:
    j = json.loads(open(f"gpurun_out/c4_{f}.json").read().strip().splitlines()[-1])
    print(f, "ms/round %.3f" % j["ms_per_step"], "value %.4g" % j["value"], j["kernel_ms"])
PY
