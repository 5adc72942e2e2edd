#!/bin/bash
# Eval v4 variants (16-byte tile loads) against eval v1 on the C2 bench workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
timeout -k 10 200 env COCOA_EVAL=v1 $B > gpurun_out/e4_v1.json 2> gpurun_out/e4_v1.err || exit $?
for v in 0 1 2 3; do
  timeout -k 10 200 env COCOA_EVAL=v6 COCOA_EVAL6=$v $B > gpurun_out/e4_$v.json 2> gpurun_out/e4_$v.err || exit $?
done
python3 - <<'PY'
import json
for f in ["v1", "0", "1", "2", "3"]:
    j = json.loads(open(f"gpurun_out/e4_{f}.json").read().strip().splitlines()[-1])
    print(f, "eval ms %.4f" % j["kernel_ms"]["eval"], "frac %.3f" % j["roofline_eval"]["frac"], "gaps", ["%.15g" % g for g in j["gap_trajectory_timed"][:3]])
PY
