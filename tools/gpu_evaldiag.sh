#!/bin/bash
# Eval v4 gather diagnostics on C2: 3 = shipped, 7 = 16 KB window of w,
# 11 = every lane reads w[0] (col stream kept), 6 = no gather (col load dead).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
for v in 3 17 18 3 17 18; do
  timeout -k 10 200 env COCOA_EVAL4=$v $B > gpurun_out/ed_$v.json 2> gpurun_out/ed_$v.err || exit $?
done
python3 - <<'PY'
import json
for f in ["3", "17", "18"]:
    j = json.loads(open(f"gpurun_out/ed_{f}.json").read().strip().splitlines()[-1])
    print(f, "eval ms %.4f" % j["kernel_ms"]["eval"], "frac %.3f" % j["roofline_eval"]["frac"])
PY
