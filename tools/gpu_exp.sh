#!/bin/bash
# GPU tests, eval kernel A/B/C, solver floor with deltaW in LDS (small d).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests.log | tail -5; [ $rc -ne 0 ] && exit $rc
for v in v1 v2 v3; do
  timeout -k 10 200 env COCOA_EVAL=$v $B > gpurun_out/bench_eval_$v.json 2> gpurun_out/bench_eval_$v.err || exit $?
done
timeout -k 10 200 $B --d 8192 > gpurun_out/bench_d8192.json 2> gpurun_out/bench_d8192.err || exit $?
timeout -k 10 200 $B --d 8192 --parts 256 > gpurun_out/bench_d8192_k256.json 2> gpurun_out/bench_d8192_k256.err || exit $?
python3 - <<'PY'
import json
for f in ["bench_eval_v1", "bench_eval_v2", "bench_eval_v3", "bench_d8192", "bench_d8192_k256"]:
    j = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    H = j["config"]["H"]
    print(f, "eval ms %.4f frac %.3f" % (j["kernel_ms"]["eval"], j["roofline_eval"]["frac"]),
          "solver ms %.3f cyc/step@2.4GHz %.0f" % (j["kernel_ms"]["solver"], j["kernel_ms"]["solver"] * 2.4e6 / H),
          "plan", j.get("plan", {}).get("vec_lds"), "value %.3g" % j["value"])
PY
