#!/bin/bash
# GPU tests (chain v3 default), then chain v1 vs v3 on C2 and on d=8192 (deltaW in LDS).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-gap"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error|Error|assert" gpurun_out/gpu_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
for c in v1 v3; do
  timeout -k 10 200 env COCOA_CHAIN=$c $B > gpurun_out/bench_chain_$c.json 2> gpurun_out/bench_chain_$c.err || exit $?
  timeout -k 10 200 env COCOA_CHAIN=$c $B --d 8192 > gpurun_out/bench_chain_${c}_d8192.json 2> gpurun_out/bench_chain_${c}_d8192.err || exit $?
done
timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_gap.json 2> gpurun_out/bench_gap.err || exit $?
python3 - <<'PY'
import json
for f in ["bench_chain_v1", "bench_chain_v3", "bench_chain_v1_d8192", "bench_chain_v3_d8192", "bench_gap"]:
    j = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    H = j["config"]["H"]
    print(f, "solver ms %.3f cyc/step@2.4GHz %.0f" % (j["kernel_ms"]["solver"], j["kernel_ms"]["solver"] * 2.4e6 / H),
          "value %.3g" % j["value"], "ttg", j.get("time_to_gap_s"), j.get("rounds_to_gap"), "gaps", ["%.3e" % g for g in j["gap_trajectory_timed"]])
PY
