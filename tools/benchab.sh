#!/bin/bash
# Same-box A/B of bench.py settings, interleaved, REPS rounds (default 2):
#   tools/benchab.sh "ENV=1 -- --flag" "ENV=0 --" ...   (env assignments, "--", bench flags)
# Each line prints ms/step, the kernels' HIP-event averages and the gfx clock /
# power the bench's amdsmi sampler saw over the timed region.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out
mkdir -p $O
STEPS=${STEPS:-20}
TAG=${TAG:-ab}
for rep in $(seq 1 ${REPS:-2}); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    envs="${v%%--*}"; flags="${v#*--}"
    env X=0 $envs timeout -k 10 300 python3 bench.py --steps $STEPS --warmup 3 --no-cpu-baseline --no-gap $flags \
      > $O/${TAG}_${i}_${rep}.json 2> $O/${TAG}_${i}_${rep}.err || exit $?
    python3 - "$O/${TAG}_${i}_${rep}.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).readlines()[-1])
tel = (d.get("gpu_telemetry") or {}).get("timed_samples") or {}
g = lambda k: round(tel[k]["mean"]) if k in tel else None
print(f"[{sys.argv[2]}]", round(d["ms_per_step"], 4), {k: round(x, 4) for k, x in d["kernel_ms"].items()},
      "sclk", g("sclk_mhz"), "avg_gfx", g("avg_gfxclk_mhz"), "mclk", g("mclk_mhz"), "fclk", g("fclk_mhz"),
      "W", g("power_w"), "T", g("temp_hotspot_c"), flush=True)
PY
  done
done
