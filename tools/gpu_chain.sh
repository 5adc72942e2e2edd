#!/bin/bash
# Solver chain A/B: per-wave busy/wait and solver ms for chain variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CHAINS:-v3 v4diag}; do
  timeout -k 10 180 env COCOA_CHAIN=$c python -u tools/prof_solver.py > gpurun_out/chain_$c.json 2> gpurun_out/chain_$c.err || exit $?
  python3 - "$c" <<'PY'
import json, sys
j = json.loads(open(f"gpurun_out/chain_{sys.argv[1]}.json").read().strip().splitlines()[-1])
for r in j["records"]:
    print(sys.argv[1], "t", r["t"], "solver ms %.3f" % r["solver_ms_total"], "cyc/step %.0f" % r["cyc_per_step_total"],
          "chain busy %.0f wait %.0f" % (r["compute_busy_cyc_mean"], r["compute_wait_cyc_mean"]),
          "loader busy %.0f wait %.0f" % (r["loader_busy_cyc_mean"], r["loader_wait_cyc_mean"]))
PY
done
