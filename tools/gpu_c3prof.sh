#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="--kind epsilon --n 400000 --d 2000 --nnz 2000 --parts 64 --rounds 2"
timeout -k 10 300 python -u tools/prof_solver.py $A > gpurun_out/c3_prof.json 2> gpurun_out/c3_prof.err || exit $?
cp gpurun_out/c3_prof.json gpurun_out/c3_prof_diag.json
python3 - <<'PY'
import json
for f in ("gpurun_out/c3_prof.json", "gpurun_out/c3_prof_diag.json"):
    j = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, j["plan"])
    for r in j["records"]:
        print(" t", r["t"], "ms %.2f" % r["solver_ms_total"], "cyc/step %.0f" % r["cyc_per_step_total"], "chain busy/wait %.0f %.0f" % (r["compute_busy_cyc_mean"], r["compute_wait_cyc_mean"]),
              "loader busy/wait %.0f %.0f" % (r["loader_busy_cyc_mean"], r["loader_wait_cyc_mean"]), "batches %.0f" % r["batches_mean"], "phases", [round(x) for x in r["step_phase_cyc_per_step"]])
PY
