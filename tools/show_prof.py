import json, sys
for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof2.jsonl"):
    d = json.loads(line)
    for r in d["records"]:
        print(d.get("tag", ""), d["lib"][-20:], "t=%d" % r["t"], "cyc/step=%d" % r["cyc_per_step_total"],
              "busy=%d" % r["cyc_per_step_compute"], "loader busy/wait=%.1f/%.1fM" % (r["loader_busy_cyc_mean"] / 1e6, r["loader_wait_cyc_mean"] / 1e6),
              "phases", [round(x) for x in r["step_phase_cyc_per_step"]], "ms=%.2f" % r["solver_ms_total"])
