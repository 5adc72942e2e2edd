#!/usr/bin/env python3
"""Summarise a tools/benchab.sh run (gpurun_out/TAG_i_rep.json) into one JSON
file: every run's ms/step, kernel averages and the amdsmi clocks / power /
temperature bench.py sampled over the timed region, and per-variant means.
  tools/ab_summary.py TAG OUT "label 1" "label 2" ...   (labels in benchab order)"""
import glob
import json
import os
import re
import sys


def main():
    tag, out, labels = sys.argv[1], sys.argv[2], sys.argv[3:]
    runs = []
    for f in sorted(glob.glob(os.path.join("gpurun_out", f"{tag}_*_*.json"))):
        m = re.search(rf"{re.escape(tag)}_(\d+)_(\d+)\.json$", f)
        lines = [ln for ln in open(f) if ln.strip().startswith("{")]
        if not m or not lines:
            continue
        d = json.loads(lines[-1])
        i, rep = int(m.group(1)), int(m.group(2))
        tel = d.get("gpu_telemetry") or {}
        runs.append({"variant": labels[i - 1] if i <= len(labels) else str(i), "rep": rep,
                     "ms_per_step": d["ms_per_step"], "kernel_ms": d.get("kernel_ms"),
                     "eval_ms": (d.get("roofline_eval") or {}).get("avg_launch_ms"),
                     "value": d["value"], "steps": d["steps"], "warmup": d["warmup"],
                     "gpu_telemetry": {"bdf": tel.get("bdf"), "timed_start": tel.get("timed_start"),
                                       "timed_end": tel.get("timed_end"), "timed_samples": tel.get("timed_samples")}})
    summary = {}
    for r in runs:
        s = summary.setdefault(r["variant"], {"ms_per_step": [], "solver_ms": [], "eval_ms": []})
        s["ms_per_step"].append(r["ms_per_step"])
        s["solver_ms"].append((r["kernel_ms"] or {}).get("solver"))
        s["eval_ms"].append((r["kernel_ms"] or {}).get("eval", r.get("eval_ms")))
    for s in summary.values():
        for k in list(s):
            v = [x for x in s[k] if x is not None]
            s[k + "_mean"] = sum(v) / len(v) if v else None
    json.dump({"tag": tag, "runs": runs, "summary": summary}, open(out, "w"), indent=1)
    for k, s in summary.items():
        ev = s["eval_ms_mean"]
        print(f"{k:40s} ms/step {s['ms_per_step_mean']:.4f}  solver {s['solver_ms_mean']:.4f}  eval "
              + (f"{ev:.4f}" if ev is not None else "-"))


if __name__ == "__main__":
    main()
