#!/usr/bin/env python3
"""Per-kernel averages of the counters in gpurun_out/spmc_*_TAG (tools/gpu_run.sh solverpmc)."""
import collections
import csv
import glob
import os
import sys

src, tag = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for d in sorted(glob.glob(os.path.join(src, "spmc_*_" + tag))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            short = ("solver_gram" if "solver_gram" in name else "gram" if "gram_kernel" in name else
                     "eval" if "eval_stream" in name else "plan" if "plan_kernel" in name else None)
            if short:
                agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print("%-12s %-24s %16.1f  (n=%d)" % (k, c, sum(v) / len(v), len(v)))
