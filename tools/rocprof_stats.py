"""Print the rocprofv3 --stats kernel summary (run_kernel_stats.csv) under a directory.

    python3 tools/rocprof_stats.py DIR [SKIP]

With SKIP, also print each kernel's average over its launches after the first
SKIP (from run_kernel_trace.csv): `bench.py --warmup W` profiled with SKIP = W
gives the timed window's average, the figure bench.py's HIP events report.
"""
import collections
import csv
import glob
import sys

for f in sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)):
    print(f)
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: -float(r.get("TotalDurationNs", 0)))
    for r in rows[:16]:
        print("%-60s calls=%6s avg_ms=%.4f total_ms=%.3f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e6,
                                                           float(r["TotalDurationNs"]) / 1e6))
if len(sys.argv) > 2:
    skip = int(sys.argv[2])
    for f in sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)):
        launches = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            launches[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        print(f"{f}: average over launches {skip + 1}.. of each kernel")
        for name, ev in sorted(launches.items(), key=lambda kv: -sum(e - s for s, e in kv[1])):
            ev.sort()
            tail = ev[skip:]
            if tail:
                print("%-60s launches=%4d avg_ms=%.4f" % (name[:60], len(tail), sum(e - s for s, e in tail) / len(tail) / 1e6))
