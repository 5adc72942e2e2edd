"""Print the rocprofv3 --stats kernel summary (run_kernel_stats.csv) under a directory."""
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
