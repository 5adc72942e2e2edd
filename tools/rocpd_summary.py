#!/usr/bin/env python3
"""Kernel summary (name, calls, total/avg/min/max ns, %) from a rocprofv3 rocpd
SQLite output (`rocprofv3 --kernel-trace --stats -d DIR -o run`), as CSV.

usage: python3 tools/rocpd_summary.py DIR_OR_DB [out.csv]
"""
import csv
import glob
import os
import sqlite3
import sys


def main():
    src = sys.argv[1]
    dbs = [src] if src.endswith(".db") else sorted(glob.glob(os.path.join(src, "**", "*.db"), recursive=True))
    rows = {}
    for db in dbs:
        c = sqlite3.connect(db)
        for name, dur in c.execute("select name, duration from kernels"):
            rows.setdefault(name, []).append(float(dur))
    tot = sum(sum(v) for v in rows.values()) or 1.0
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), f"{sum(v):.0f}", f"{sum(v) / len(v):.1f}", f"{min(v):.0f}", f"{max(v):.0f}",
                    f"{100 * sum(v) / tot:.2f}"])


if __name__ == "__main__":
    main()
