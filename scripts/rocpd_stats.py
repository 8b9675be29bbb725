#!/usr/bin/env python3
"""Kernel statistics (calls, total/avg/min/max ns) from a rocprofv3 rocpd SQLite output, written
as the CSV layout of `rocprofv3 --stats` (kernel_stats.csv).  Usage:
  python scripts/rocpd_stats.py run_results.db out.csv"""
import csv
import sqlite3
import sys


def main(db, out):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = list(c.execute(f"select {name}, start, end from kernels"))
    agg = {}
    for k, s, e in rows:
        agg.setdefault(k, []).append(e - s)
    tot = sum(sum(v) for v in agg.values()) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs",
                    "MaxNs"])
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
