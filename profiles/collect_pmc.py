#!/usr/bin/env python3
"""Turn rocprofv3 runs of bench.py into the committed profile summaries.

Inputs (written by scripts/gpu_profile_round.sh on the GPU box):
  <dir>/stats/*kernel_stats.csv        rocprofv3 --kernel-trace --stats --output-format csv
  <dir>/fetch/*counter_collection.csv  rocprofv3 --kernel-trace --pmc FETCH_SIZE  (own pass)
  <dir>/write/*counter_collection.csv  rocprofv3 --kernel-trace --pmc WRITE_SIZE  (own pass)

Outputs:
  profiles/pmc_<workload>.json  {"kernel", "dispatches", "fetch_kb", "write_kb",
                                 "hbm_bytes_per_launch", ...} — read by bench.py for
                                 roofline.traffic
HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half of the
bytes of a 16-B/lane coalesced streaming read on gfx950, so it is doubled (the rollout's bound
loads are exactly that pattern); WRITE_SIZE (KB) is exact for 16-B/lane streaming stores.

Usage: python profiles/collect_pmc.py <dir> <workload> <kernel-substring>
"""
import csv
import glob
import json
import os
import sys


def _rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def counter_mean(d, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in
            _rows(os.path.join(d, "**", "*counter_collection.csv"))
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    d, workload, kernel = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, nf = counter_mean(os.path.join(d, "fetch"), "FETCH_SIZE", kernel)
    write, nw = counter_mean(os.path.join(d, "write"), "WRITE_SIZE", kernel)
    out = {"kernel": kernel, "workload": workload, "dispatches": [nf, nw],
           "fetch_kb": fetch, "write_kb": write, "hbm_bytes_per_launch": None,
           "correction": "2*FETCH_SIZE (gfx950 16-B/lane read halving) + WRITE_SIZE, KB=1024 B"}
    if fetch is not None and write is not None:
        out["hbm_bytes_per_launch"] = 2 * fetch * 1024 + write * 1024
    stats = _rows(os.path.join(d, "stats", "**", "*kernel_stats.csv"))
    for r in stats:
        if kernel in r.get("Name", ""):
            out["rocprof_avg_ns"] = float(r["AverageNs"])
            out["rocprof_calls"] = int(r["Calls"])
    root = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(root, f"pmc_{workload}.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
