"""Mean of every rocprofv3 counter over the dispatches of kernels whose name contains a
substring: python scripts/pmc_summary.py <dir> <kernel-substring>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
names = set()
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if sub in r["Kernel_Name"]:
                names.add(r["Kernel_Name"][:90])
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
out["_kernels"] = sorted(names)
out["_dispatches"] = max((len(v) for v in vals.values()), default=0)
print(json.dumps(out, indent=1))
