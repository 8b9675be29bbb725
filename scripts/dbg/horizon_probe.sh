#!/bin/bash
# Unconstrained horizon probe around the sweep's dip: kernel names and times at N = 150..190.
set -u
OUT=gpurun_out/${1:-r4hp}
mkdir -p "$OUT"
export TMPDIR=/tmp
for N in 150 160 170 180 190; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n$N" -o run -- python3 bench.py --horizon $N --steps 20 --warmup 3 --no-cpu-baseline --no-dense-leg > "$OUT/n$N.json" 2> "$OUT/n$N.err" || exit $?
  python3 - "$OUT/n$N" "$N" <<'PY'
import csv, glob, sys
rows = [r for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(f))]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print(sys.argv[2], [(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows[:3]])
PY
done
