#!/bin/bash
# Strict LQ variant A/B at config 3 (bench line + FETCH/WRITE PMC per variant).
# Usage: bash scripts/gpu_strict_ab2.sh <tag> <variant>...   outputs under gpurun_out/<tag>/
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in "$@"; do
  env ZMPC_STRICT_LQ=$V timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/$V.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/$V.json')); r=d['roofline']; print('$V', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], 'pps %.3f' % r['passes_per_solve'], 'lane_eff %.3f' % r['lane_efficiency'])"
  ZMPC_STRICT_LQ=$V timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/f_$V" -o b -- python3 bench.py --config 3 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> "$OUT/f_$V.err"
  rc=$?; [ $rc -ne 0 ] && exit $rc
  python3 - "$OUT/f_$V" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/*counter_collection.csv")
     for r in csv.DictReader(open(f)) if "strict_lq_kernel" in r["Kernel_Name"]]
print("  FETCH_SIZE GB/launch (x2 corrected):", 2 * sum(v) / len(v) * 1024 / 1e9)
PY
done
