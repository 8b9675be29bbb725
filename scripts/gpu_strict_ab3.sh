#!/bin/bash
# Strict LQ: GPU strict parity tests on the default variant, then config-3 bench per variant.
# Usage: bash scripts/gpu_strict_ab3.sh <tag> <variant>...   outputs under gpurun_out/<tag>/
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k strict -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/pytest_strict.log" 2>&1
rc=$?; echo "pytest strict rc=$rc"; tail -3 "$OUT/pytest_strict.log"; [ $rc -ne 0 ] && exit $rc
for V in "$@"; do
  env ZMPC_STRICT_LQ=$V timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/$V.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/$V.json')); r=d['roofline']; print('$V', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], 'pps %.3f' % r['passes_per_solve'], 'lane_eff %.3f' % r['lane_efficiency'])"
done
