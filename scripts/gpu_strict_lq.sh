#!/bin/bash
# Strict LQ kernel: parity tests, then config-3-shaped timing per kernel variant
# (ZMPC_STRICT_VARIANT=chol = the reduced-Cholesky kernel; ZMPC_STRICT_LQ=SxW).
# Usage: bash scripts/gpu_strict_lq.sh <tag> [B]
set -u
OUT=gpurun_out/${1:-slq}
B=${2:-16384}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "strict" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for V in 8x1 4x2 8x2 4x1 chol; do
  if [ $V = chol ]; then E="ZMPC_STRICT_VARIANT=chol"; else E="ZMPC_STRICT_LQ=$V"; fi
  env $E timeout -k 10 300 python bench.py --config 3 --batch $B --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/$V.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/$V.json')); print('$V', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
env ZMPC_DEBUG_STRICT=1 timeout -k 10 300 python scripts/strict_once.py $B > "$OUT/dbg.log" 2>&1
rc=$?; grep "dbg" "$OUT/dbg.log" | tail -3; exit $rc
