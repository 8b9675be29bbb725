#!/bin/bash
# Strict LQ kernel variants at config-3 size: parity, timing per variant, pass counters.
# Usage: bash scripts/gpu_strict_lq2.sh <tag> [B] [variants...]
set -u
OUT=gpurun_out/${1:-slq}
B=${2:-65536}
shift 2 || true
VARS=${@:-8x1 4x2 8x2}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "strict" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for V in $VARS; do
  if [ $V = chol ]; then E="ZMPC_STRICT_VARIANT=chol"; else E="ZMPC_STRICT_LQ=$V"; fi
  env $E timeout -k 10 300 python bench.py --config 3 --batch $B --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err"
  rc=$?; if [ $rc -ne 0 ]; then tail -5 "$OUT/$V.err"; exit $rc; fi
  python -c "import json; d=json.load(open('$OUT/$V.json')); print('$V', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
  env $E ZMPC_DEBUG_STRICT=1 timeout -k 10 300 python scripts/strict_once.py $B > "$OUT/dbg_$V.log" 2>&1
  rc=$?; grep "dbg" "$OUT/dbg_$V.log" | tail -1; [ $rc -ne 0 ] && exit $rc
done
exit 0
