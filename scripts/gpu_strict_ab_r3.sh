#!/bin/bash
# Strict LQ kernel A/B (config 3, B = 65536): variants SxWxG[p] and the window-traffic
# diagnostic; the prefetch variant's parity first (strict GPU tests with it forced).
set -u
OUT=gpurun_out/${1:-r3s}
mkdir -p "$OUT"
export TMPDIR=/tmp
ZMPC_STRICT_LQ=8x2x8p timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "strict" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_pk.log" 2>&1
rc=$?; echo "pytest pk rc=$rc"; tail -3 "$OUT/pytest_pk.log"; [ $rc -ne 0 ] && exit $rc
for V in 8x2x8 8x2x8p 4x3x4; do
  for D in 0 1; do
    [ "$V" = "4x3x4" ] && [ $D = 1 ] && continue
    ZMPC_STRICT_LQ=$V ZMPC_DEBUG_LQ=$D timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_${V}_d$D.json" 2> "$OUT/c3_${V}_d$D.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c3_${V}_d$D.err"; exit $rc; }
    python -c "import json; d=json.load(open('$OUT/c3_${V}_d$D.json')); r=d['roofline']; print('$V dbg $D', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], 'passes %.3f' % r['passes_per_solve'])"
  done
done
for V in 8x2x8 8x2x8p; do
  ZMPC_STRICT_LQ=$V timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c4_${V}.json" 2> "$OUT/c4_${V}.err"
  rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c4_${V}.err"; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/c4_${V}.json')); r=d['roofline']; print('c4 $V', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'])"
done
exit 0
