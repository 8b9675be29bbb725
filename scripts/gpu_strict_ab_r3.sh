#!/bin/bash
# Strict LQ kernel A/B (config 3, B = 65536): variants SxWxG and the window-traffic diagnostic.
set -u
OUT=gpurun_out/${1:-r3s}
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in 8x2x8 4x3x4 8x2x4; do
  for D in 0 1; do
    ZMPC_STRICT_LQ=$V ZMPC_DEBUG_LQ=$D timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c3_${V}_d$D.json" 2> "$OUT/c3_${V}_d$D.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c3_${V}_d$D.err"; exit $rc; }
    python -c "import json; d=json.load(open('$OUT/c3_${V}_d$D.json')); r=d['roofline']; print('$V dbg $D', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], 'passes %.3f' % r['passes_per_solve'])"
  done
done
exit 0
