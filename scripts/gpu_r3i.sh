#!/bin/bash
# Round 3: config-2 rollout variants A/B (8 default persistent split, 9/10 independent axes).
set -u
OUT=gpurun_out/r3i
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "variants_agree or full_size_config2 or controller_com" --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for B in 4096 8192; do
  for V in 8 13 14; do
    ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --batch $B --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_b${B}_v$V.json" 2> "$OUT/c2_b${B}_v$V.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_b${B}_v$V.err"; exit $rc; }
    python -c "import json; d=json.load(open('$OUT/c2_b${B}_v$V.json')); r=d['roofline']; print('B $B v $V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'])"
  done
done
exit 0
