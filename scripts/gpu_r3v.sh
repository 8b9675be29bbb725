#!/bin/bash
# Round 3: Herdt slab with non-temporal stores/loads (ZMPC_HERDT_SLAB_NT) A/B, config 6.
set -u
OUT=gpurun_out/r3v
mkdir -p "$OUT"
export TMPDIR=/tmp
ZMPC_HERDT_SLAB_NT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_herdt.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_nt.log" 2>&1
rc=$?; echo "pytest(nt) rc=$rc"; tail -2 "$OUT/pytest_nt.log"; [ $rc -ne 0 ] && exit $rc
for R in 1 2; do
for V in 0 1; do
  ZMPC_HERDT_SLAB_NT=$V timeout -k 10 300 python bench.py --config 6 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/c6_nt${V}_$R.json" 2> "$OUT/c6_nt${V}_$R.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c6_nt${V}_$R.json')); r=d['roofline']; print('c6 nt $V', '%.3e' % d['value'], '%.2f ms' % r['kernel_ms'], r.get('max_passes_per_solve'))"
done
done
