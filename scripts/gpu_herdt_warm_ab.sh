#!/bin/bash
# Herdt warm start A/B (ZMPC_HERDT_WARM 0 = row N−1 free, 1 = row N−2 free + copy, 2 = copy),
# config 6, Herdt GPU tests under each.
set -u
OUT=gpurun_out/${1:-r3hwarm2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in 3 4; do
  ZMPC_HERDT_WARM=$m timeout -k 10 400 python -u -m pytest tests/test_gpu_herdt.py -m gpu -x -q --timeout 280 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_herdt_w$m.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest_herdt_w$m.log"; [ $rc -ne 0 ] && exit $rc
done
for i in 1 2; do
  for m in 2 3 4; do
    ZMPC_HERDT_WARM=$m timeout -k 10 300 python bench.py --config 6 --steps 2 --warmup 1 --no-cpu-baseline \
      > "$OUT/c6_w${m}_$i.json" 2> "$OUT/c6_w${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c6_w${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], r['kernel_ms'], r['passes_per_solve'], r['max_passes_per_solve'], d.get('com_rmse_vs_ref'))" "$OUT/c6_w${m}_$i.json"
  done
done
