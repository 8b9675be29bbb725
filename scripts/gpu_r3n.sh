#!/bin/bash
# Round 3: chunk-sum local scan (plan columns Ā^p B) — rollout parity tests, config-2 A/B.
set -u
OUT=gpurun_out/r3n
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not strict and not herdt" > "$OUT/pytest_rollout.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_rollout.log"; [ $rc -ne 0 ] && exit $rc
for R in 1 2 3; do
for V in 8 17; do
  ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/c2_v${V}_$R.json" 2> "$OUT/c2_v${V}_$R.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c2_v${V}_$R.json')); r=d['roofline']; print('c2 v $V', '%.3e' % d['value'], '%.2f us' % (r['kernel_ms']*1e3), '%.3f' % r['frac'], d.get('com_rmse_vs_ref'))"
done
done
timeout -k 10 600 python scripts/ablate_rollout.py 8 0,12,13 4096 > "$OUT/ablation.jsonl" 2>&1 || exit $?
cat "$OUT/ablation.jsonl"
