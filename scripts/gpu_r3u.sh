#!/bin/bash
# Round 3: strict LQ drift A/B (ZMPC_STRICT_LQ_DRIFT: timesteps a lane may run ahead of its
# wave's slowest lane), config 3 (alternating) and config 4 strict.
set -u
OUT=gpurun_out/r3u
mkdir -p "$OUT"
export TMPDIR=/tmp
for R in 1 2 3; do
for D in 2 3 4; do
  ZMPC_STRICT_LQ_DRIFT=$D timeout -k 10 300 python scripts/strict_axis_diag.py 65536 0 > "$OUT/c3_drift_${D}_$R.jsonl" 2>&1 || exit $?
  echo "c3 drift $D: $(cut -c1-70 $OUT/c3_drift_${D}_$R.jsonl)"
done
done
for D in 2 4; do
  ZMPC_STRICT_LQ_DRIFT=$D timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/c4_drift_$D.json" 2> "$OUT/c4_drift_$D.err" || exit $?
  python -c "import json; d=json.load(open('$OUT/c4_drift_$D.json')); print('c4 drift $D', '%.3e' % d['value'], d['ms_per_step'])"
done
