#!/bin/bash
# Strict A/B: parity tests, then config-3-shaped timing per variant env.
set -u
OUT=gpurun_out/${1:-sab}
B=${2:-16384}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "strict or plan" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for V in default ZMPC_STRICT_LDS_G ZMPC_STRICT_LDS_CHOL; do
  if [ $V = default ]; then E=""; else E="$V=1"; fi
  env $E timeout -k 10 300 python bench.py --config 3 --batch $B --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/$V.json" 2> "$OUT/$V.err" || { tail -5 "$OUT/$V.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$V.json')); print('$V', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
