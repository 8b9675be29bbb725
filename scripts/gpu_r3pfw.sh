#!/bin/bash
# Round 3: wide-kernel next-round prefetch A/B (config 5: B = 2048 is ~2.7 rounds; ZMPC_PF_ROUNDS
# 3 turns it on, 2 = default leaves it off there), rollout tests first.
set -u
OUT=gpurun_out/${1:-r3pfw}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "not strict" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for m in 3 2; do
    ZMPC_PF_ROUNDS=$m timeout -k 10 300 python bench.py --config 5 --steps 30 --warmup 3 --no-cpu-baseline --no-dense-leg \
      > "$OUT/c5_pfr${m}_$i.json" 2> "$OUT/c5_pfr${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c5_pfr${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c5_pfr${m}_$i.json"
  done
done
