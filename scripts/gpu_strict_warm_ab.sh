#!/bin/bash
# Strict LQ warm start A/B: the previous terminal slot starts free (default) vs kept
# (ZMPC_STRICT_WARM=0); strict GPU tests first, then configs 3 and 4 alternating.
set -u
OUT=gpurun_out/${1:-r3warm}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "strict" > "$OUT/pytest_strict.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_strict.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 1 0; do
    for c in 3 4; do
      ZMPC_STRICT_WARM=$m timeout -k 10 300 python bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline \
        > "$OUT/c${c}_w${m}_$i.json" 2> "$OUT/c${c}_w${m}_$i.err"
      rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c${c}_w${m}_$i.err"; exit $rc; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], r['kernel_ms'], r['passes_per_solve'], r['max_passes_per_solve'])" "$OUT/c${c}_w${m}_$i.json"
    done
  done
done
