#!/bin/bash
# Round 3: sparse correlation in the wide kernel — parity (sparse/FFT/direct/variants), then
# config 5 bench A/B (default sparse vs ZMPC_SPARSE_CORR=0) and config 2.
set -u
OUT=gpurun_out/${1:-r3wide}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "not strict" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for m in 1 0; do
    ZMPC_SPARSE_CORR=$m timeout -k 10 300 python bench.py --config 5 --steps 30 --warmup 3 --no-cpu-baseline \
      > "$OUT/c5_sparse${m}_$i.json" 2> "$OUT/c5_sparse${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c5_sparse${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['roofline']['frac'], d['roofline']['bound'])" "$OUT/c5_sparse${m}_$i.json"
  done
done
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > "$OUT/c2.json" 2> "$OUT/c2.err"
rc=$?; cat "$OUT/c2.json"; exit $rc
