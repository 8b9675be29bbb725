#!/bin/bash
# Round 3: sparse correlation from an LDS change list (default) vs the bit walk
# (ZMPC_SPARSE_CORR=2), config 2, three alternations; rollout tests first.
set -u
OUT=gpurun_out/${1:-r3list}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 280 \
  --timeout-method thread -p no:cacheprovider -k "sparse or variants or full_size_config2 or batch_unconstrained or controller_com or long_walks or fft" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for m in 1 2; do
    ZMPC_SPARSE_CORR=$m timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dense-leg \
      > "$OUT/c2_sc${m}_$i.json" 2> "$OUT/c2_sc${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_sc${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c2_sc${m}_$i.json"
  done
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --config 5 --steps 30 --warmup 3 --no-cpu-baseline --no-dense-leg \
    > "$OUT/c5_$i.json" 2> "$OUT/c5_$i.err"
  rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c5_$i.err"; exit $rc; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c5_$i.json"
done
