#!/bin/bash
# Round 3: sparse-difference correlation — rollout parity tests, then config-2 A/B
# (default sparse vs ZMPC_SPARSE_CORR=0 dense), three alternations on one box.
set -u
OUT=gpurun_out/${1:-r3sp}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 \
  --timeout-method thread -p no:cacheprovider -k "not strict" > "$OUT/pytest_rollout.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_rollout.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for m in 1 0; do
    ZMPC_SPARSE_CORR=$m timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline \
      > "$OUT/c2_sparse${m}_$i.json" 2> "$OUT/c2_sparse${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_sparse${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['roofline']['frac'], d.get('com_rmse_vs_ref'))" "$OUT/c2_sparse${m}_$i.json"
  done
done
