#!/bin/bash
# Round 3: next-round bound prefetch A/B (config 2, default vs ZMPC_PREFETCH=0), three
# alternations, plus the batch sweep with it.
set -u
OUT=gpurun_out/${1:-r3pf}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 \
  --timeout-method thread -p no:cacheprovider -k "sparse or variants or multi_walk or full_size_config2 or batch_unconstrained" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for m in 1 0; do
    ZMPC_PREFETCH=$m timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline \
      > "$OUT/c2_pf${m}_$i.json" 2> "$OUT/c2_pf${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_pf${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['ms_per_step']*1e3, d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c2_pf${m}_$i.json"
  done
done
ABL_DATA=cop timeout -k 10 300 python scripts/ablate_rollout.py 8 0 2048,4096,6144,8192,16384 > "$OUT/batch_cop.jsonl" 2> "$OUT/abl.err"
rc=$?; cat "$OUT/batch_cop.jsonl"; exit $rc
