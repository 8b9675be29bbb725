#!/bin/bash
# Round 3: prefetch issue point A/B (1 early = with the walk's own loads, 2 late = after they
# landed, 0 off), config 2, three alternations; batch sweep at 3 rounds.
set -u
OUT=gpurun_out/${1:-r3pf2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2 3; do
  for m in 1 2 0; do
    ZMPC_PREFETCH=$m timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dense-leg \
      > "$OUT/c2_pf${m}_$i.json" 2> "$OUT/c2_pf${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_pf${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c2_pf${m}_$i.json"
  done
done
for i in 1 2; do
  for m in 1 2; do
    ZMPC_ROLLOUT_VARIANT=12 ZMPC_PREFETCH=$m timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dense-leg \
      > "$OUT/c2_v12_pf${m}_$i.json" 2> "$OUT/c2_v12_pf${m}_$i.err"
    rc=$?; [ $rc -ne 0 ] && { tail -5 "$OUT/c2_v12_pf${m}_$i.err"; exit $rc; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['roofline']['kernel_ms']*1e3, d['roofline']['frac'])" "$OUT/c2_v12_pf${m}_$i.json"
  done
done
