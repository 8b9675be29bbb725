#!/bin/bash
# Round 4 GPU session e: tests touched this round (wave kernel, run-length bounds), strict
# small-batch sweep, config 3/4 with rows vs run-length bounds, SQ/traffic counters of config 3.
set -u
OUT=gpurun_out/${1:-r4e}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-strict or environment or herdt}" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 500 python scripts/strict_small_batch.py > "$OUT/small_batch.jsonl" 2> "$OUT/small_batch.err"
step small $?; cat "$OUT/small_batch.jsonl"
for c in 3 4; do
  for b in 1 2; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --option strict_bounds=$b \
      > "$OUT/bench_c${c}_b$b.json" 2> "$OUT/bench_c${c}_b$b.err"
    step "config$c bounds$b" $?; cut -c1-200 "$OUT/bench_c${c}_b$b.json"
  done
done
bash scripts/gpu_strict_sq.sh ${1:-r4e}/sq_b1 65536 strict_bounds=1 > "$OUT/sq_b1.log" 2>&1
step sq_b1 $?; tail -30 "$OUT/sq_b1.log"
bash scripts/gpu_strict_sq.sh ${1:-r4e}/sq_b2 65536 strict_bounds=2 > "$OUT/sq_b2.log" 2>&1
step sq_b2 $?; tail -30 "$OUT/sq_b2.log"
