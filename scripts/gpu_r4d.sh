#!/bin/bash
# Round 4 combined GPU session: tests touched this round, strict small-batch sweep, config 3,
# the horizon sweep (product vs the round-3 persistent even-CW rule), SQ counters of config 3.
set -u
OUT=gpurun_out/${1:-r4d}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-strict or environment or variants or chunk or fft or sparse or nccl or herdt}" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 500 python scripts/strict_small_batch.py > "$OUT/small_batch.jsonl" 2> "$OUT/small_batch.err"
step small $?; cat "$OUT/small_batch.jsonl"
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
step config3 $?; cut -c1-160 "$OUT/bench_c3.json"
bash scripts/gpu_r4_sweep.sh ${1:-r4d}/sweep 10:300:10 pers > "$OUT/sweep.log" 2>&1
step sweep $?; cat "$OUT/sweep.log" | cut -c1-300
bash scripts/gpu_strict_sq.sh ${1:-r4d}/sq 65536 > "$OUT/sq.log" 2>&1
step sq $?; tail -30 "$OUT/sq.log"
