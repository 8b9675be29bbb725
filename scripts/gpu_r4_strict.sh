#!/bin/bash
# Round 4 strict iteration: strict GPU tests, config 3 / 4 bench lines, small-batch strict timings.
set -u
OUT=gpurun_out/${1:-r4s}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "${2:-strict}" > "$OUT/pytest_strict.log" 2>&1
rc=$?; echo "strict tests rc=$rc"; tail -2 "$OUT/pytest_strict.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
rc=$?; echo "config3 rc=$rc"; cut -c1-200 "$OUT/bench_c3.json"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
rc=$?; echo "config4 rc=$rc"; cut -c1-200 "$OUT/bench_c4.json"; [ $rc -ne 0 ] && exit $rc
if [ "${3:-}" = "small" ]; then
  timeout -k 10 400 python scripts/strict_small_batch.py > "$OUT/small_batch.jsonl" 2> "$OUT/small_batch.err"
  rc=$?; echo "small batch rc=$rc"; cat "$OUT/small_batch.jsonl"; exit $rc
fi
