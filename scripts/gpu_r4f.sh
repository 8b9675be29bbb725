#!/bin/bash
# Round 4 GPU session f: the parallel-in-time small-batch strict kernel — strict tests, the
# small-batch sweep, config 3 (large-batch path unchanged).
set -u
OUT=gpurun_out/${1:-r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-strict}" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 500 python scripts/strict_small_batch.py > "$OUT/small_batch.jsonl" 2> "$OUT/small_batch.err"
step small $?; cat "$OUT/small_batch.jsonl"
