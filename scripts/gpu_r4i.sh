#!/bin/bash
# Round 4 GPU session i: tests touched by the CW-8 routing and the scan crossover, the
# unconstrained horizon probe and the full horizon sweep.
set -u
OUT=gpurun_out/${1:-r4i}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-strict or variants or herdt or fft or sparse or chunk or controller}" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
bash scripts/dbg/horizon_probe.sh ${1:-r4i}/probe > "$OUT/probe.log" 2>&1
step probe $?; cat "$OUT/probe.log" | cut -c1-200
timeout -k 10 900 python bench.py --sweep-horizon 10:300:10 --no-cpu-baseline > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
step sweep $?; tail -1 "$OUT/sweep.jsonl" | cut -c1-200
