#!/bin/bash
# Round 4 GPU session y: config 4 (shared CoP) with run-length bounds (strict_bounds=2) against
# the automatic choice (rows for a shared CoP), now that the run cursor tests once per segment.
set -u
OUT=gpurun_out/${1:-r4y}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
for r in 1 2; do
  for v in runs auto; do
    opt=""; [ $v = runs ] && opt="--option strict_bounds=2"
    timeout -k 10 300 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline $opt > "$OUT/c4_${v}_$r.json" 2> "$OUT/c4_${v}_$r.err"
    step "config4 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/c4_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['passes_per_solve'], d['config'].get('plan_options'))"
  done
done
