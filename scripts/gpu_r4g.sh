#!/bin/bash
# Round 4 GPU session g: the horizon sweep (run_compare_runtime.py:139 semantics; strict leg at
# 1024 walks now on the small-batch kernel), kernel stats of the default bench line.
set -u
OUT=gpurun_out/${1:-r4g}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python bench.py --sweep-horizon ${2:-10:300:10} --no-cpu-baseline > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
step sweep $?; tail -1 "$OUT/sweep.jsonl" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_default" -o run -- python3 bench.py --no-dense-leg > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default_prof $?; cut -c1-300 "$OUT/bench_default.json"
