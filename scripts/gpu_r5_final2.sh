#!/bin/bash
# Round 5 closing session, part 2: config 6 kernel stats + HBM PMC passes, then the bench lines
# of configs 3, 4, 5, 6, 4-unconstrained and the default line, each with its CPU leg.
set -u
T=${1:-r5fin}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
bash scripts/gpu_profile_round.sh ${T}_c6 config6_n150_b32768 zmpc_herdt "--config 6 --steps 2 --warmup 1" > "$OUT/c6prof.log" 2>&1
step profile_c6 $?; tail -1 "$OUT/c6prof.log" | cut -c1-200
for c in 3 4 5 6; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 2 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  step "config$c" $?; cut -c1-200 "$OUT/bench_c$c.json"
done
timeout -k 10 600 python bench.py --config 4 --unconstrained --steps 20 --warmup 3 > "$OUT/bench_c4unc.json" 2> "$OUT/bench_c4unc.err"
step "config4 unc" $?; cut -c1-200 "$OUT/bench_c4unc.json"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cut -c1-300 "$OUT/bench_default.json"
