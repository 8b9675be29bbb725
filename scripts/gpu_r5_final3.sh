#!/bin/bash
# Round 5 closing session 3 (after the per-segment flag words and the run cursor's deferred
# refill): every GPU test, smoke, config 3 and 4 strict kernel stats + HBM PMC passes, their
# bench lines with CPU legs, the default line.
set -u
T=${1:-r5fin3}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step smoke $?; tail -1 "$OUT/smoke.log"
bash scripts/gpu_profile_round.sh ${T}_c3 config3_n150_b65536 zmpc_strict_lq_kernel "--config 3 --steps 2 --warmup 1" > "$OUT/c3prof.log" 2>&1
step profile_c3 $?; tail -1 "$OUT/c3prof.log" | cut -c1-200
bash scripts/gpu_profile_round.sh ${T}_c4 config4_n150_b125000 zmpc_strict_lq_kernel "--config 4 --steps 2 --warmup 1" > "$OUT/c4prof.log" 2>&1
step profile_c4 $?; tail -1 "$OUT/c4prof.log" | cut -c1-200
for c in 3 4; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 2 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  step "config$c" $?; cut -c1-200 "$OUT/bench_c$c.json"
done
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cut -c1-300 "$OUT/bench_default.json"
