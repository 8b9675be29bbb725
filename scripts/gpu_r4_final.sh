#!/bin/bash
# Round 4 closing session: every GPU test, smoke, the default bench line with kernel stats and
# HBM PMC passes, PMC passes of config 4 strict and config 6, the other configs' bench lines with
# their CPU legs, and the small-batch strict sweep.
set -u
T=${1:-r4fin}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step smoke $?; tail -1 "$OUT/smoke.log"
bash scripts/gpu_profile_round.sh ${T}_c2 > "$OUT/c2.log" 2>&1
step profile_c2 $?; tail -1 "$OUT/c2.log" | cut -c1-300
bash scripts/gpu_pmc_strict_herdt.sh $T > "$OUT/pmc.log" 2>&1
step pmc $?
for c in 3 4 5 6; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 2 > "$OUT/bench_c$c.json" 2> "$OUT/bench_c$c.err"
  step "config$c" $?; cut -c1-200 "$OUT/bench_c$c.json"
done
timeout -k 10 600 python bench.py --config 4 --unconstrained --steps 20 --warmup 3 > "$OUT/bench_c4unc.json" 2> "$OUT/bench_c4unc.err"
step "config4 unc" $?; cut -c1-200 "$OUT/bench_c4unc.json"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cat "$OUT/bench_default.json" | cut -c1-300
