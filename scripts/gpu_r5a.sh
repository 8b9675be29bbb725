#!/bin/bash
# Round 5, first check of the z-input strict step (strict_eta.h): every GPU test (the Herdt
# weight fixtures excluded until generated), smoke, config 3 / 4 strict bench lines, the
# default line.
set -u
T=${1:-r5a}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not herdt_weights" > "$OUT/pytest.log" 2>&1
echo "== pytest rc=$?"; tail -15 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step smoke $?; tail -1 "$OUT/smoke.log"
timeout -k 10 600 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
step config3 $?; cut -c1-400 "$OUT/bench_c3.json"
timeout -k 10 600 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
step config4 $?; cut -c1-400 "$OUT/bench_c4.json"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cut -c1-300 "$OUT/bench_default.json"
