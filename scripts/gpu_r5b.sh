#!/bin/bash
# Round 5: the strict LQ kernel without spills (free-slot flags written in the forward,
# 32-bit lane counters, uniform run-table bases): every GPU test (Herdt weight fixtures
# excluded until generated), config 3 / 4 bench lines, and the diagnostics build's per-phase
# clocks (ZMPC_LQ_PROF) for both.
set -u
T=${1:-r5b}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not herdt_weights" > "$OUT/pytest.log" 2>&1
echo "== pytest rc=$?"; tail -15 "$OUT/pytest.log"
timeout -k 10 600 python bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
step config3 $?; cut -c1-300 "$OUT/bench_c3.json"
timeout -k 10 600 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
step config4 $?; cut -c1-300 "$OUT/bench_c4.json"
ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_PROF=1 timeout -k 10 600 python bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err"
step prof_c3 $?; grep "lq prof" "$OUT/prof_c3.err" | tail -4
ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_PROF=1 timeout -k 10 600 python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err"
step prof_c4 $?; grep "lq prof" "$OUT/prof_c4.err" | tail -4
