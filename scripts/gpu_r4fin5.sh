#!/bin/bash
# Round 4 fifth closing session: the strict LQ task body as a lambda (libzmpc.so) — every GPU
# test, smoke, config 4 kernel stats + HBM PMC passes + bench line with its CPU legs, config 3
# bench line with its CPU legs, the default bench line.
set -u
T=${1:-r4fin5}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step smoke $?; tail -1 "$OUT/smoke.log"
bash scripts/gpu_profile_round.sh ${T}_c4 config4_n150_b125000 zmpc_strict_lq_kernel "--config 4 --steps 2 --warmup 1" > "$OUT/c4prof.log" 2>&1
step profile_c4 $?; tail -1 "$OUT/c4prof.log" | cut -c1-200
timeout -k 10 600 python bench.py --config 4 --steps 5 --warmup 2 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
step config4 $?; cut -c1-200 "$OUT/bench_c4.json"
timeout -k 10 600 python bench.py --config 3 --steps 5 --warmup 2 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"
step config3 $?; cut -c1-200 "$OUT/bench_c3.json"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cut -c1-300 "$OUT/bench_default.json"
