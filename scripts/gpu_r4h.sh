#!/bin/bash
# Round 4 GPU session h: Herdt A/B of this round's two changes (each alone), the small-batch
# kernel's crossover with the LQ kernel at larger batches, the horizon sweep.
set -u
OUT=gpurun_out/${1:-r4h}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for v in hbase hlo hdb hbase hlo hdb; do
  ZMPC_LIB=$PWD/$L/ab/libzmpc_$v.so timeout -k 10 300 python bench.py --config 6 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c6_$v.json" 2> "$OUT/bench_c6_$v.err"
  step "config6 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/bench_c6_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d.get('com_rmse_vs_ref'))"
done
SIZES=4096,8192,16384 SOLVERS=4,3 timeout -k 10 600 python scripts/strict_small_batch.py > "$OUT/crossover.jsonl" 2> "$OUT/crossover.err"
step crossover $?; cut -c1-120 "$OUT/crossover.jsonl"
timeout -k 10 900 python bench.py --sweep-horizon 10:300:10 --no-cpu-baseline > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
step sweep $?; tail -1 "$OUT/sweep.jsonl" | cut -c1-300
