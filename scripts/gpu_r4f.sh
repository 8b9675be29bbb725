#!/bin/bash
# Round 4 GPU session f: the parallel-in-time small-batch strict kernel — strict tests, the
# small-batch sweep, config 3 (large-batch path unchanged).
set -u
OUT=gpurun_out/${1:-r4f}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "${2:-strict or herdt}" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 500 python scripts/strict_small_batch.py > "$OUT/small_batch.jsonl" 2> "$OUT/small_batch.err"
step small $?; cat "$OUT/small_batch.jsonl"
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for v in base hbase base hbase; do  # Herdt: this build vs the last commit's herdt.hip, alternated
  if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
  ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config 6 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c6_$v.json" 2> "$OUT/bench_c6_$v.err"
  step "config6 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/bench_c6_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline'].get('kernel_ms'), d.get('com_rmse_vs_ref'))"
done
# strict LQ kernel A/B of build-time parameters (csrc/Makefile `ab`): segment length, drift
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for c in 3 4; do
  for v in base s6 d8 s6d8; do
    if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
    ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_c${c}_$v.json" 2> "$OUT/ab_c${c}_$v.err"
    step "ab config$c $v" $?; python3 -c "import json,sys; d=json.loads(open('$OUT/ab_c${c}_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['passes_per_solve'], d['roofline']['lane_efficiency'])"
  done
done
