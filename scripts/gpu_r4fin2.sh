#!/bin/bash
# Round 4 second closing session: (1) A/B of the Herdt kernel with sweep 1 branch-free too
# (ab/libzmpc_bf3.so) against the product build; (2) the product build: every GPU test, smoke,
# config 6 kernel stats + HBM PMC passes + bench line, config 6 with its CPU leg, the default
# bench line.
set -u
T=${1:-r4fin2}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
ZMPC_LIB=$PWD/$L/ab/libzmpc_bf3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k herdt > "$OUT/pytest_bf3.log" 2>&1
step pytest_bf3 $?; tail -1 "$OUT/pytest_bf3.log"
ZMPC_LIB=$PWD/$L/ab/libzmpc_bf3.so timeout -k 10 120 python scripts/herdt_once.py 512 /tmp/new.npy > "$OUT/once_new.log" 2>&1
step once_new $?
ZMPC_LIB=$PWD/$L/libzmpc.so timeout -k 10 120 python scripts/herdt_once.py 512 /tmp/old.npy > "$OUT/once_old.log" 2>&1
step once_old $?
python3 -c "import numpy as np; a=np.load('/tmp/new.npy'); b=np.load('/tmp/old.npy'); print('bitwise equal', np.array_equal(a,b,equal_nan=True), 'max abs diff', np.nanmax(np.abs(a-b)), 'nan pattern equal', np.array_equal(np.isnan(a), np.isnan(b)))"
for v in bf3 base bf3 base; do
  if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
  ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config 6 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_c6_$v.json" 2> "$OUT/ab_c6_$v.err"
  step "ab config6 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/ab_c6_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline'].get('passes_per_solve'), d.get('com_rmse_vs_ref'))"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
step smoke $?; tail -1 "$OUT/smoke.log"
bash scripts/gpu_profile_round.sh ${T}_c6 config6_n150_b32768 zmpc_herdt "--config 6 --steps 2 --warmup 1" > "$OUT/c6prof.log" 2>&1
step profile_c6 $?; tail -1 "$OUT/c6prof.log" | cut -c1-200
timeout -k 10 600 python bench.py --config 6 --steps 5 --warmup 2 > "$OUT/bench_c6.json" 2> "$OUT/bench_c6.err"
step config6 $?; cut -c1-200 "$OUT/bench_c6.json"
timeout -k 10 300 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err"
step default $?; cut -c1-300 "$OUT/bench_default.json"
