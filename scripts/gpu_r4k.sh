#!/bin/bash
# Round 4 GPU session k: the wide kernel's padded history staging — unconstrained tests, config 5
# and the long-walk horizons against the previous commit's rollout.hip.
set -u
OUT=gpurun_out/${1:-r4k}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "not strict and not herdt and not nccl and not bench" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for v in new head new head; do
  if [ $v = new ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_rohead.so; fi
  ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config 5 --steps 20 --warmup 3 --no-cpu-baseline --no-dense-leg > "$OUT/c5_$v.json" 2> "$OUT/c5_$v.err"
  step "config5 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['frac'])"
  for N in 230 260; do
    ZMPC_LIB=$lib timeout -k 10 300 python bench.py --horizon $N --steps 20 --warmup 3 --no-cpu-baseline --no-dense-leg > "$OUT/n${N}_$v.json" 2> "$OUT/n${N}_$v.err"
    step "N$N $v" $?; python3 -c "import json; d=json.loads(open('$OUT/n${N}_$v.json').read().strip().splitlines()[-1]); print('$v N=$N', d['ms_per_step'])"
  done
done
