#!/bin/bash
# Round 4 GPU session l: mixed-axis waves in the strict LQ kernel — strict tests (LQ paths) and
# configs 3 / 4 against the axis-pure build, alternated.
set -u
OUT=gpurun_out/${1:-r4l}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "strict" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for c in 3 4; do
  for v in mix nomix mix nomix; do
    if [ $v = mix ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
    ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_$v.json" 2> "$OUT/c${c}_$v.err"
    step "config$c $v" $?; python3 -c "import json; d=json.loads(open('$OUT/c${c}_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c $v', d['ms_per_step'], r['passes_per_solve'], r['lane_efficiency'], r['working_set_slot_frac'])"
  done
done
