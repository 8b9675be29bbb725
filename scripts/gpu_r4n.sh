#!/bin/bash
# Round 4 GPU session n: the free-segment form of sweep B (strict LQ kernel) — strict tests, then
# configs 3 / 4: this build (S = 8), S = 6, and the previous commit's kernel, alternated.
set -u
OUT=gpurun_out/${1:-r4n}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "strict" > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for c in 3 4; do
  for v in free lqhead s6free free lqhead s6free; do
    if [ $v = free ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
    ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/c${c}_$v.json" 2> "$OUT/c${c}_$v.err"
    step "config$c $v" $?; python3 -c "import json; d=json.loads(open('$OUT/c${c}_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c $v', round(d['ms_per_step'], 2), r['passes_per_solve'])"
  done
done
