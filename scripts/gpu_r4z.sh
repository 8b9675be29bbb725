#!/bin/bash
# Round 4 GPU session z: strict LQ task queue, the task loop inlined (q: a resident grid, each wave refilled with the
# next y then x task when it finishes) vs the product build (base) — strict GPU tests on q,
# configs 3 and 4 alternated.
set -u
OUT=gpurun_out/${1:-r4z}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
ZMPC_LIB=$PWD/$L/ab/libzmpc_q.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k strict > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
for c in 3 4; do
  for v in q base q base; do
    if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
    ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_c${c}_$v.json" 2> "$OUT/ab_c${c}_$v.err"
    step "ab config$c $v" $?; python3 -c "import json; d=json.loads(open('$OUT/ab_c${c}_$v.json').read().strip().splitlines()[-1]); print('$c $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['passes_per_solve'])"
  done
done
