#!/bin/bash
# Round 4 GPU session aa: the strict LQ task body as a lambda (lam: the queue instance spills 37-60
# VGPRs instead of 105-115, the loop-free one 56 instead of 33) vs the product build — strict
# GPU tests on lam, configs 4 and 3 alternated.
set -u
OUT=gpurun_out/${1:-r4aa}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
ZMPC_LIB=$PWD/$L/ab/libzmpc_lam.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k strict > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
for c in 4 3; do
  for r in 1 2; do
    for v in lam base; do
      if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
      ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/ab_c${c}_${v}_$r.json" 2> "$OUT/ab_c${c}_${v}_$r.err"
      step "ab config$c $v" $?; python3 -c "import json; d=json.loads(open('$OUT/ab_c${c}_${v}_$r.json').read().strip().splitlines()[-1]); print('$c $v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['passes_per_solve'])"
    done
  done
done
