#!/bin/bash
# Round 4 GPU session w: Herdt per-timestep epilogue — the kind pass skipped for windows without
# standing rows, the warm-start shift as dword rounds (ep) vs the product build (base).
set -u
OUT=gpurun_out/${1:-r4w}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
ZMPC_LIB=$PWD/$L/ab/libzmpc_ep.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k herdt > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
ZMPC_LIB=$PWD/$L/ab/libzmpc_ep.so timeout -k 10 120 python scripts/herdt_once.py 512 /tmp/new.npy > "$OUT/once_new.log" 2>&1
step once_new $?
ZMPC_LIB=$PWD/$L/libzmpc.so timeout -k 10 120 python scripts/herdt_once.py 512 /tmp/old.npy > "$OUT/once_old.log" 2>&1
step once_old $?
python3 -c "import numpy as np; a=np.load('/tmp/new.npy'); b=np.load('/tmp/old.npy'); print('bitwise equal', np.array_equal(a,b,equal_nan=True), 'max abs diff', np.nanmax(np.abs(a-b)), 'nan pattern equal', np.array_equal(np.isnan(a), np.isnan(b)))"
for v in ep base ep base; do
  if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
  ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config 6 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c6_$v.json" 2> "$OUT/bench_c6_$v.err"
  step "config6 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/bench_c6_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline'].get('passes_per_solve'), d.get('com_rmse_vs_ref'))"
done
