#!/bin/bash
# Round 4 GPU session t: how long the Herdt forward sweep waits on its slab-row loads
# (diagnostics build, ZMPC_HERDT_PROF: an explicit vmcnt(0) wait after each block's loads).
set -u
OUT=gpurun_out/${1:-r4t}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
ZMPC_HERDT_PROF=1 ZMPC_LIB=$PWD/$L/ab/libzmpc_hcen_diag.so timeout -k 10 180 python scripts/herdt_once.py 32768 > "$OUT/prof_hcen.log" 2>&1
step prof $?; grep "herdt prof" "$OUT/prof_hcen.log" | tail -1
# the forward sweep with two 4-row blocks ping-ponging (libzmpc.so) vs the single 8-row block
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k herdt > "$OUT/pytest.log" 2>&1
step pytest $?; tail -1 "$OUT/pytest.log"
for v in base hcen base hcen; do
  if [ $v = base ]; then lib=$PWD/$L/libzmpc.so; else lib=$PWD/$L/ab/libzmpc_$v.so; fi
  ZMPC_LIB=$lib timeout -k 10 300 python bench.py --config 6 --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c6_$v.json" 2> "$OUT/bench_c6_$v.err"
  step "config6 $v" $?; python3 -c "import json; d=json.loads(open('$OUT/bench_c6_$v.json').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline'].get('kernel_ms'), d['roofline'].get('passes_per_solve'), d.get('com_rmse_vs_ref'))"
done
