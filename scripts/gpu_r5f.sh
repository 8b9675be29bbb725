#!/bin/bash
# Round 5: config 4 A/B of the strict LQ kernel's bound form (rows / runs) and checkpoint policy
# (cached / non-temporal), diagnostics build for all four (ZMPC_LQ_NT), alternated twice.
set -u
T=${1:-r5f}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for rep in 1 2; do
  for cfg in "rows 0 1" "runs 0 2" "rows 1 1" "runs 1 2"; do
    set -- $cfg
    ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_NT=$2 timeout -k 10 300 python bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline --option strict_bounds=$3 > "$OUT/c4_$1_nt$2_$rep.json" 2> "$OUT/c4_$1_nt$2_$rep.err" || exit $?
    python -c "import json;d=json.load(open('$OUT/c4_$1_nt$2_$rep.json'));print('$1 nt=$2 rep $rep', round(d['roofline']['kernel_ms'],2))"
  done
done
