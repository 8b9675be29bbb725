#!/bin/bash
# Strict LQ phase clocks (diagnostics build, ZMPC_LQ_PROF) for the given bench configs.
# Usage: scripts/gpu_lqprof.sh TAG [CONFIGS...]
set -u
T=$1; shift
CONFIGS=${*:-3 4}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for c in $CONFIGS; do
  ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_PROF=1 timeout -k 10 300 python bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c$c.json" 2> "$OUT/prof_c$c.err" || exit $?
  grep "lq prof" "$OUT/prof_c$c.err" | tail -2
done
