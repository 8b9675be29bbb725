#!/bin/bash
# Round 4 GPU session q: Herdt per-phase clocks (diagnostics builds, ZMPC_HERDT_PROF) of the last
# commit's kernel and of the light-sweep-2 variant, config 6 inputs.
set -u
OUT=gpurun_out/${1:-r4q}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
for v in hbase_diag light_diag; do
  ZMPC_HERDT_PROF=1 ZMPC_LIB=$PWD/$L/ab/libzmpc_$v.so timeout -k 10 180 python scripts/herdt_once.py 32768 > "$OUT/prof_$v.log" 2>&1
  step "prof $v" $?; grep -v amdgpu.ids "$OUT/prof_$v.log"
done
