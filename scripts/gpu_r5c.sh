#!/bin/bash
# Round 5: the Herdt weight fixtures on the device, and the strict LQ kernel's per-phase clocks
# (diagnostics build, ZMPC_LQ_PROF) for config 3 and config 4.
set -u
T=${1:-r5c}
OUT=gpurun_out/$T
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 600 python -u -m pytest tests/test_gpu_herdt.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_herdt.log" 2>&1
echo "== pytest herdt rc=$?"; grep -E "PASS|FAIL|Error|assert" "$OUT/pytest_herdt.log" | head -30
ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_PROF=1 timeout -k 10 600 python bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c3.json" 2> "$OUT/prof_c3.err"
step prof_c3 $?; grep "lq prof" "$OUT/prof_c3.err" | tail -2
ZMPC_LIB=$PWD/$L/libzmpc_diag.so ZMPC_LQ_PROF=1 timeout -k 10 600 python bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof_c4.json" 2> "$OUT/prof_c4.err"
step prof_c4 $?; grep "lq prof" "$OUT/prof_c4.err" | tail -2
