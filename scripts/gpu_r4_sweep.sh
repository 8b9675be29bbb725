#!/bin/bash
# Horizon sweep (run_compare_runtime.py:139 semantics) with the product library, then the
# diagnostics library with the round-3 persistent even-CW rule (ZMPC_PERSISTENT) for A/B.
set -u
OUT=gpurun_out/${1:-r4sw}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --sweep-horizon ${2:-10:300:10} --no-cpu-baseline > "$OUT/sweep.jsonl" 2> "$OUT/sweep.err"
rc=$?; echo "sweep rc=$rc"; tail -1 "$OUT/sweep.jsonl" | cut -c1-600; [ $rc -ne 0 ] && exit $rc
if [ -n "${3:-}" ]; then
  ZMPC_LIB=$PWD/model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/libzmpc_diag.so ZMPC_PERSISTENT=1 \
    timeout -k 10 600 python bench.py --sweep-horizon ${2:-10:300:10} --no-cpu-baseline > "$OUT/sweep_pers.jsonl" 2> "$OUT/sweep_pers.err"
  rc=$?; echo "sweep pers rc=$rc"; tail -1 "$OUT/sweep_pers.jsonl" | cut -c1-600
fi
exit $rc
