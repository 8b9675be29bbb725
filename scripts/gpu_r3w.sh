#!/bin/bash
# Round 3: strict LQ — segment 0 reused between the sweeps (current libzmpc.so) vs the base build
# (libzmpc_base.so, A/B only), config 3; strict GPU tests on the new build.
set -u
OUT=gpurun_out/r3w
mkdir -p "$OUT"
export TMPDIR=/tmp
D=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "strict" > "$OUT/pytest_strict.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest_strict.log"; [ $rc -ne 0 ] && exit $rc
for R in 1 2 3; do
  ZMPC_LIB=$D/libzmpc_base.so timeout -k 10 300 python scripts/strict_axis_diag.py 65536 0 > "$OUT/base_$R.jsonl" 2>&1 || exit $?
  timeout -k 10 300 python scripts/strict_axis_diag.py 65536 0 > "$OUT/new_$R.jsonl" 2>&1 || exit $?
  echo "base $(cut -c1-60 $OUT/base_$R.jsonl) | new $(cut -c1-60 $OUT/new_$R.jsonl)"
done
