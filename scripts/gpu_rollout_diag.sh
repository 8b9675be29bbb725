#!/bin/bash
# Rollout kernel diagnostics: SQ counters (own passes, kernel-trace).
set -u
OUT=gpurun_out/${1:-diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in 5 1; do
  for C in "SQ_WAVES SQ_WAVE_CYCLES" "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_SALU SQ_INSTS_SMEM"; do
    T=$(echo $C | tr ' ' '_')
    ZMPC_ROLLOUT_VARIANT=$V timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv \
      -d "$OUT/pmc_v${V}_$T" -o run -- python3 scripts/rollout_once.py > "$OUT/pmc_v${V}_$T.log" 2>&1 || exit $?
  done
done
echo done
