#!/bin/bash
# Strict-kernel SQ counters (each set in its own rocprofv3 pass, kernel-trace only).
set -u
OUT=gpurun_out/${1:-spmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in "SQ_WAVES SQ_WAVE_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA" "SQ_INSTS_VMEM_RD SQ_INSTS_LDS" "SQ_INSTS_VALU SQ_INSTS_SALU" \
         "SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD" "SQ_INSTS_BRANCH SQ_INSTS_SMEM" "SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA" \
         "SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC"; do
  T=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/$T" -o run -- \
    python3 scripts/strict_once.py ${2:-2048} > "$OUT/$T.log" 2>&1 || exit $?
done
echo done
