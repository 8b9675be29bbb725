#!/bin/bash
# SQ/GRBM counters of the Herdt kernel (scripts/herdt_once.py), one rocprofv3 pass
# per counter set (kernel-trace only), for the ZMPC_* env the caller exports.
# usage: bash scripts/gpu_herdt_pmc.sh <tag> [B]
set -u
OUT=gpurun_out/$1
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/p$i" -o run -- \
    python3 scripts/herdt_once.py ${2:-32768} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done
python3 scripts/pmc_summary.py "$OUT" herdt > "$OUT/summary.json"; cat "$OUT/summary.json"
