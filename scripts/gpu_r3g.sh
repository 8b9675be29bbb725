#!/bin/bash
# Round 3: strict LQ A/B (prefetch variant) + MFMA counters of the plan Gram kernels.
set -u
OUT=gpurun_out/r3g
mkdir -p "$OUT"
export TMPDIR=/tmp
bash scripts/gpu_strict_ab_r3.sh r3s || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_gram" -o run -- python3 scripts/plan_timing.py 150 512 2048 > "$OUT/pmc_gram.log" 2>&1
rc=$?; echo "pmc gram rc=$rc"; tail -2 "$OUT/pmc_gram.log"
exit $rc
