#!/bin/bash
# PMC + ablation session for the unconstrained rollout kernel (diagnostics only).
# Counters are collected in their own runs (kernel-trace only), one counter group per pass.
set -u
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 600 python scripts/ablate_rollout.py > "$OUT/ablate.jsonl" 2> "$OUT/ablate.err"
rc=$?; echo "ablate rc=$rc"; cat "$OUT/ablate.jsonl"
[ $rc -ne 0 ] && exit $rc
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 $BENCH > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err"
  rc=$?; echo "pmc pass $i ($pmc) rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
