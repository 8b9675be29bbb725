#!/bin/bash
# Strict LQ kernel at config-3 size (strict_once.py, B walks): SQ counter passes (each set in its
# own rocprofv3 run, kernel-trace only) + FETCH_SIZE / WRITE_SIZE passes + kernel stats.
set -u
OUT=gpurun_out/${1:-r4sq}
B=${2:-65536}
shift 2 2>/dev/null
OPTS="$*"  # plan options NAME=VALUE
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- \
  python3 scripts/strict_once.py $B $OPTS > "$OUT/stats.log" 2>&1 || exit $?
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  T=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C --output-format csv -d "$OUT/$T" -o run -- \
    python3 scripts/strict_once.py $B $OPTS > "$OUT/$T.log" 2>&1 || exit $?
done
python3 scripts/pmc_summary.py "$OUT" zmpc_strict_lq > "$OUT/summary.json" 2>&1
cat "$OUT/summary.json"
