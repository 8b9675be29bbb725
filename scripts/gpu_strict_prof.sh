#!/bin/bash
# Strict (config 3/4) profile: rocprofv3 kernel stats, HBM PMC passes (FETCH_SIZE / WRITE_SIZE
# in their own runs, kernel-trace only), SQ issue/wait counters, L2 hit counters.
# Usage: bash scripts/gpu_strict_prof.sh <tag> [config]     outputs under gpurun_out/<tag>/
set -u
TAG=${1:-sprof}
CONF=${2:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$CONF" = 3 ]; then WL=config3_n150_b65536; else WL=config4_n150_b125000; fi
K=zmpc_strict_lq_kernel
ARGS="--config $CONF --steps 3 --warmup 1 --no-cpu-baseline"
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o bench -- \
    python3 bench.py $ARGS > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
step stats $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- \
    python3 bench.py $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
step fetch $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- \
    python3 bench.py $ARGS > "$OUT/write_bench.json" 2> "$OUT/write.err"
step write $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    --output-format csv -d "$OUT/sq" -o bench -- \
    python3 bench.py $ARGS > "$OUT/sq_bench.json" 2> "$OUT/sq.err"
step sq $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum \
    --output-format csv -d "$OUT/tcc" -o bench -- \
    python3 bench.py $ARGS > "$OUT/tcc_bench.json" 2> "$OUT/tcc.err"
step tcc $?
python3 profiles/collect_pmc.py "$OUT" "$WL" "$K" > "$OUT/pmc.json"
step collect $?
exit 0
