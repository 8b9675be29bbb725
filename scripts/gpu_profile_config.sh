#!/bin/bash
# Profile one bench workload: rocprofv3 kernel stats, HBM PMC passes (FETCH_SIZE / WRITE_SIZE,
# each in its own kernel-trace-only run), profiles/pmc_<workload>.json, then the bench line
# with that traffic.  Usage:
#   bash scripts/gpu_profile_config.sh <tag> <workload> <kernel-substring> [bench args...]
# e.g. bash scripts/gpu_profile_config.sh r2_c5 config5_n512_b2048 wide_kernel --config 5
set -u
TAG=$1; WL=$2; K=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="$* --steps 10 --warmup 2 --no-cpu-baseline"
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
python3 profiles/collect_pmc.py "$OUT" "$WL" "$K" > "$OUT/pmc.json"
step collect $?
cp profiles/pmc_$WL.json "$OUT/"
timeout -k 10 400 python3 bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench $?
cat "$OUT/bench.json"
