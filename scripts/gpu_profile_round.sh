#!/bin/bash
# Round profile: bench, rocprofv3 kernel stats, HBM PMC passes (FETCH_SIZE / WRITE_SIZE in their
# own runs, kernel-trace only), then the bench again with the traffic it now reads.
# Usage: bash scripts/gpu_profile_round.sh <tag> [workload kernel-substring bench-args...]
#   default: config2_n150_b4096 zmpc_rollout_unc "--steps 20 --warmup 3"
# outputs under gpurun_out/<tag>/
set -u
TAG=${1:-round}
WL=${2:-config2_n150_b4096}
K=${3:-zmpc_rollout_unc}
shift 3 2>/dev/null || shift $#
ARGS="${*:---steps 20 --warmup 3} --no-cpu-baseline --no-dense-leg"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 rc=$2"; if [ "$2" -ne 0 ]; then exit "$2"; fi; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o bench -- \
    python3 bench.py $ARGS > "$OUT/stats_bench.json" 2> "$OUT/stats.err"
step stats $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- \
    python3 bench.py $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
step fetch $?
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- \
    python3 bench.py $ARGS > "$OUT/write_bench.json" 2> "$OUT/write.err"
step write $?
python3 profiles/collect_pmc.py "$OUT" "$WL" "$K" > "$OUT/pmc.json"
step collect $?
cp profiles/pmc_$WL.json "$OUT/"
timeout -k 10 600 python3 bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
step bench $?
cat "$OUT/bench.json"
