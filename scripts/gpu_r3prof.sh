#!/bin/bash
# Round 3 (sparse correlation): profile rounds for config 2 and config 5, then the default
# bench lines with their CPU legs.
set -u
export TMPDIR=/tmp
bash scripts/gpu_profile_round.sh r3prof_c2 config2_n150_b4096 zmpc_rollout_unc "--steps 20 --warmup 3" || exit $?
bash scripts/gpu_profile_round.sh r3prof_c5 config5_n512_b2048 zmpc_rollout_unc "--config 5 --steps 20 --warmup 3" || exit $?
OUT=gpurun_out/r3prof
mkdir -p $OUT
timeout -k 10 600 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
timeout -k 10 600 python bench.py --config 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit $?
cat $OUT/bench_c5.json
