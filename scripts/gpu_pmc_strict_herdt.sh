#!/bin/bash
# HBM PMC passes (and kernel stats) for config 4 strict and config 6 Herdt, so their bench lines
# carry roofline.traffic.
set -u
export TMPDIR=/tmp
bash scripts/gpu_profile_round.sh ${1:-r3pmc}_c4 config4_n150_b125000 zmpc_strict_lq_kernel "--config 4 --steps 2 --warmup 1" || exit $?
bash scripts/gpu_profile_round.sh ${1:-r3pmc}_c6 config6_n150_b32768 zmpc_herdt "--config 6 --steps 2 --warmup 1" || exit $?
