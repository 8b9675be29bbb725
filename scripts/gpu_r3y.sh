#!/bin/bash
# Round 3: refresh the HBM PMC traffic files of configs 3, 4u and 5 for the current kernels.
set -u
bash scripts/gpu_profile_round.sh r3y/c3 config3_n150_b65536 strict_lq_kernel --config 3 --steps 2 --warmup 1 > gpurun_out/r3y_c3.log 2>&1
rc=$?; tail -3 gpurun_out/r3y_c3.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile_round.sh r3y/c4u config4_unc_n150_b125000 splitd_kernel --config 4 --unconstrained --steps 3 --warmup 1 > gpurun_out/r3y_c4u.log 2>&1
rc=$?; tail -3 gpurun_out/r3y_c4u.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_profile_round.sh r3y/c5 config5_n512_b2048 wide_kernel --config 5 --steps 5 --warmup 1 > gpurun_out/r3y_c5.log 2>&1
rc=$?; tail -3 gpurun_out/r3y_c5.log; exit $rc
