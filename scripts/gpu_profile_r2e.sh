#!/bin/bash
# Round-2 closing profiles: kernel stats + HBM PMC + bench line for configs 2, 4 (unc), 5, 3.
set -u
bash scripts/gpu_profile_config.sh r2e_c2 config2_n150_b4096 pers_kernel || exit $?
bash scripts/gpu_profile_config.sh r2e_c4u config4_unc_n150_b125000 split_kernel --config 4 --unconstrained --cpu-seconds 5 || exit $?
bash scripts/gpu_profile_config.sh r2e_c5 config5_n512_b2048 wide_kernel --config 5 --cpu-seconds 5 || exit $?
bash scripts/gpu_profile_config.sh r2e_c3 config3_n150_b65536 strict_lq_kernel --config 3 --cpu-seconds 5 --steps 3 --warmup 1 || exit $?
