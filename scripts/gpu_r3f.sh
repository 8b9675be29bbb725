#!/bin/bash
# Round 3: r3e (bench, kernel stats, plan stats, sweep) + strict LQ A/B.
set -u
bash scripts/gpu_r3e.sh || exit $?
bash scripts/gpu_strict_ab_r3.sh r3s
