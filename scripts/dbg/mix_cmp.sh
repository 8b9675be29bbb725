#!/bin/bash
set -u
mkdir -p gpurun_out/mix
L=model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal
timeout -k 10 120 python scripts/dbg/mix_cmp.py gpurun_out/mix/mix.npz 64 || exit $?
ZMPC_LIB=$PWD/$L/ab/libzmpc_nomix.so timeout -k 10 120 python scripts/dbg/mix_cmp.py gpurun_out/mix/nomix.npz 64 || exit $?
python3 - <<'PY'
import numpy as np
a = np.load("gpurun_out/mix/mix.npz"); b = np.load("gpurun_out/mix/nomix.npz")
for k in ("h1", "h2"):
    d = np.abs(a[k] - b[k])
    print(k, "x axis max", d[:, :, 0].max(), "y axis max", d[:, :, 1].max(), "first step", np.argmax(d.max(axis=(0, 2, 3)) > 1e-12))
PY
