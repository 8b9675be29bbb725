"""Debug: LQ kernel histories with the library in ZMPC_LIB, B walks, saved to argv[1]."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd"),
                os.path.join(ROOT, "tests")]
from conftest import golden  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402

cop = golden("walk_n150.npz")
B = int(sys.argv[2])
zmax = np.repeat(cop["zmax"][None], B, 0).copy()
zmin = np.repeat(cop["zmin"][None], B, 0).copy()
dt = float(cop["dt"])
n = zmax.shape[1]
x0 = np.zeros((B, 2, 3))
out = {}
for bounds in (1, 2):
    p = Plan(0, 150, dt, 0.75, 9.81, 1.0, 1e-6, True).set_option("strict_solver", 3)
    p.set_option("strict_bounds", bounds)
    p.counters(reset=True)
    h, st = p.rollout(zmax, zmin, x0)
    out[f"h{bounds}"] = h.cpu().numpy()
    out[f"st{bounds}"] = st.cpu().numpy()
    print(bounds, "status", np.unique(out[f"st{bounds}"]), p.counters()["instance_passes"] / (B * (n - 1) * 2))
np.savez(sys.argv[1], **out)
