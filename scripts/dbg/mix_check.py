"""Debug: the kick-order test's batch through the LQ kernel — statuses and pass counters."""
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
B = 1000
rng = np.random.default_rng(21)
off = rng.uniform(-0.02, 0.02, (B, 1, 2))
zmax = cop["zmax"][None] + off
zmin = cop["zmin"][None] + off
x0 = np.zeros((B, 2, 3))
x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
dt = float(cop["dt"])
n = zmax.shape[1]
rng = np.random.default_rng(22)
F = rng.uniform(-800.0, 800.0, B)
ks = rng.integers(n // 4, 3 * n // 4, B).astype(np.int64)
for mode in (1, 0):
    p = Plan(0, 150, dt, 0.75, 9.81, 1.0, 1e-6, True).set_option("strict_solver", 3)
    p.set_option("kick_order", mode)
    p.counters(reset=True)
    h, st = p.rollout(zmax, zmin, x0, kick=dt * F / 40.0, kick_step=ks)
    st = st.cpu().numpy()
    c = p.counters()
    bad = np.nonzero(st)[0]
    print("kick_order", mode, "bad walks", bad[:20], len(bad), "F", F[bad[:5]], "ks", ks[bad[:5]], c)
