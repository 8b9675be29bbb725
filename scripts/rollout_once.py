"""Diagnostic driver for profilers: 20 launches of the config-2-shaped unconstrained rollout
(B from argv, default 4096) with whatever ZMPC_* env vars the caller set."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "model-predictive-control-for-bipedal-locomotion_amd"))
from mpc_bipedal.solver import Plan  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N, n = 150, 420
p = Plan(0, N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, False)
rng = np.random.default_rng(0)
zc = np.cumsum(rng.normal(0, 0.01, (B, n, 2)), 1)
zmax = torch.as_tensor(zc + 0.05, device="cuda")
zmin = torch.as_tensor(zc - 0.05, device="cuda")
x0 = torch.zeros((B, 2, 3), dtype=torch.float64, device="cuda")
L = p.rollout_launcher(zmax, zmin, x0)
for _ in range(20):
    L()
torch.cuda.synchronize()
print("ok")
