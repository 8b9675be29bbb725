"""Diagnostic: config-2 rollouts back to back on one stream vs alternating two streams
(separate history buffers) — how much of the per-step time is launch gap / tail."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd")):
    sys.path.insert(0, p)
from bench import DEFAULT_JSON, make_batch  # noqa: E402
from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402

B = 4096
cfg = MPCConfig(**dict(DEFAULT_JSON, strict=False))
_, _, zmax, zmin, x0, F = make_batch(B, 0, cfg, False)
n = zmax.shape[1]
p = Plan(0, cfg.horizon, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, False)
d = lambda a: torch.as_tensor(a, device="cuda")
zx, zn, xx, kk = d(zmax), d(zmin), d(x0), d(cfg.dt * F / cfg.m)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
Ls = []
for s in streams:
    with torch.cuda.stream(s):
        Ls.append(p.rollout_launcher(zx, zn, xx, kick=kk, kick_step=n // 2))
K = 200
for ns in (1, 2):
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            s = streams[k % ns]
            with torch.cuda.stream(s):
                Ls[k % ns]()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
    print(f"streams={ns}: {dt * 1e6:.1f} us/step, {B * (n - 1) * 2 / dt:.3e} solves/s")
