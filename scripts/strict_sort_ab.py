"""A/B: strict rollout time and active-set work with the walks in input order vs grouped by
kick (F_ext) magnitude, config 3 (per-walk bounds) and config 4 (shared CoP).  Prints one JSON
line per case.  Diagnostic only."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd")):
    sys.path.insert(0, p)
from bench import DEFAULT_JSON, make_batch  # noqa: E402
from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402

cfg = MPCConfig(**dict(DEFAULT_JSON))
p = Plan(0, cfg.horizon, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, True)
cases = [(3, 65536, False), (4, 125000, True)]
if len(sys.argv) > 1:
    cases = [c for c in cases if str(c[0]) in sys.argv[1].split(",")]
for conf, B, shared in cases:
    _, _, zmax, zmin, x0, F = make_batch(B, 0, cfg, shared)
    n = zmax.shape[-2]
    for order in ("input", "sorted"):
        idx = np.argsort(F, kind="stable") if order == "sorted" else np.arange(B)
        zx = zmax if shared else zmax[idx]
        zn = zmin if shared else zmin[idx]
        L = p.rollout_launcher(torch.as_tensor(np.ascontiguousarray(zx), device="cuda"),
                               torch.as_tensor(np.ascontiguousarray(zn), device="cuda"),
                               torch.as_tensor(np.ascontiguousarray(x0[idx]), device="cuda"),
                               kick=torch.as_tensor(cfg.dt * F[idx] / cfg.m, device="cuda"),
                               kick_step=n // 2)
        L()
        torch.cuda.synchronize()
        p.counters(reset=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        K = 2
        for _ in range(K):
            L()
        e1.record()
        torch.cuda.synchronize()
        c = p.counters()
        ms = e0.elapsed_time(e1) / K
        print(json.dumps({"config": conf, "B": B, "order": order, "ms": round(ms, 3),
                          "wave_passes": c["wave_passes"] // K,
                          "lane_eff": c["instance_passes"] / max(1, 64 * c["wave_passes"]),
                          "ws_slots_per_lane_pass": c["working_set_slots"] / max(1, c["instance_passes"]),
                          "status_max": int(L.status.max())}), flush=True)
