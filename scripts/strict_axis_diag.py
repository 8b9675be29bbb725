"""Diagnostic: config-3 strict rollouts timed with both axes, with the x waves
exiting at once (ZMPC_DEBUG_LQ=2: each SIMD's y wave runs alone) and with the y waves exiting
(=4).  If y alone is about as slow as both, the x waves' instructions fill the y waves' stalls
(latency-bound single wave); if it is much faster, the SIMD is issue-bound.
usage: python scripts/strict_axis_diag.py [B] [dbg,dbg,...]"""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json, numpy as np, torch
sys.path[:0] = [os.environ["ROOT"], os.environ["PKG"]]
from bench import DEFAULT_JSON, make_batch
from mpc_bipedal.config import MPCConfig
from mpc_bipedal.solver import Plan
B = int(sys.argv[1])
cfg = MPCConfig(**dict(DEFAULT_JSON))
_, _, zmax, zmin, x0, F = make_batch(B, 0, cfg, False)
n = zmax.shape[1]
p = Plan(0, cfg.horizon, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, True)
L = p.rollout_launcher(torch.as_tensor(zmax, device="cuda"), torch.as_tensor(zmin, device="cuda"),
                       torch.as_tensor(x0, device="cuda"),
                       kick=torch.as_tensor(cfg.dt * F / cfg.m, device="cuda"), kick_step=n // 2)
L(); torch.cuda.synchronize()
ms = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); L(); b.record(); torch.cuda.synchronize(); ms.append(a.elapsed_time(b))
print(json.dumps(dict(B=B, dbg=os.environ.get("ZMPC_DEBUG_LQ", "0"), ms=sorted(ms)[1],
                      counters=p.counters())))
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
env0 = dict(os.environ, ROOT=root,
            PKG=os.path.join(root, "model-predictive-control-for-bipedal-locomotion_amd"))
B = sys.argv[1] if len(sys.argv) > 1 else "65536"
for d in (sys.argv[2] if len(sys.argv) > 2 else "0,2,4,0").split(","):
    r = subprocess.run([sys.executable, "-c", CHILD, B], env=dict(env0, ZMPC_DEBUG_LQ=d),
                       capture_output=True, text=True, timeout=300)
    print(r.stdout.strip() or r.stderr[-800:], flush=True)
