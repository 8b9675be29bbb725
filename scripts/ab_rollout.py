"""Diagnostic A/B of the unconstrained rollout kernels: median HIP-event time of one launch per
(environment, batch shape).  Each configuration runs in a child process (the kernel-choice
environment variables are read once per process).

usage: python scripts/ab_rollout.py '[{"ZMPC_ROLLOUT_VARIANT": "8"}, {"ZMPC_PIPE_G": "4"}]' \
           '[[4096, 150, 420], [16384, 150, 420]]'
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, os, json, numpy as np, torch
sys.path.insert(0, os.environ["PKG"])
from mpc_bipedal.solver import Plan
B = int(sys.argv[1]); N = int(sys.argv[2]); n = int(sys.argv[3])
p = Plan(0, N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, False)
rng = np.random.default_rng(0)
zc = np.cumsum(rng.normal(0, 0.01, (B, n, 2)), 1)
zmax = torch.as_tensor(zc + 0.05, device="cuda"); zmin = torch.as_tensor(zc - 0.05, device="cuda")
x0 = torch.as_tensor(rng.uniform(-0.01, 0.01, (B, 2, 3)), device="cuda")
kick = torch.as_tensor(rng.uniform(0, 0.1, B), device="cuda")
L = p.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=n // 2)
for _ in range(3): L()
torch.cuda.synchronize()
h = L.hist.clone() if hasattr(L, "hist") else None
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
for a, b in ev:
    a.record(); L(); b.record()
torch.cuda.synchronize()
out = dict(B=B, N=N, n=n, us=float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
if h is not None:
    out["hist_sum"] = float(h.sum())
print(json.dumps(out))
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
env0 = dict(os.environ, PKG=os.path.join(root, "model-predictive-control-for-bipedal-locomotion_amd"))
variants = json.loads(sys.argv[1]) if len(sys.argv) > 1 else [{}]
shapes = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [[4096, 150, 420]]
for B, N, n in shapes:
    for var in variants:
        env = dict(env0, **{k: str(v) for k, v in var.items()})
        r = subprocess.run([sys.executable, "-c", CHILD, str(B), str(N), str(n)], env=env,
                           capture_output=True, text=True, timeout=120)
        line = r.stdout.strip()
        if line:
            rec = json.loads(line)
            rec["env"] = var
            print(json.dumps(rec), flush=True)
        else:
            print(json.dumps(dict(B=B, N=N, n=n, env=var, error=r.stderr[-600:])), flush=True)
