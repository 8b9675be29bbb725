"""Diagnostic: per-workgroup timeline of the persistent config-2 kernel (ZMPC_PERS_TRACE).
Runs the launch a few times in a child per environment and keeps the last launch's trace
(grid x 8 u64: HW_ID, XCC_ID, realtime0, memtime0, memtime after walk 0..3).

usage: python scripts/pers_trace.py OUTDIR '[{}, {"ZMPC_DEBUG_ROLLOUT": "12"}]' [B]
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import sys, os, numpy as np, torch
sys.path.insert(0, os.environ["PKG"])
from mpc_bipedal.solver import Plan
B = int(sys.argv[1]); N = 150; n = 420
p = Plan(0, N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, False)
rng = np.random.default_rng(0)
zc = np.cumsum(rng.normal(0, 0.01, (B, n, 2)), 1)
zmax = torch.as_tensor(zc + 0.05, device="cuda"); zmin = torch.as_tensor(zc - 0.05, device="cuda")
x0 = torch.as_tensor(rng.uniform(-0.01, 0.01, (B, 2, 3)), device="cuda")
kick = torch.as_tensor(rng.uniform(0, 0.1, B), device="cuda")
L = p.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=n // 2)
for _ in range(5): L()
torch.cuda.synchronize()
print("ok")
'''

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = sys.argv[1]
os.makedirs(out, exist_ok=True)
variants = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
B = sys.argv[3] if len(sys.argv) > 3 else "4096"
for i, var in enumerate(variants):
    env = dict(os.environ, PKG=os.path.join(root, "model-predictive-control-for-bipedal-locomotion_amd"),
               ZMPC_PERS_TRACE=os.path.join(out, f"trace{i}.bin"), **{k: str(v) for k, v in var.items()})
    r = subprocess.run([sys.executable, "-c", CHILD, B], env=env, capture_output=True, text=True,
                       timeout=120)
    print(i, var, r.stdout.strip(), r.stderr[-300:] if r.returncode else "", flush=True)
