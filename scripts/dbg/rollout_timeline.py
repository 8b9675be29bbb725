"""Diagnostic: per-walk phase timeline of the unconstrained split kernel, or of the wide kernel
for walks of more than 513 samples (diagnostics build,
ZMPC_ROLLOUT_TL): each walk's wave 0 stamps the 100 MHz constant clock at its start, once its
bounds are in LDS, after the correlation, after the staged history and after issuing the copy-out.
Prints the mean phase durations per dispatch round and a chip-wide occupancy profile (walks in
each phase per 0.5 us bin).  Usage (GPU box):
  ZMPC_LIB=.../libzmpc_diag.so python scripts/dbg/rollout_timeline.py [B] [N]"""
import json
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd"))
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
N = int(sys.argv[2]) if len(sys.argv) > 2 else 150
path = os.path.join(tempfile.gettempdir(), f"zmpc_tl_{os.getpid()}.bin")
os.environ["ZMPC_ROLLOUT_TL"] = path
from bench import DEFAULT_JSON, make_batch  # noqa: E402
from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402

cfg = MPCConfig(**dict(DEFAULT_JSON, horizon=N, strict=False))
_, _, zx, zn, x0, F = make_batch(B, 0, cfg, False)
n = zx.shape[1]
p = Plan(0, N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, False)
dev = torch.device("cuda", 0)
L = p.rollout_launcher(torch.as_tensor(zx, device=dev), torch.as_tensor(zn, device=dev),
                       torch.as_tensor(x0, device=dev),
                       kick=torch.as_tensor(cfg.dt * F / cfg.m, device=dev), kick_step=n // 2)
for _ in range(6):
    L()
torch.cuda.synchronize()
t = np.fromfile(path, np.uint64).reshape(B, 5).astype(np.float64) * 0.01  # us (100 MHz)
os.remove(path)
t -= t[:, 0].min()
dur = np.diff(t, axis=1)
start = t[:, 0]
# dispatch rounds: a walk that starts after the first walk to end is a later round
first_end = t[:, 4].min()
rnd = (start > first_end).astype(int)
split = n - 1 <= 512
out = {"B": B, "N": N, "n": n, "span_us": float(t[:, 4].max()),
       "phases": ["load+stage", "correlation", "scan+replay", "copy-out issue"] if split else
       ["load+stage", "correlation", "scan+chain", "replay+copy-out rounds"]}
for r in (0, 1):
    m = rnd == r
    if m.any():
        out[f"round{r}"] = {"walks": int(m.sum()),
                            "start_us": [float(start[m].min()), float(np.median(start[m])),
                                         float(start[m].max())],
                            "end_us": [float(t[m, 4].min()), float(np.median(t[m, 4])),
                                       float(t[m, 4].max())],
                            "mean_phase_us": [float(v) for v in dur[m].mean(axis=0)]}
print(json.dumps(out), flush=True)
bins = np.arange(0.0, t[:, 4].max() + 0.5, 0.5)
for b0 in bins:
    c = [int(((t[:, k] <= b0) & (t[:, k + 1] > b0)).sum()) for k in range(4)]
    print(f"{b0:6.1f} us  load {c[0]:5d}  corr {c[1]:5d}  scan/replay {c[2]:5d}  copy {c[3]:5d}")
