#!/usr/bin/env python3
"""Where in the horizon the strict working set lives (CPU, oracle): per solve the number of
active slots and the last active slot, over a few config-3 walks.  Design input for the strict
kernel's free-tail path; diagnostics only.

usage: python scripts/strict_active_stats.py [walks] [F_ext]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd")]

from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.generators import CoPGenerator  # noqa: E402
from oracle import zmp_oracle as O  # noqa: E402

DEFAULT_JSON = dict(ssp_duration=0.24, dsp_duration=0.03, standing_duration=1.0, distance=2.1,
                    step_length=0.3, foot_spread=0.1, horizon=150, Q=1.0, R=1e-6, S=1.0, h=0.75,
                    g=9.81, m=40.0, F_ext=400.0, strict=True, add_force=True)


def main():
    walks = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    fmax = float(sys.argv[2]) if len(sys.argv) > 2 else 800.0
    cfg = MPCConfig(**DEFAULT_JSON)
    zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory()
    n, N = len(zmax), cfg.horizon
    rng = np.random.default_rng(20251226)
    A, Bv, _ = O.lipm(cfg.dt, cfg.h, cfg.g)
    H, V, Px, Pu = O.strict_matrices(N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R)
    last = np.full((walks, 2, n - 1), -1)
    cnt = np.zeros((walks, 2, n - 1), int)
    for w in range(walks):
        off = rng.uniform(-0.02, 0.02, 2)
        F = rng.uniform(0.0, fmax)
        zx = O._extend(zmax + off, N)
        zn = O._extend(zmin + off, N)
        st = [np.zeros(3), np.zeros(3)]
        st[0][0], st[1][0] = rng.uniform(-0.01, 0.01, 2)
        Ws = [None, None]
        for i in range(n - 1):
            for a in range(2):
                hi, lo = zx[i + 1:i + 1 + N, a], zn[i + 1:i + 1 + N, a]
                W0 = None if Ws[a] is None else np.concatenate([Ws[a][1:], Ws[a][-1:]])
                u0, W, _, _ = O.strict_u0(st[a], hi, lo, H, Px, Pu[0, 0], cfg.Q, W0)
                Ws[a] = W
                act = np.nonzero(W)[0]
                cnt[w, a, i] = len(act)
                last[w, a, i] = act.max() if len(act) else -1
                st[a] = A @ st[a] + Bv[:, 0] * u0
            if i == n // 2:
                st[1] = st[1] - np.array([0.0, cfg.dt * F / cfg.m, 0.0])
        print(f"walk {w}: F={F:.0f} mean active {cnt[w].mean():.1f}, "
              f"solves with any active {np.mean(last[w] >= 0):.2f}, "
              f"mean last+1 {np.mean(last[w] + 1):.1f}", flush=True)
    l1 = last + 1
    print("per axis mean active:", cnt.mean(axis=(0, 2)))
    print("per axis mean (last active slot + 1):", l1.mean(axis=(0, 2)))
    # a wave = the max over its lanes at the same timestep (walks of one axis)
    print("per axis mean over timesteps of max over walks of (last+1):",
          l1.max(axis=0).mean(axis=1))
    for a in range(2):
        hist = np.percentile(l1[:, a, :], [50, 75, 90, 99, 100])
        print(f"axis {a} (last+1) percentiles 50/75/90/99/100:", hist)
    # by time: fraction of solves with an active slot, 20-step bins
    frac = (last >= 0).mean(axis=0)
    for a in range(2):
        print(f"axis {a} active fraction per 20 steps:",
              " ".join(f"{v:.2f}" for v in frac[a].reshape(-1)[:(n - 1) // 20 * 20]
                       .reshape(-1, 20).mean(axis=1)))


if __name__ == "__main__":
    main()
