#!/usr/bin/env python3
"""Strict-path fixtures from the CPU ORACLE (not from the reference).

The reference's strict branch (zmp_controller.py:173-195) needs cvxpy + OSQP, which are not
installed in this container (no network): parity with OSQP is UNPINNED.  These fixtures hold
the exact, KKT-certified box-QP solutions of the same problems (oracle/zmp_oracle.py
rollout_strict / strict_step_batch), so the device solver can be checked against them without
re-running the (slow, pure NumPy) oracle on the GPU box.

Usage: python tests/golden/make_strict_golden.py          → strict_oracle.npz
       python tests/golden/make_strict_golden.py --long   → strict_long_oracle.npz (horizons
       the LQ kernel runs with 4, 2 and 1 waves per workgroup, and the Cholesky kernel's
       320 < N <= 512 range)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import zmp_oracle as O  # noqa: E402

H_, G_, Q_, R_, M_ = 0.75, 9.81, 1.0, 1e-6, 40.0


def walk(N):
    d = np.load(os.path.join(HERE, f"walk_n{N}.npz"))
    return d["zmax"], d["zmin"], float(d["dt"])


def main():
    out = {}
    for N in (64, 150):
        zx, zn, dt = walk(N)
        n = len(zx)
        out[f"n{N}_zmax"], out[f"n{N}_zmin"] = zx, zn
        for F in (0.0, 400.0, 800.0):
            hist, worst = O.rollout_strict(np.zeros(3), np.zeros(3), zx, zn, N, dt, H_, G_, Q_, R_,
                                           kick=dt * F / M_, kick_step=n // 2, return_kkt=True)
            assert worst["primal"] <= 1e-13 and worst["stationarity"] < 1e-10, worst
            out[f"n{N}_F{int(F)}_hist"] = hist
            print(f"N={N} F={F}: kkt {worst}")
        # a non-zero initial state, no force
        x0 = np.array([0.01, 0.05, -0.4])
        y0 = np.array([-0.02, 0.1, 1.5])
        out[f"n{N}_x0"], out[f"n{N}_y0"] = x0, y0
        out[f"n{N}_x0_hist"] = O.rollout_strict(x0, y0, zx, zn, N, dt, H_, G_, Q_, R_)
    # cold-start single solves with heavily active bounds
    rng = np.random.default_rng(20251226)
    for N in (16, 64, 150):
        dt = 1.5 / N
        B = 48
        x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                      rng.uniform(-6, 6, B)], 1)
        ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(rng.normal(0, 0.003, (B, N)), 1)
        zmax = ctr + rng.uniform(0.005, 0.06, (B, N))
        zmin = ctr - rng.uniform(0.005, 0.06, (B, N))
        out[f"step{N}_x"], out[f"step{N}_zmax"], out[f"step{N}_zmin"] = x, zmax, zmin
        out[f"step{N}_out"] = O.strict_step_batch(x, zmax, zmin, N, dt, H_, G_, Q_, R_)
        print(f"step N={N}: {B} cases")
    np.savez_compressed(os.path.join(HERE, "strict_oracle.npz"), **out)


def main_long():
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)),
                                    "model-predictive-control-for-bipedal-locomotion_amd"))
    from mpc_bipedal.config import MPCConfig
    from mpc_bipedal.generators import CoPGenerator
    out = {}
    # N = 400: 300 samples of the default walk's stepping phase, started at rest at the CoP
    # centre, 800 N kick at the middle (heavily active y bounds)
    N = 400
    cfg = MPCConfig(horizon=N)
    zmax, zmin = CoPGenerator(cfg).generate_cop_trajectory()[:2]
    zx, zn = zmax[100:400].copy(), zmin[100:400].copy()
    n = len(zx)
    mid = (zx[0] + zn[0]) / 2
    x0 = np.array([mid[0], 0.0, 0.0])
    y0 = np.array([mid[1], 0.0, 0.0])
    kick = cfg.dt * 800.0 / M_
    hist, worst = O.rollout_strict(x0, y0, zx, zn, N, cfg.dt, H_, G_, Q_, R_, kick=kick,
                                   kick_step=n // 2, return_kkt=True)
    assert worst["primal"] <= 1e-13 and worst["stationarity"] < 1e-10, worst
    out.update(n400_zmax=zx, n400_zmin=zn, n400_x0=x0, n400_y0=y0, n400_kick=kick,
               n400_hist=hist)
    print(f"rollout N={N}, n={n}: kkt {worst}")
    rng = np.random.default_rng(20251227)
    for N, B in ((400, 16), (700, 8), (1300, 4)):
        dt = 1.5 / N
        x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                      rng.uniform(-6, 6, B)], 1)
        ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(rng.normal(0, 0.003 * np.sqrt(150 / N),
                                                                      (B, N)), 1)
        zmax_w = ctr + rng.uniform(0.005, 0.06, (B, N))
        zmin_w = ctr - rng.uniform(0.005, 0.06, (B, N))
        out[f"step{N}_x"], out[f"step{N}_zmax"], out[f"step{N}_zmin"] = x, zmax_w, zmin_w
        out[f"step{N}_out"] = O.strict_step_batch(x, zmax_w, zmin_w, N, dt, H_, G_, Q_, R_)
        print(f"step N={N}: {B} cases")
    np.savez_compressed(os.path.join(HERE, "strict_long_oracle.npz"), **out)


if __name__ == "__main__":
    if "--long" in sys.argv:
        main_long()
    else:
        main()
