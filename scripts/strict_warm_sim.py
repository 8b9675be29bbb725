#!/usr/bin/env python3
"""CPU simulation of the strict LQ kernel's primal-dual active-set iteration (strict_lq.hip:
release wrong-signed multipliers, add violated free slots, stop when the set repeats) on the
y axis of the reference's default walk at F_ext = 0 / 400 / 800 N, to compare warm starts by
the passes per solve they need.  Diagnostics only (design input for DESIGN.md §4.3).

Warm starts (W = the previous timestep's converged set, N slots):
  b  shifted one slot, slot N−1 copies the old terminal slot (round-2/3 kernel)
  a  as b, slot N−1 free
  c  as b, slots N−2 and N−1 free
  d  as b, slot N−2 (the old terminal slot) free   — the kernel's default since round 3
  f  as b, slot N−2 takes the old slot N−2
  g  as d, slot N−3 free too
  h  as d, slot N−1 takes the old slot N−2
Measured here: b 1.387, a 1.495, c 1.517, d 1.310, f 1.325, g 1.325, h 1.531 passes per solve.

usage: python scripts/strict_warm_sim.py [modes, default "b,d"]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd")]

from oracle import zmp_oracle as O  # noqa: E402

TOL = 1e-13  # strict_lq.hip: primal tolerance and tolnu (Q = 1)


def pdas(H, q, lo, hi, W, maxit=64):
    """The kernel's iteration in z-space (same iterates; EQP by dense solves)."""
    for passes in range(1, maxit + 1):
        F = W == 0
        z = np.where(W == 1, hi, np.where(W == 2, lo, 0.0))
        if F.any():
            z[F] = np.linalg.solve(H[np.ix_(F, F)], -q[F] - H[np.ix_(F, ~F)] @ z[~F])
        nu = -(H @ z + q)
        Wn = W.copy()
        Wn[(W == 1) & (nu < -TOL)] = 0
        Wn[(W == 2) & (nu > TOL)] = 0
        Wn[F & (z > hi + TOL)] = 1
        Wn[F & (z < lo - TOL)] = 2
        if np.array_equal(Wn, W):
            return z, W, passes
        W = Wn
    return z, W, maxit


def warm(W, mode):
    W0 = np.concatenate([W[1:], W[-1:]])
    if mode in ("a", "c"):
        W0[-1] = 0
    if mode in ("c", "d"):
        W0[-2] = 0
    if mode == "f":
        W0[-2] = W[-2]
    if mode == "g":  # d, and slot N−3 free too
        W0[-2] = W0[-3] = 0
    if mode == "h":  # d, slot N−1 takes the old pre-terminal slot
        W0[-2], W0[-1] = 0, W[-2]
    return W0


def run(mode):
    d = np.load(os.path.join(ROOT, "tests", "golden", "walk_n150.npz"))
    N, dt, h, g, Q, R, m = 150, float(d["dt"]), 0.75, 9.81, 1.0, 1e-6, 40.0
    H, _, Px, Pu = O.strict_matrices(N, dt, h, g, Q, R)
    p0 = Pu[0, 0]
    A, Bv, _ = O.lipm(dt, h, g)
    zx, zn = O._extend(d["zmax"], N), O._extend(d["zmin"], N)
    n = len(d["zmax"])
    hist = {}
    for F_ext in (0.0, 400.0, 800.0):
        st, W = np.zeros(3), np.zeros(N, np.int8)
        for i in range(n - 1):
            hi, lo = zx[i + 1:i + 1 + N, 1], zn[i + 1:i + 1 + N, 1]
            c = Px @ st
            q = -Q * (hi + lo) / 2 - (H @ c - Q * c)
            z, W, p = pdas(H, q, lo, hi, warm(W, mode))
            hist[p] = hist.get(p, 0) + 1
            st = A @ st + Bv[:, 0] * (z[0] - c[0]) / p0
            if i == n // 2:
                st[1] -= dt * F_ext / m
    tot = sum(k * v for k, v in hist.items())
    print(f"{mode}: passes histogram {dict(sorted(hist.items()))}, "
          f"{tot / sum(hist.values()):.4f} passes per solve", flush=True)


if __name__ == "__main__":
    for mode in (sys.argv[1] if len(sys.argv) > 1 else "b,d").split(","):
        run(mode)
