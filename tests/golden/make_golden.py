#!/usr/bin/env python3
"""Generate golden vectors for the Wieber ZMP-MPC hot path FROM THE REFERENCE ITSELF.

Runs only in the build container (the reference is mounted read-only at
/root/reference and never travels to the GPU box).  It imports the reference
package unchanged, with an empty ``cvxpy`` module injected because cvxpy/OSQP
are not installed here: the unconstrained NumPy branch
(`zmp_controller.py:196-198`) is then the exact reference code path.

Outputs (small .npz fixtures, data only) next to this script:

* ``cop_<tag>.npz``            CoPGenerator.generate_cop_trajectory  (cop_generator.py:34-115)
* ``walk_n<N>.npz``            generate_com_trajectory_wieber         (zmp_controller.py:59-108)
                               generate_state_trajectory_wieber       (zmp_controller.py:110-147)
* ``predict_n<N>.npz``         predict_wieber_axis single calls       (zmp_controller.py:149-201)
                               + the Px / Pu / inv(M) the reference built inside those calls
                               (captured by wrapping the module's ``np`` namespace; the
                               reference arithmetic is untouched)

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--skip-512-walk]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 20251226


def _import_reference():
    sys.dont_write_bytecode = True
    sys.modules.setdefault("cvxpy", types.ModuleType("cvxpy"))
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.generators import CoPGenerator
    from src.mpc_bipedal.controllers import ZMPController
    from src.mpc_bipedal.controllers import zmp_controller as zc
    return MPCConfig, CoPGenerator, ZMPController, zc


class _NpSpy:
    """Proxy for the reference module's ``np`` that records what it builds.

    ``np.zeros`` calls made by predict_wieber_axis return the Px / Pu arrays the
    reference then fills in place (zmp_controller.py:162-171), and
    ``np.linalg.inv`` records M and inv(M) (zmp_controller.py:198).
    """

    def __init__(self, real):
        self._real = real
        self.zeros_log = []
        self.inv_log = []
        spy = self

        class _Linalg:
            def __getattr__(self, name):
                return getattr(real.linalg, name)

            @staticmethod
            def inv(a):
                r = real.linalg.inv(a)
                spy.inv_log.append((np.array(a), np.array(r)))
                return r

        self.linalg = _Linalg()

    def zeros(self, *a, **k):
        arr = self._real.zeros(*a, **k)
        self.zeros_log.append(arr)
        return arr

    def __getattr__(self, name):
        return getattr(self._real, name)


STATE_CODE = {"STANDING": 0, "DOUBLE_SUPPORT": 1, "SINGLE_SUPPORT": 2}


def default_mpc_dict():
    with open(os.path.join(REF, "configs", "default.json")) as f:
        return json.load(f)["mpc"]


def gen_cop(MPCConfig, CoPGenerator):
    """CoP bounds for several horizons / walk parameters (input producer, §8f row 1)."""
    cases = {
        "default_n150": dict(),
        "default_n10": dict(horizon=10),
        "default_n64": dict(horizon=64),
        "default_n512": dict(horizon=512),
        "classdefaults_n150": None,  # MPCConfig() with class defaults
        "long_n100": dict(horizon=100, distance=3.0, step_length=0.4),
        "short_n200": dict(horizon=200, distance=0.5, step_length=0.25, ssp_duration=0.3,
                           dsp_duration=0.05, standing_duration=0.4, foot_spread=0.12),
    }
    for tag, over in cases.items():
        if over is None:
            cfg = MPCConfig()
        else:
            d = default_mpc_dict()
            d.update(over)
            cfg = MPCConfig(**d)
        zmax, zmin, states = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
        np.savez_compressed(
            os.path.join(OUT, f"cop_{tag}.npz"),
            zmax=zmax, zmin=zmin,
            states=np.array([STATE_CODE[s.value] for s in states], dtype=np.int8),
            dt=cfg.dt, horizon=cfg.horizon, distance=cfg.distance, step_length=cfg.step_length,
            foot_spread=cfg.foot_spread, ssp_duration=cfg.ssp_duration,
            dsp_duration=cfg.dsp_duration, standing_duration=cfg.standing_duration)
        print(f"cop_{tag}: n={len(zmax)}")


def gen_walk(MPCConfig, CoPGenerator, ZMPController, horizon, full=True):
    d = default_mpc_dict()
    d["horizon"] = horizon
    d["strict"] = False  # strict branch needs cvxpy/OSQP (absent here): SURVEY §8c
    out = {}
    for add_force in ((True, False) if full else (True,)):
        d["add_force"] = add_force
        cfg = MPCConfig(**d)
        zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
        ctrl = ZMPController(cfg)
        x0 = np.zeros((3, 1))
        y0 = np.zeros((3, 1))
        with contextlib.redirect_stdout(io.StringIO()):
            com, y_hist = ctrl.generate_com_trajectory(x0, y0, zmax, zmin)
        tag = "force" if add_force else "noforce"
        out[f"com_{tag}"] = com
        out[f"y_hist_{tag}"] = y_hist
        out["zmax"], out["zmin"] = zmax, zmin
        if add_force:
            # ZMP estimate as run_mpc.py:294 computes it
            out["zmp_y_force"] = np.tensordot(y_hist[:, :, 0], ctrl.C, axes=([1], [0]))
    ctrl = ZMPController(cfg)
    xs, ys = ctrl.generate_state_trajectory_wieber(np.zeros((3, 1)), np.zeros((3, 1)),
                                                   out["zmax"], out["zmin"])
    out["state_x_hist"], out["state_y_hist"] = xs, ys
    if not full:
        out.update(dt=cfg.dt, horizon=cfg.horizon, h=cfg.h, g=cfg.g, Q=cfg.Q, R=cfg.R,
                   F_ext=cfg.F_ext, m=cfg.m)
        np.savez_compressed(os.path.join(OUT, f"walk_n{horizon}.npz"), **out)
        print(f"walk_n{horizon}: n={len(out['zmax'])}")
        return
    # a non-zero initial state, no force (state variant)
    x0 = np.array([[0.01], [0.02], [-0.1]])
    y0 = np.array([[-0.005], [0.0], [0.3]])
    xs, ys = ctrl.generate_state_trajectory_wieber(x0, y0, out["zmax"], out["zmin"])
    out["state_x_hist_x0"], out["state_y_hist_x0"] = xs, ys
    out["state_x0"], out["state_y0"] = x0, y0
    out.update(dt=cfg.dt, horizon=cfg.horizon, h=cfg.h, g=cfg.g, Q=cfg.Q, R=cfg.R,
               F_ext=cfg.F_ext, m=cfg.m)
    np.savez_compressed(os.path.join(OUT, f"walk_n{horizon}.npz"), **out)
    print(f"walk_n{horizon}: n={len(out['zmax'])}")


def gen_predict(MPCConfig, ZMPController, zc, N, ncases=64, nparam=16):
    """Single predict_wieber_axis calls + the matrices the reference built inside them."""
    rng = np.random.default_rng(SEED + N)
    real_np = zc.np
    spy = _NpSpy(real_np)
    zc.np = spy
    try:
        rows = []
        for c in range(ncases + nparam):
            if c < ncases:
                params = dict(horizon=N, Q=1.0, R=1e-6, h=0.75, g=9.81)
            else:
                params = dict(horizon=N, Q=float(rng.uniform(0.5, 2.0)),
                              R=float(10 ** rng.uniform(-7, -4)),
                              h=float(rng.uniform(0.6, 1.0)), g=9.81)
            cfg = MPCConfig(strict=False, **params)
            ctrl = ZMPController(cfg)
            x = np.array([[rng.uniform(-0.05, 0.05)], [rng.uniform(-0.3, 0.3)],
                          [rng.uniform(-3.0, 3.0)]])
            centre = rng.uniform(-0.15, 0.15) + np.cumsum(rng.normal(0, 0.004, N))
            half = rng.uniform(0.02, 0.1, N)
            zmax = (centre + half).reshape(N, 1)
            zmin = (centre - half).reshape(N, 1)
            spy.zeros_log.clear()
            spy.inv_log.clear()
            res = ctrl.predict_wieber_axis(x, N, zmax, zmin)
            Px, Pu = spy.zeros_log[0], spy.zeros_log[1]
            M, Minv = spy.inv_log[0]
            rows.append(dict(x=x, zmax=zmax, zmin=zmin, out=res, Q=params["Q"], R=params["R"],
                             h=params["h"], g=params["g"], dt=cfg.dt, Px=Px, Pu=Pu, M=M,
                             Minv=Minv))
    finally:
        zc.np = real_np
    first = rows[0]
    k = (first["Minv"] @ first["Pu"].T)[0, :]
    payload = dict(
        N=N, dt=first["dt"],
        x=np.stack([r["x"] for r in rows]), zmax=np.stack([r["zmax"] for r in rows]),
        zmin=np.stack([r["zmin"] for r in rows]), out=np.stack([r["out"] for r in rows]),
        Q=np.array([r["Q"] for r in rows]), R=np.array([r["R"] for r in rows]),
        h=np.array([r["h"] for r in rows]), g=np.array([r["g"] for r in rows]),
        Px=first["Px"], gain_k=k, gain_kPx=k @ first["Px"],
    )
    Pu = first["Pu"]
    # Pu is lower-triangular Toeplitz (zmp_controller.py:170-171): keep its first column, and
    # the whole matrix only where it is small.
    assert np.array_equal(np.triu(Pu, 1), np.zeros_like(Pu))
    for i in range(N):
        assert np.array_equal(np.diag(Pu, -i), np.full(N - i, Pu[i, 0]))
    payload["Pu_col0"] = Pu[:, 0].copy()
    if N <= 150:
        payload["Pu"] = Pu
        payload["Minv"] = first["Minv"]
    np.savez_compressed(os.path.join(OUT, f"predict_n{N}.npz"), **payload)
    print(f"predict_n{N}: {len(rows)} cases")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-512-walk", action="store_true")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    MPCConfig, CoPGenerator, ZMPController, zc = _import_reference()
    only = set(a.only.split(",")) if a.only else None
    if not only or "cop" in only:
        gen_cop(MPCConfig, CoPGenerator)
    if not only or "predict" in only:
        for N in (10, 64, 150, 512):
            gen_predict(MPCConfig, ZMPController, zc, N)
    if not only or "walk" in only:
        gen_walk(MPCConfig, CoPGenerator, ZMPController, 150)
        gen_walk(MPCConfig, CoPGenerator, ZMPController, 10)
        gen_walk(MPCConfig, CoPGenerator, ZMPController, 64)
    if (not only or "walk512" in only) and not a.skip_512_walk:
        gen_walk(MPCConfig, CoPGenerator, ZMPController, 512, full=False)


if __name__ == "__main__":
    main()
