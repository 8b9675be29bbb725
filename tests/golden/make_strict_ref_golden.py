#!/usr/bin/env python3
"""Strict-path golden vectors from the REFERENCE's own strict branch (this container only).

The reference's strict solve (zmp_controller.py:173-195) builds its QP in NumPy — H = R·I,
A_ineq = [Pu; −Pu], b_ineq = [z_max − Px x; −z_min + Px x], the objective
½Q‖Px x + Pu J − z_ref‖² + ½JᵀHJ — and hands it to cvxpy → OSQP.  cvxpy and OSQP are not
installed (no network; cvxpy is pinned only as cvxpy>=1.2.0, requirements.txt:2, OSQP not at
all), so the reference is imported with a RECORDING stand-in for the `cp` module (the
technique of make_herdt_golden.py): `cp.Variable`, `cp.sum_squares`, `cp.quad_form`,
`A @ J <= b`, `cp.Problem(...).solve()` record the problem exactly as the reference states
it, and `solve()` answers with the exact KKT point from oracle/zmp_oracle.py (solve_box_qp in
z = Px x + Pu J; J = Pu⁻¹(z − Px x) by forward substitution).  Parity with OSQP itself stays
unpinned (OSQP is a tolerance-based ADMM; the exact optimum is the point it approximates).

Everything else is the reference's code running unchanged with strict=True: the padding
(:81-88), the time loop (:93-104), the force kick (:105-106), the Px/Pu build (:162-171), the
problem assembly (:173-190), `J.value[0]` and the state advance (:195-201).

Checked here, at every captured QP:
* the oracle's z-space problem equals the captured J-space problem: the quadratic form
  ½Q·PuᵀPu + ½R·I, the linear term Q·Puᵀ(Px x − z_ref), A_ineq = [Pu; −Pu] and b_ineq — to
  ≤ 1e-13 relative (`max_rel_problem_diff`);
* the answer's KKT residuals (z-space box QP: primal, stationarity, multiplier signs);
* the reference-driven rollouts equal the oracle's own rollout_strict (`max_abs_vs_oracle`).

Saved (tests/golden/strict_ref.npz):
* n{64,150}_zmax/zmin: the reference CoPGenerator's default.json bounds at that horizon;
* n{N}_F{0,400,800}_com / _yhist: generate_com_trajectory(strict=True, add_force=F>0) from rest;
* n{N}_x0 / _y0 / _x0_xhist / _x0_yhist: generate_state_trajectory_wieber from a non-zero state;
* step{16,64,150}_x / _zmax / _zmin / _out: cold predict_wieber_axis calls with heavily active
  bounds (48 per horizon), out = the reference's returned state;
* max_rel_problem_diff, kkt_worst, max_abs_vs_oracle.

Usage: PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_strict_ref_golden.py          → strict_ref.npz
       PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_strict_ref_golden.py --long   → strict_long_ref.npz
       PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_strict_ref_golden.py --weights-long
                                                                    → strict_weights_long_ref.npz
"""
import contextlib
import io
import json
import os
import sys
import types

import numpy as np
from scipy.linalg import solve_triangular

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import zmp_oracle as O  # noqa: E402

REF = "/root/reference"


class _Rec:
    """What the stand-in records: the last predict_wieber_axis arguments, the warm-start
    working sets per axis, and per-QP diagnostics."""
    call = None          # (x_init, nb_steps, z_max, z_min, cfg)
    axis = 0             # 0 = x, 1 = y inside a rollout (calls alternate, :95-104)
    warm = [None, None]  # working sets of the previous timestep per axis (None = cold)
    rollout = False
    n_qp = 0
    max_rel = 0.0
    kkt = dict(primal=0.0, stationarity=0.0, dual_hi=0.0, dual_lo=0.0)
    mats = {}


class _Var:
    __array_ufunc__ = None  # `ndarray @ J` defers to __rmatmul__

    def __init__(self, n):
        self.n = n
        self.value = None

    def __rmatmul__(self, A):
        return _Aff(np.asarray(A, np.float64), np.zeros(np.asarray(A).shape[0]))


class _Aff:
    """A @ J + c."""
    __array_ufunc__ = None

    def __init__(self, A, c):
        self.A, self.c = A, np.asarray(c, np.float64).ravel()

    def __radd__(self, v):
        return _Aff(self.A, self.c + np.asarray(v, np.float64).ravel())

    __add__ = __radd__

    def __sub__(self, v):
        return _Aff(self.A, self.c - np.asarray(v, np.float64).ravel())

    def __le__(self, b):
        return ("le", self.A, np.asarray(b, np.float64).ravel() - self.c)


class _Quad:
    """Jᵀ P J + qᵀ J + r."""

    def __init__(self, P, q, r=0.0):
        self.P, self.q, self.r = P, q, r

    def __rmul__(self, s):
        s = float(s)
        return _Quad(s * self.P, s * self.q, s * self.r)

    def __add__(self, o):
        return _Quad(self.P + o.P, self.q + o.q, self.r + o.r)


def _sum_squares(a):
    return _Quad(a.A.T @ a.A, 2.0 * a.A.T @ a.c, float(a.c @ a.c))


def _quad_form(J, H):
    H = np.asarray(H, np.float64)
    return _Quad(H, np.zeros(H.shape[0]))


_VAR = [None]


def _variable(n):
    _VAR[0] = _Var(n)
    return _VAR[0]


def _oracle_mats(N, cfg):
    key = (N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R)
    if key not in _Rec.mats:
        _Rec.mats[key] = O.strict_matrices(N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R)
    return _Rec.mats[key]


class _Problem:
    def __init__(self, obj, cons):
        self.obj, self.cons = obj, cons

    def solve(self, **kw):
        assert kw.get("solver") == "OSQP"
        x, N, zmax, zmin, cfg = _Rec.call
        assert len(self.cons) == 1 and self.cons[0][0] == "le"
        _, G, h = self.cons[0]
        Hz, V, Px, Pu = _oracle_mats(N, cfg)
        c = (Px @ x).ravel()
        zx, zn = zmax.ravel(), zmin.ravel()
        z_ref = (zx + zn) / 2
        # the oracle's statement of the same problem, in the reference's J variables
        P_or = 0.5 * cfg.Q * (Pu.T @ Pu) + 0.5 * cfg.R * np.eye(N)
        q_or = cfg.Q * Pu.T @ (c - z_ref)
        G_or = np.vstack([Pu, -Pu])
        h_or = np.concatenate([zx - c, -zn + c])

        def rel(a, b):
            return float(np.abs(a - b).max() / max(1.0, np.abs(b).max()))
        d = max(rel(self.obj.P, P_or), rel(self.obj.q, q_or), rel(G, G_or), rel(h, h_or))
        _Rec.max_rel = max(_Rec.max_rel, d)
        # the exact answer (z-space box QP), warm-started as oracle.rollout_strict does
        a = _Rec.axis
        W = _Rec.warm[a]
        W0 = None if (W is None or not _Rec.rollout) else np.concatenate([W[1:], W[-1:]])
        u0, Wn, z, q = O.strict_u0(x.ravel(), zx, zn, Hz, Px, Pu[0, 0], cfg.Q, W0)
        if _Rec.rollout:
            _Rec.warm[a] = Wn
        r = O.kkt_check(Hz, q, z, zn, zx, scale=max(1.0, float(np.abs(q).max())))
        for k in _Rec.kkt:
            _Rec.kkt[k] = max(_Rec.kkt[k], r[k])
        J = solve_triangular(Pu, z - c, lower=True)
        assert J[0] == u0
        _VAR[0].value = J
        _Rec.n_qp += 1
        return 0.5 * float(J @ (2 * self.obj.P) @ J) + float(self.obj.q @ J) + self.obj.r


def make_cp():
    cp = types.ModuleType("cvxpy")
    cp.Variable = _variable
    cp.sum_squares = _sum_squares
    cp.quad_form = _quad_form
    cp.Minimize = lambda o: o
    cp.Problem = _Problem
    cp.OSQP = "OSQP"
    return cp


def default_mpc_dict():
    with open(os.path.join(REF, "configs", "default.json")) as f:
        return json.load(f)["mpc"]


def main():
    sys.modules["cvxpy"] = make_cp()
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.generators import CoPGenerator
    from src.mpc_bipedal.controllers import ZMPController

    def instrument(ctl):
        orig = ctl.predict_wieber_axis

        def record(x_init, nb_steps, z_max, z_min):
            _Rec.call = (np.array(x_init, np.float64), nb_steps, np.array(z_max), np.array(z_min),
                         ctl.config)
            out = orig(x_init, nb_steps, z_max, z_min)
            _Rec.axis ^= 1
            return out
        ctl.predict_wieber_axis = record
        return ctl

    def start_rollout():
        _Rec.rollout, _Rec.axis, _Rec.warm = True, 0, [None, None]

    out = {}
    dev = 0.0
    for N in (64, 150):
        d = default_mpc_dict()
        d.update(horizon=N, strict=True)
        cfg = MPCConfig(**d)
        zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
        n = len(zmax)
        out[f"n{N}_zmax"], out[f"n{N}_zmin"] = zmax, zmin
        for F in (0.0, 400.0, 800.0):
            d2 = dict(d, add_force=F > 0, F_ext=F)
            ctl = instrument(ZMPController(MPCConfig(**d2)))
            start_rollout()
            with contextlib.redirect_stdout(io.StringIO()), \
                    contextlib.redirect_stderr(io.StringIO()):
                com, y_hist = ctl.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                          zmax, zmin)
            out[f"n{N}_F{int(F)}_com"], out[f"n{N}_F{int(F)}_yhist"] = com, y_hist[:, :, 0]
            ref = O.rollout_strict(np.zeros(3), np.zeros(3), zmax, zmin, N, cfg.dt, cfg.h,
                                   cfg.g, cfg.Q, cfg.R, kick=cfg.dt * F / cfg.m,
                                   kick_step=n // 2)
            e = max(float(np.abs(ref[:, :, 0] - com).max()),
                    float(np.abs(ref[:, 1] - y_hist[:, :, 0]).max()))
            dev = max(dev, e)
            print(f"N={N} F={F:.0f}: reference-driven rollout vs oracle max |d| {e:.2e}, "
                  f"{_Rec.n_qp} QPs so far, max rel problem diff {_Rec.max_rel:.2e}")
        # generate_state_trajectory_wieber from a non-zero state (no kick, :110-147)
        x0 = np.array([[0.01], [0.05], [-0.4]])
        y0 = np.array([[-0.02], [0.1], [1.5]])
        ctl = instrument(ZMPController(cfg))
        start_rollout()
        with contextlib.redirect_stderr(io.StringIO()):
            xs, ys = ctl.generate_state_trajectory_wieber(x0, y0, zmax, zmin)
        out[f"n{N}_x0"], out[f"n{N}_y0"] = x0.ravel(), y0.ravel()
        out[f"n{N}_x0_xhist"], out[f"n{N}_x0_yhist"] = xs[:, :, 0], ys[:, :, 0]
        ref = O.rollout_strict(x0.ravel(), y0.ravel(), zmax, zmin, N, cfg.dt, cfg.h, cfg.g,
                               cfg.Q, cfg.R)
        e = max(float(np.abs(ref[:, 0] - xs[:, :, 0]).max()),
                float(np.abs(ref[:, 1] - ys[:, :, 0]).max()))
        dev = max(dev, e)
        print(f"N={N} x0: vs oracle max |d| {e:.2e}")
    # cold single predict_wieber_axis calls with heavily active bounds
    _Rec.rollout = False
    rng = np.random.default_rng(20251226)
    for N in (16, 64, 150):
        d = default_mpc_dict()
        d.update(horizon=N, strict=True)
        ctl = instrument(ZMPController(MPCConfig(**d)))
        B = 48
        x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                      rng.uniform(-6, 6, B)], 1)
        ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(rng.normal(0, 0.003, (B, N)), 1)
        zmax_w = ctr + rng.uniform(0.005, 0.06, (B, N))
        zmin_w = ctr - rng.uniform(0.005, 0.06, (B, N))
        res = np.stack([ctl.predict_wieber_axis(x[b].reshape(3, 1), N, zmax_w[b].reshape(N, 1),
                                                zmin_w[b].reshape(N, 1)).ravel()
                        for b in range(B)])
        ref = O.strict_step_batch(x, zmax_w, zmin_w, N, 1.5 / N, d["h"], d["g"], d["Q"],
                                  d["R"])
        e = float(np.abs(res - ref).max())
        dev = max(dev, e)
        out[f"step{N}_x"], out[f"step{N}_zmax"], out[f"step{N}_zmin"] = x, zmax_w, zmin_w
        out[f"step{N}_out"] = res
        print(f"step N={N}: {B} cold calls, vs oracle max |d| {e:.2e}")
    print(f"{_Rec.n_qp} captured QPs; max rel problem diff {_Rec.max_rel:.2e}; KKT {_Rec.kkt}")
    assert _Rec.max_rel <= 1e-13, _Rec.max_rel
    assert _Rec.kkt["primal"] <= 1e-13 and _Rec.kkt["stationarity"] <= 1e-10, _Rec.kkt
    assert _Rec.kkt["dual_hi"] <= 1e-10 and _Rec.kkt["dual_lo"] <= 1e-10, _Rec.kkt
    assert dev <= 1e-12, dev
    out["max_rel_problem_diff"] = _Rec.max_rel
    out["kkt_worst"] = np.array([_Rec.kkt[k] for k in ("primal", "stationarity", "dual_hi",
                                                         "dual_lo")])
    out["max_abs_vs_oracle"] = dev
    out["n_qps"] = _Rec.n_qp
    np.savez_compressed(os.path.join(HERE, "strict_ref.npz"), **out)
    print("saved", os.path.join(HERE, "strict_ref.npz"))


def main_long():
    """Long horizons (the LQ kernel's 4/2/1-wave workgroups, the Cholesky kernel's
    320 < N <= 512 range) → strict_long_ref.npz:
    * n400_*: 300 samples of the default walk's stepping phase (reference CoPGenerator at
      horizon 400, rows 100..399) from rest at the first CoP centre, generate_com_trajectory
      with an 800 N kick at n//2;
    * step{400,700,1300}_*: cold predict_wieber_axis calls with heavily active bounds."""
    sys.modules["cvxpy"] = make_cp()
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.generators import CoPGenerator
    from src.mpc_bipedal.controllers import ZMPController

    def instrument(ctl):
        orig = ctl.predict_wieber_axis

        def record(x_init, nb_steps, z_max, z_min):
            _Rec.call = (np.array(x_init, np.float64), nb_steps, np.array(z_max), np.array(z_min),
                         ctl.config)
            out = orig(x_init, nb_steps, z_max, z_min)
            _Rec.axis ^= 1
            return out
        ctl.predict_wieber_axis = record
        return ctl

    out = {}
    N = 400
    d = default_mpc_dict()
    d.update(horizon=N, strict=True, add_force=True, F_ext=800.0)
    cfg = MPCConfig(**d)
    zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
    zx, zn = zmax[100:400].copy(), zmin[100:400].copy()
    n = len(zx)
    mid = (zx[0] + zn[0]) / 2
    x0 = np.array([mid[0], 0.0, 0.0])
    y0 = np.array([mid[1], 0.0, 0.0])
    ctl = instrument(ZMPController(cfg))
    _Rec.rollout, _Rec.axis, _Rec.warm = True, 0, [None, None]
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        com, y_hist = ctl.generate_com_trajectory(x0.reshape(3, 1), y0.reshape(3, 1), zx, zn)
    kick = cfg.dt * cfg.F_ext / cfg.m
    ref = O.rollout_strict(x0, y0, zx, zn, N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, kick=kick,
                           kick_step=n // 2)
    dev = max(float(np.abs(ref[:, :, 0] - com).max()),
              float(np.abs(ref[:, 1] - y_hist[:, :, 0]).max()))
    print(f"rollout N={N}, n={n}: reference-driven vs oracle max |d| {dev:.2e}")
    out.update(n400_zmax=zx, n400_zmin=zn, n400_x0=x0, n400_y0=y0, n400_kick=kick,
               n400_com=com, n400_yhist=y_hist[:, :, 0])
    _Rec.rollout = False
    rng = np.random.default_rng(20251227)
    for N, B in ((400, 16), (700, 8), (1300, 4)):
        d = default_mpc_dict()
        d.update(horizon=N, strict=True)
        ctl = instrument(ZMPController(MPCConfig(**d)))
        x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                      rng.uniform(-6, 6, B)], 1)
        ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(
            rng.normal(0, 0.003 * np.sqrt(150 / N), (B, N)), 1)
        zmax_w = ctr + rng.uniform(0.005, 0.06, (B, N))
        zmin_w = ctr - rng.uniform(0.005, 0.06, (B, N))
        res = np.stack([ctl.predict_wieber_axis(x[b].reshape(3, 1), N, zmax_w[b].reshape(N, 1),
                                                zmin_w[b].reshape(N, 1)).ravel()
                        for b in range(B)])
        e = float(np.abs(res - O.strict_step_batch(x, zmax_w, zmin_w, N, 1.5 / N, d["h"],
                                                   d["g"], d["Q"], d["R"])).max())
        dev = max(dev, e)
        out[f"step{N}_x"], out[f"step{N}_zmax"], out[f"step{N}_zmin"] = x, zmax_w, zmin_w
        out[f"step{N}_out"] = res
        print(f"step N={N}: {B} cold calls, vs oracle max |d| {e:.2e}")
    print(f"{_Rec.n_qp} captured QPs; max rel problem diff {_Rec.max_rel:.2e}; KKT {_Rec.kkt}")
    assert _Rec.max_rel <= 1e-13, _Rec.max_rel
    assert _Rec.kkt["primal"] <= 1e-13 and _Rec.kkt["stationarity"] <= 1e-10, _Rec.kkt
    assert dev <= 1e-12, dev
    out["max_rel_problem_diff"] = _Rec.max_rel
    out["kkt_worst"] = np.array([_Rec.kkt[k] for k in ("primal", "stationarity", "dual_hi",
                                                         "dual_lo")])
    out["max_abs_vs_oracle"] = dev
    np.savez_compressed(os.path.join(HERE, "strict_long_ref.npz"), **out)
    print("saved", os.path.join(HERE, "strict_long_ref.npz"))


# (Q, R, h, g) points beyond default.json's (Q = 1, R = 1e-6, h = 0.75, g = 9.81): the strict
# QP depends on all four (zmp_controller.py:174,184-188; config.py:31-35).  R/Q spans 1e-10 ..
# 1e-2, Q 0.1 .. 100, h 0.5 .. 1.0, g 3.71 .. 9.81.
WEIGHT_POINTS = (
    (1.0, 1e-9, 0.75, 9.81),
    (100.0, 1e-2, 1.0, 9.81),
    (0.1, 1e-3, 0.5, 9.81),
    (10.0, 1e-5, 0.9, 3.71),
    (0.1, 1e-11, 1.0, 9.81),
)


def main_weights():
    """Non-default weights → strict_weights_ref.npz.  Per point w (WEIGHT_POINTS[w]):
    * w{w}_n{64,150}_com / _yhist: the default.json walk at that horizon (the reference's own
      CoPGenerator), generate_com_trajectory(strict=True) with a 400 N kick at n//2, from rest;
    * w{w}_step{16,64,150}_x / _zmax / _zmin / _out: 48 cold predict_wieber_axis calls with
      heavily active bounds (as main()'s step cases)."""
    sys.modules["cvxpy"] = make_cp()
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.generators import CoPGenerator
    from src.mpc_bipedal.controllers import ZMPController

    def instrument(ctl):
        orig = ctl.predict_wieber_axis

        def record(x_init, nb_steps, z_max, z_min):
            _Rec.call = (np.array(x_init, np.float64), nb_steps, np.array(z_max), np.array(z_min),
                         ctl.config)
            out = orig(x_init, nb_steps, z_max, z_min)
            _Rec.axis ^= 1
            return out
        ctl.predict_wieber_axis = record
        return ctl

    out = {"weights": np.array(WEIGHT_POINTS)}
    dev = 0.0
    rng = np.random.default_rng(20251228)
    for w, (Qv, Rv, hv, gv) in enumerate(WEIGHT_POINTS):
        for N in (64, 150):
            d = default_mpc_dict()
            d.update(horizon=N, strict=True, add_force=True, F_ext=400.0, Q=Qv, R=Rv, h=hv,
                     g=gv)
            cfg = MPCConfig(**d)
            zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
            n = len(zmax)
            ctl = instrument(ZMPController(cfg))
            _Rec.rollout, _Rec.axis, _Rec.warm = True, 0, [None, None]
            with contextlib.redirect_stdout(io.StringIO()), \
                    contextlib.redirect_stderr(io.StringIO()):
                com, y_hist = ctl.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                          zmax, zmin)
            out[f"w{w}_n{N}_zmax"], out[f"w{w}_n{N}_zmin"] = zmax, zmin
            out[f"w{w}_n{N}_com"], out[f"w{w}_n{N}_yhist"] = com, y_hist[:, :, 0]
            ref = O.rollout_strict(np.zeros(3), np.zeros(3), zmax, zmin, N, cfg.dt, hv, gv, Qv,
                                   Rv, kick=cfg.dt * cfg.F_ext / cfg.m, kick_step=n // 2)
            e = max(float(np.abs(ref[:, :, 0] - com).max()),
                    float(np.abs(ref[:, 1] - y_hist[:, :, 0]).max()))
            dev = max(dev, e)
            print(f"w{w} (Q={Qv:g}, R={Rv:g}, h={hv:g}, g={gv:g}) N={N}: rollout vs oracle "
                  f"max |d| {e:.2e}, {_Rec.n_qp} QPs, max rel problem diff {_Rec.max_rel:.2e}",
                  flush=True)
        _Rec.rollout = False
        for N in (16, 64, 150):
            d = default_mpc_dict()
            d.update(horizon=N, strict=True, Q=Qv, R=Rv, h=hv, g=gv)
            ctl = instrument(ZMPController(MPCConfig(**d)))
            B = 48
            x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                          rng.uniform(-6, 6, B)], 1)
            ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(rng.normal(0, 0.003, (B, N)), 1)
            zmax_w = ctr + rng.uniform(0.005, 0.06, (B, N))
            zmin_w = ctr - rng.uniform(0.005, 0.06, (B, N))
            res = np.stack([ctl.predict_wieber_axis(x[b].reshape(3, 1), N,
                                                    zmax_w[b].reshape(N, 1),
                                                    zmin_w[b].reshape(N, 1)).ravel()
                            for b in range(B)])
            ref = O.strict_step_batch(x, zmax_w, zmin_w, N, 1.5 / N, hv, gv, Qv, Rv)
            e = float(np.abs(res - ref).max())
            dev = max(dev, e)
            out[f"w{w}_step{N}_x"], out[f"w{w}_step{N}_zmax"] = x, zmax_w
            out[f"w{w}_step{N}_zmin"], out[f"w{w}_step{N}_out"] = zmin_w, res
            print(f"w{w} step N={N}: {B} cold calls, vs oracle max |d| {e:.2e}", flush=True)
    print(f"{_Rec.n_qp} captured QPs; max rel problem diff {_Rec.max_rel:.2e}; KKT {_Rec.kkt}")
    assert _Rec.max_rel <= 1e-13, _Rec.max_rel
    assert _Rec.kkt["primal"] <= 1e-13 and _Rec.kkt["stationarity"] <= 1e-10, _Rec.kkt
    assert _Rec.kkt["dual_hi"] <= 1e-10 and _Rec.kkt["dual_lo"] <= 1e-10, _Rec.kkt
    assert dev <= 1e-12, dev
    out["max_rel_problem_diff"] = _Rec.max_rel
    out["kkt_worst"] = np.array([_Rec.kkt[k] for k in ("primal", "stationarity", "dual_hi",
                                                         "dual_lo")])
    out["max_abs_vs_oracle"] = dev
    out["n_qps"] = _Rec.n_qp
    np.savez_compressed(os.path.join(HERE, "strict_weights_ref.npz"), **out)
    print("saved", os.path.join(HERE, "strict_weights_ref.npz"))


def main_weights_long():
    """Non-default weights at long horizons → strict_weights_long_ref.npz.  Per point w
    (WEIGHT_POINTS[w]):
    * w{w}_n400_*: 200 samples of the default walk's stepping phase at horizon 400 (reference
      CoPGenerator, rows 100..299) from rest at the first CoP centre, generate_com_trajectory
      with an 800 N kick at n//2 (as main_long()'s n400 case);
    * w{w}_step700_*: 8 cold predict_wieber_axis calls at horizon 700 with heavily active
      bounds."""
    sys.modules["cvxpy"] = make_cp()
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.generators import CoPGenerator
    from src.mpc_bipedal.controllers import ZMPController

    def instrument(ctl):
        orig = ctl.predict_wieber_axis

        def record(x_init, nb_steps, z_max, z_min):
            _Rec.call = (np.array(x_init, np.float64), nb_steps, np.array(z_max), np.array(z_min),
                         ctl.config)
            out = orig(x_init, nb_steps, z_max, z_min)
            _Rec.axis ^= 1
            return out
        ctl.predict_wieber_axis = record
        return ctl

    out = {"weights": np.array(WEIGHT_POINTS)}
    dev = 0.0
    rng = np.random.default_rng(20261018)
    for w, (Qv, Rv, hv, gv) in enumerate(WEIGHT_POINTS):
        N = 400
        d = default_mpc_dict()
        d.update(horizon=N, strict=True, add_force=True, F_ext=800.0, Q=Qv, R=Rv, h=hv, g=gv)
        cfg = MPCConfig(**d)
        zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory(save_footsteps=False)
        zx, zn = zmax[100:300].copy(), zmin[100:300].copy()
        n = len(zx)
        mid = (zx[0] + zn[0]) / 2
        x0 = np.array([mid[0], 0.0, 0.0])
        y0 = np.array([mid[1], 0.0, 0.0])
        ctl = instrument(ZMPController(cfg))
        _Rec.rollout, _Rec.axis, _Rec.warm = True, 0, [None, None]
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            com, y_hist = ctl.generate_com_trajectory(x0.reshape(3, 1), y0.reshape(3, 1), zx, zn)
        kick = cfg.dt * cfg.F_ext / cfg.m
        ref = O.rollout_strict(x0, y0, zx, zn, N, cfg.dt, hv, gv, Qv, Rv, kick=kick,
                               kick_step=n // 2)
        e = max(float(np.abs(ref[:, :, 0] - com).max()),
                float(np.abs(ref[:, 1] - y_hist[:, :, 0]).max()))
        dev = max(dev, e)
        out.update({f"w{w}_n400_zmax": zx, f"w{w}_n400_zmin": zn, f"w{w}_n400_x0": x0,
                    f"w{w}_n400_y0": y0, f"w{w}_n400_kick": kick, f"w{w}_n400_com": com,
                    f"w{w}_n400_yhist": y_hist[:, :, 0]})
        print(f"w{w} (Q={Qv:g}, R={Rv:g}, h={hv:g}, g={gv:g}) N=400: rollout vs oracle "
              f"max |d| {e:.2e}, {_Rec.n_qp} QPs", flush=True)
        _Rec.rollout = False
        N, B = 700, 8
        d = default_mpc_dict()
        d.update(horizon=N, strict=True, Q=Qv, R=Rv, h=hv, g=gv)
        ctl = instrument(ZMPController(MPCConfig(**d)))
        x = np.stack([rng.uniform(-0.05, 0.05, B), rng.uniform(-0.6, 0.6, B),
                      rng.uniform(-6, 6, B)], 1)
        ctr = rng.uniform(-0.05, 0.05, (B, 1)) + np.cumsum(
            rng.normal(0, 0.003 * np.sqrt(150 / N), (B, N)), 1)
        zmax_w = ctr + rng.uniform(0.005, 0.06, (B, N))
        zmin_w = ctr - rng.uniform(0.005, 0.06, (B, N))
        res = np.stack([ctl.predict_wieber_axis(x[b].reshape(3, 1), N, zmax_w[b].reshape(N, 1),
                                                zmin_w[b].reshape(N, 1)).ravel()
                        for b in range(B)])
        e = float(np.abs(res - O.strict_step_batch(x, zmax_w, zmin_w, N, 1.5 / N, hv, gv, Qv,
                                                   Rv)).max())
        dev = max(dev, e)
        out[f"w{w}_step700_x"], out[f"w{w}_step700_zmax"] = x, zmax_w
        out[f"w{w}_step700_zmin"], out[f"w{w}_step700_out"] = zmin_w, res
        print(f"w{w} step N=700: {B} cold calls, vs oracle max |d| {e:.2e}", flush=True)
    print(f"{_Rec.n_qp} captured QPs; max rel problem diff {_Rec.max_rel:.2e}; KKT {_Rec.kkt}")
    assert _Rec.max_rel <= 1e-13, _Rec.max_rel
    assert _Rec.kkt["primal"] <= 1e-13 and _Rec.kkt["stationarity"] <= 1e-10, _Rec.kkt
    assert dev <= 1e-12, dev
    out["max_rel_problem_diff"] = _Rec.max_rel
    out["kkt_worst"] = np.array([_Rec.kkt[k] for k in ("primal", "stationarity", "dual_hi",
                                                         "dual_lo")])
    out["max_abs_vs_oracle"] = dev
    out["n_qps"] = _Rec.n_qp
    np.savez_compressed(os.path.join(HERE, "strict_weights_long_ref.npz"), **out)
    print("saved", os.path.join(HERE, "strict_weights_long_ref.npz"))


if __name__ == "__main__":
    if "--long" in sys.argv:
        main_long()
    elif "--weights-long" in sys.argv:
        main_weights_long()
    elif "--weights" in sys.argv:
        main_weights()
    else:
        main()
