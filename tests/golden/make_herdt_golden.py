#!/usr/bin/env python3
"""Herdt-path golden vectors from the REFERENCE's own code (this container only).

The reference's Herdt QP (zmp_controller.py:533-826) is built by its own NumPy code and handed
to cvxpy → OSQP at zmp_controller.py:785-787.  cvxpy and OSQP are not installed (no network;
cvxpy is pinned only as cvxpy>=1.2.0, requirements.txt:2, OSQP not at all), so the reference is
imported with a RECORDING stand-in for the `cp` module: it captures the problem exactly as the
reference states it (quadratic form, linear term, every `A @ u <= b` constraint) and answers
`prob.solve()` with the exact KKT solution of oracle/herdt_oracle.py (parity with OSQP itself
stays unpinned).  Everything else — find_nb_steps, the support-phase segmentation, the
prediction/velocity matrices, constraint assembly, the rollout's foot bookkeeping and force
kick — is the reference's code running unchanged.  The reference's per-step plot
(plot_solution, matplotlib PNGs into results/<side>/) is switched off.

Checked here, at every QP of the rollout: oracle.herdt_oracle.herdt_qp rebuilds the same
(Q, p, G, h) (max abs difference recorded), and the oracle's own rollout reproduces the
reference-driven one.  Saved (tests/golden/herdt_default.npz): the default walk's inputs
(v_ref, states), find_nb_steps of the padded states, the polytope half-spaces, the rollout
outputs (com, y_hist, foot_hist), and 12 single steps (inputs + outputs).

Usage: python tests/golden/make_herdt_golden.py
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import herdt_oracle as HO  # noqa: E402

CAPTURE = {"N": None, "qps": [], "solve_inputs": []}


class _Var:
    __array_ufunc__ = None  # make `ndarray @ var` defer to __rmatmul__

    def __init__(self, n):
        self.n = n
        self.value = None

    def __rmatmul__(self, A):
        return _Lin(np.asarray(A, np.float64))


class _Lin:
    def __init__(self, A):
        self.A = A

    def __le__(self, b):
        return ("le", self.A, np.asarray(b, np.float64).ravel())


class _Quad:
    def __init__(self, Q, c=1.0):
        self.Q, self.c = Q, c

    def __rmul__(self, c):
        return _Quad(self.Q, self.c * c)

    def __add__(self, lin):
        return ("obj", self.c, self.Q, lin.A)


class _Problem:
    def __init__(self, obj, cons):
        self.obj, self.cons = obj, cons

    def solve(self, **kw):
        _, c, Q, p = self.obj
        assert c == 0.5
        G = np.vstack([A for _, A, _ in self.cons]) if self.cons else None
        h = np.concatenate([b for _, _, b in self.cons]) if self.cons else None
        N = CAPTURE["N"]
        n = Q.shape[0]
        m = (n - 2 * N) // 2
        x, lam = HO.herdt_solve(Q, p, G, h, N, m)
        kkt = HO.qp_kkt(Q, p, G, h, x, lam)
        CAPTURE["qps"].append(dict(Q=Q, p=p, G=G, h=h, x=x, kkt=kkt))
        _VAR[0].value = x
        return 0.0


_VAR = [None]


def _variable(n):
    v = _Var(n)
    _VAR[0] = v
    return v


def make_cp():
    cp = types.ModuleType("cvxpy")
    cp.Variable = _variable
    cp.quad_form = lambda u, Q: _Quad(np.asarray(Q, np.float64))
    cp.psd_wrap = lambda Q: Q
    cp.Minimize = lambda o: o
    cp.Problem = _Problem
    cp.OSQP = "OSQP"
    return cp


def main():
    sys.modules["cvxpy"] = make_cp()
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.controllers import ZMPController
    from src.mpc_bipedal.generators.speed_generation import SpeedTrajectoryGenerator
    from src.mpc_bipedal.generators.cop_generator import State

    SMAP = {State.STANDING: HO.STANDING, State.DOUBLE_SUPPORT: HO.DOUBLE_SUPPORT,
            State.SINGLE_SUPPORT: HO.SINGLE_SUPPORT}
    out = {}
    cfg = MPCConfig(method="herdt", add_force=True)  # defaults: horizon 150, classic speeds
    CAPTURE["N"] = cfg.horizon
    sg = SpeedTrajectoryGenerator(cfg)
    vx, vy, states = sg.generate_speed_and_state(save_footsteps=False)
    v_ref = np.stack([vx, vy], 1)
    st_int = np.array([SMAP[s] for s in states], np.int8)
    ctl = ZMPController(cfg)
    ctl.plot_solution = lambda *a, **k: None  # no per-step PNGs (results/<side>/ absent)
    calls = []
    orig = ctl.predict_herdt_joint

    def record(*args):
        calls.append([np.array(a, copy=True) if isinstance(a, np.ndarray) else a for a in args])
        return orig(*args)
    ctl.predict_herdt_joint = record
    # find_nb_steps on the padded state sequence, as the rollout calls it (:468-470)
    spad = np.concatenate([np.array(states), np.repeat(np.array(states)[-1:], cfg.horizon)])
    nb = np.array(ctl.find_nb_steps(spad), np.int64)
    assert np.array_equal(nb, np.array(HO.find_nb_steps(
        np.concatenate([st_int, np.repeat(st_int[-1:], cfg.horizon)])))), "find_nb_steps"
    out.update(v_ref=v_ref, states=st_int, nb_steps=nb, dt=cfg.dt)
    for side, verts in (("left", cfg.left_foot_polytope), ("right", cfg.right_foot_polytope)):
        A, b = ctl._polytope_halfspace(np.array(verts))
        out[f"poly_{side}_A"], out[f"poly_{side}_b"] = A, b
    # the reference rollout, every QP captured and solved exactly
    com, y_hist, foot = ctl.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                    v_ref=v_ref, state_ref=np.array(states))
    out.update(com=com, y_hist=y_hist[:, :, 0], foot_hist=foot)
    qps = CAPTURE["qps"]
    worst = {k: max(q["kkt"].get(k, 0.0) for q in qps) for k in
             ("stationarity", "primal", "dual", "complementarity")}
    print(f"{len(qps)} QPs, worst KKT {worst}")
    # the oracle's restatement of the rollout reproduces the reference-driven one
    com2, yh2, foot2, _ = HO.herdt_rollout(cfg, np.zeros(3), np.zeros(3), v_ref, st_int)
    print("oracle rollout vs reference-driven: com", np.abs(com2 - com).max(), "foot",
          np.abs(foot2 - foot).max(), "y", np.abs(yh2 - y_hist[:, :, 0]).max())
    assert np.abs(com2 - com).max() <= 1e-12 and np.abs(foot2 - foot).max() <= 1e-12
    # the oracle's QP builder rebuilds the captured problems from the reference's own inputs
    n = len(v_ref)
    dmax = 0.0
    steps = []
    pick = set(np.linspace(0, n - 2, 12).astype(int).tolist())
    for i, c in enumerate(calls):
        (x_in, y_in, vwin, xfc, yfc, cur, swin, nbs, _nbn, _xa, _ya, side, _idx) = c
        curi = SMAP[cur]
        wini = np.array([SMAP[t] for t in swin], np.int8)
        Q, p, G, h, N, m = HO.herdt_qp(cfg, x_in, y_in, vwin, float(xfc), float(yfc), curi, wini,
                                       side)
        R = qps[i]
        assert Q.shape == R["Q"].shape and G.shape == R["G"].shape, i

        def rel(a, b):
            return np.abs(a - b).max() / max(1.0, np.abs(b).max()) if a.size else 0.0
        dmax = max(dmax, rel(Q, R["Q"]), rel(p, R["p"]), rel(G, R["G"]), rel(h, R["h"]))
        if i in pick:
            steps.append(dict(x=np.asarray(x_in).ravel(), y=np.asarray(y_in).ravel(), v=vwin,
                              fx=float(xfc), fy=float(yfc), cur=curi, win=wini,
                              side=0 if side == "left" else 1, sol=R["x"], N=N, m=m))
    print(f"oracle QP builder vs captured reference QPs: max rel diff {dmax:.3e}")
    assert dmax <= 1e-13
    out["builder_max_rel_diff"] = dmax
    out["kkt_worst"] = np.array([worst[k] for k in ("stationarity", "primal", "dual",
                                                     "complementarity")])
    for k, s in enumerate(steps):
        for key, val in s.items():
            out[f"step{k}_{key}"] = np.asarray(val)
    out["n_steps_saved"] = len(steps)
    np.savez_compressed(os.path.join(HERE, "herdt_default.npz"), **out)
    print("saved", os.path.join(HERE, "herdt_default.npz"))


# (alpha, beta, gamma) points beyond the class defaults (1e-6, 1, 1): the Herdt QP weights the
# jerk, the velocity tracking and the ZMP centring by them (zmp_controller.py:740-760,
# config.py:43-45).
# (α/γ from 1e-4 down to 2e-7: at 1e-9 (1e-8, 0.1, 10) and 1e-7 (1e-5, 1, 100) the jerk-space
# QP the reference hands to OSQP is conditioned past what an exact FP64 solve of it reproduces
# — the oracle's own rollout moved by more than 1e-11 against the reference-driven one, or its
# Goldfarb–Idnani step broke down — so those points pin nothing.)
WEIGHT_POINTS = (
    (1e-4, 1.0, 1.0),
    (1e-6, 10.0, 0.1),
    (1e-6, 0.5, 5.0),
    (1e-5, 3.0, 20.0),
)


def main_weights(points=None, out_name="herdt_weights.npz"):
    """Non-default Herdt weights → herdt_weights.npz: per point w the default walk's rollout
    (com, y_hist, foot_hist; v_ref and states are the ones of herdt_default.npz) and 6 single
    steps (inputs + the exact solution), every QP captured from the reference's own code.
    `--point w` writes point w alone (herdt_weights_w.npz, for parallel runs), `--merge` joins
    them."""
    sys.modules["cvxpy"] = make_cp()
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    from src.mpc_bipedal.config import MPCConfig
    from src.mpc_bipedal.controllers import ZMPController
    from src.mpc_bipedal.generators.speed_generation import SpeedTrajectoryGenerator
    from src.mpc_bipedal.generators.cop_generator import State

    SMAP = {State.STANDING: HO.STANDING, State.DOUBLE_SUPPORT: HO.DOUBLE_SUPPORT,
            State.SINGLE_SUPPORT: HO.SINGLE_SUPPORT}
    out = {"weights": np.array(WEIGHT_POINTS)}
    worst = dict(stationarity=0.0, primal=0.0, dual=0.0, complementarity=0.0)
    for w, (al, be, ga) in enumerate(WEIGHT_POINTS):
        if points is not None and w not in points:
            continue
        cfg = MPCConfig(method="herdt", add_force=True, alpha=al, beta=be, gamma=ga)
        CAPTURE["N"], CAPTURE["qps"] = cfg.horizon, []
        sg = SpeedTrajectoryGenerator(cfg)
        vx, vy, states = sg.generate_speed_and_state(save_footsteps=False)
        v_ref = np.stack([vx, vy], 1)
        st_int = np.array([SMAP[s] for s in states], np.int8)
        ctl = ZMPController(cfg)
        ctl.plot_solution = lambda *a, **k: None
        calls = []
        orig = ctl.predict_herdt_joint

        def record(*args):
            calls.append([np.array(a, copy=True) if isinstance(a, np.ndarray) else a
                          for a in args])
            return orig(*args)
        ctl.predict_herdt_joint = record
        com, y_hist, foot = ctl.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                        v_ref=v_ref, state_ref=np.array(states))
        qps = CAPTURE["qps"]
        for k in worst:
            worst[k] = max(worst[k], max(q["kkt"].get(k, 0.0) for q in qps))
        com2, yh2, foot2, _ = HO.herdt_rollout(cfg, np.zeros(3), np.zeros(3), v_ref, st_int)
        e = max(np.abs(com2 - com).max(), np.abs(foot2 - foot).max())
        print(f"w{w} (alpha={al:g}, beta={be:g}, gamma={ga:g}): {len(qps)} QPs, oracle rollout "
              f"vs reference-driven {e:.2e}", flush=True)
        assert e <= 1e-11
        out[f"w{w}_max_abs_oracle_vs_reference_driven"] = e
        out[f"w{w}_v_ref"], out[f"w{w}_states"] = v_ref, st_int
        out[f"w{w}_com"], out[f"w{w}_y_hist"], out[f"w{w}_foot_hist"] = com, y_hist[:, :, 0], foot
        n = len(v_ref)
        pick = np.linspace(0, n - 2, 6).astype(int).tolist()
        for j, i in enumerate(pick):
            (x_in, y_in, vwin, xfc, yfc, cur, swin, nbs, _nbn, _xa, _ya, side, _idx) = calls[i]
            fxc, fyc = float(np.ravel(xfc)[0]), float(np.ravel(yfc)[0])
            Q, p, G, h, N, m = HO.herdt_qp(cfg, x_in, y_in, vwin, fxc, fyc,
                                           SMAP[cur], np.array([SMAP[t] for t in swin], np.int8),
                                           side)
            assert Q.shape == qps[i]["Q"].shape
            s = dict(x=np.asarray(x_in).ravel(), y=np.asarray(y_in).ravel(), v=vwin,
                     fx=fxc, fy=fyc, cur=SMAP[cur],
                     win=np.array([SMAP[t] for t in swin], np.int8),
                     side=0 if side == "left" else 1, sol=qps[i]["x"], N=N, m=m)
            for key, val in s.items():
                out[f"w{w}_step{j}_{key}"] = np.asarray(val)
        out[f"w{w}_n_steps_saved"] = len(pick)
    print(f"worst KKT {worst}")
    out["kkt_worst"] = np.array([worst[k] for k in ("stationarity", "primal", "dual",
                                                     "complementarity")])
    np.savez_compressed(os.path.join(HERE, out_name), **out)
    print("saved", os.path.join(HERE, out_name))


def merge_weights():
    out = {"weights": np.array(WEIGHT_POINTS)}
    kkt = np.zeros(4)
    for w in range(len(WEIGHT_POINTS)):
        path = os.path.join(HERE, f"herdt_weights_{w}.npz")
        d = np.load(path)
        for k in d.files:
            if k.startswith(f"w{w}_"):
                out[k] = d[k]
        kkt = np.maximum(kkt, d["kkt_worst"])
    out["kkt_worst"] = kkt
    print("worst KKT", kkt)
    np.savez_compressed(os.path.join(HERE, "herdt_weights.npz"), **out)
    for w in range(len(WEIGHT_POINTS)):
        os.remove(os.path.join(HERE, f"herdt_weights_{w}.npz"))
    print("saved", os.path.join(HERE, "herdt_weights.npz"))


if __name__ == "__main__":
    if "--point" in sys.argv:
        w = int(sys.argv[sys.argv.index("--point") + 1])
        main_weights({w}, f"herdt_weights_{w}.npz")
    elif "--merge" in sys.argv:
        merge_weights()
    elif "--weights" in sys.argv:
        main_weights()
    else:
        main()
