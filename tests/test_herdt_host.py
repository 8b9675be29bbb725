"""Herdt joint footstep QP on CPU: the oracle pinned to the reference's own golden vectors, and
the product's host bookkeeping (find_nb_steps, polytopes, footstep bound, C struct layout).

tests/golden/herdt_default.npz comes from tests/golden/make_herdt_golden.py, which ran the
reference's own Herdt code (find_nb_steps, predict_herdt_joint, generate_com_trajectory_herdt)
in the build container with a recording stand-in for cvxpy: the QP data are the reference's,
checked there against oracle.herdt_oracle.herdt_qp to 2.3e-16 relative at all 301 QPs of the
default walk; each QP is solved exactly (KKT-certified).  Parity with OSQP itself is unpinned
(cvxpy/OSQP are not installed, no network).
"""
import ctypes

import numpy as np
import pytest

from conftest import golden
from oracle import herdt_oracle as HO

from mpc_bipedal import _native
from mpc_bipedal.config import MPCConfig
from mpc_bipedal.controllers import herdt as H


def test_oracle_find_nb_steps_vs_reference():
    d = golden("herdt_default.npz")
    st = d["states"]
    pad = np.concatenate([st, np.repeat(st[-1:], 150)])
    assert np.array_equal(np.array(HO.find_nb_steps(pad)), d["nb_steps"])


def test_product_find_nb_steps_vs_reference_and_oracle():
    d = golden("herdt_default.npz")
    st = d["states"]
    pad = np.concatenate([st, np.repeat(st[-1:], 150)])
    assert np.array_equal(np.array(H.find_nb_steps(pad)), d["nb_steps"])
    rng = np.random.default_rng(3)
    for _ in range(200):
        # random phase sequences with runs (any order of the three states)
        runs = rng.integers(1, 6, rng.integers(1, 12))
        seq = np.concatenate([np.full(r, rng.integers(0, 3)) for r in runs]).astype(np.int8)
        assert H.find_nb_steps(seq) == HO.find_nb_steps(seq), seq


def test_polytope_halfspace_vs_reference():
    d = golden("herdt_default.npz")
    cfg = MPCConfig()
    for side, verts in (("left", cfg.left_foot_polytope), ("right", cfg.right_foot_polytope)):
        A, b = H.polytope_halfspace(np.array(verts))
        assert np.array_equal(A, d[f"poly_{side}_A"]) and np.array_equal(b, d[f"poly_{side}_b"])
    with pytest.raises(ValueError, match="shape"):
        H.polytope_halfspace([[0, 0], [1, 1]])


def test_max_footsteps_brute_force():
    d = golden("herdt_default.npz")
    st = d["states"]
    N = 150
    pad = np.concatenate([st, np.repeat(st[-1:], N)])
    n = len(st)
    brute = max(len(HO.support_segments(pad[i], pad[i + 1: i + 1 + N])) - 1
                for i in range(n - 1))
    assert H.max_footsteps(pad[None], N, n) == brute


def test_herdt_params_struct_layout():
    """HerdtParams mirrors zmpc_herdt_params (include/zmpc.h): 6 doubles, int32[2],
    double[2][16][3], int32 max_footsteps, int32 max_passes — 832 bytes."""
    assert ctypes.sizeof(H.HerdtParams) == 6 * 8 + 2 * 4 + 2 * 16 * 3 * 8 + 4 + 4
    assert H.HerdtParams.max_passes.offset == 6 * 8 + 2 * 4 + 2 * 16 * 3 * 8 + 4
    p = H.make_params(MPCConfig(), 6)
    assert p.nfacets[0] == len(golden("herdt_default.npz")["poly_left_b"])
    assert p.max_footsteps == 6
    assert p.max_passes == 0  # the library's default cap
    with pytest.raises(ValueError, match="footsteps"):
        H.make_params(MPCConfig(), 9)


def test_encode_states():
    from mpc_bipedal.generators.cop_generator import State
    s = H.encode_states([State.STANDING, State.DOUBLE_SUPPORT, State.SINGLE_SUPPORT, "STANDING", 2])
    assert s.dtype == np.int8 and s.tolist() == [0, 1, 2, 0, 2]


def test_oracle_steps_vs_reference_qp():
    """The saved steps of the reference-driven rollout: the oracle rebuilds and re-solves them
    (a different code path from the capture) and lands on the same optimum."""
    d = golden("herdt_default.npz")
    cfg = MPCConfig(method="herdt")
    for k in range(int(d["n_steps_saved"])):
        g = lambda key: d[f"step{k}_{key}"]
        side = "left" if int(g("side")) == 0 else "right"
        Q, p, G, h, N, m = HO.herdt_qp(cfg, g("x"), g("y"), g("v"), float(g("fx")),
                                       float(g("fy")), int(g("cur")), g("win"), side)
        assert (N, m) == (int(g("N")), int(g("m")))
        u, lam = HO.herdt_solve(Q, p, G, h, N, m)
        kkt = HO.qp_kkt(Q, p, G, h, u, lam)
        assert kkt["primal"] <= 1e-10 and kkt["stationarity"] <= 1e-8, (k, kkt)
        assert np.abs(u - g("sol")).max() <= 1e-8 * max(1.0, np.abs(g("sol")).max()), k


def test_qp_solve_kkt_random():
    """The oracle's Goldfarb–Idnani solver: KKT on random strictly convex QPs."""
    rng = np.random.default_rng(7)
    for _ in range(20):
        n, m = 12, 30
        A = rng.normal(size=(n, n))
        Q = A @ A.T + 0.1 * np.eye(n)
        p = rng.normal(size=n)
        G = rng.normal(size=(m, n))
        h = rng.uniform(0.1, 1.0, m)
        x, lam = HO.qp_solve(Q, p, G, h)
        k = HO.qp_kkt(Q, p, G, h, x, lam)
        assert k["primal"] < 1e-10 and k["stationarity"] < 1e-9 and k["dual"] == 0.0
        assert k["complementarity"] < 1e-9
