"""Parity of the device Herdt joint footstep QP (csrc/herdt.hip, through the C-ABI) with the
reference-driven golden vectors (tests/golden/herdt_default.npz: the reference's own Herdt code
with each QP solved exactly — see tests/golden/make_herdt_golden.py; parity with OSQP unpinned)
and with the CPU oracle (oracle/herdt_oracle.py).

Tolerances: the reference and the device compute the same exact optimum in FP64; CoM RMSE
<= 1e-9 and footsteps <= 1e-9 here (measured ≈1e-13), the north-star bar is 1e-6.
"""
import numpy as np
import pytest
import torch

from conftest import golden, rmse
from oracle import herdt_oracle as HO

pytestmark = pytest.mark.gpu

from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.controllers import ZMPController  # noqa: E402
from mpc_bipedal.controllers import herdt as H  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")


def test_herdt_rollout_vs_reference():
    """generate_com_trajectory (method='herdt', add_force) on the default walk: CoM, y state
    history and foot positions vs the reference-driven rollout."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt", add_force=True))
    com, y_hist, foot = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                  v_ref=d["v_ref"], state_ref=d["states"])
    assert com.shape == d["com"].shape and y_hist.shape == (len(com), 3, 1)
    assert rmse(com, d["com"]) <= 1e-9
    assert np.abs(foot - d["foot_hist"]).max() <= 1e-9
    assert np.abs(y_hist[:, :, 0] - d["y_hist"]).max() <= 1e-8
    zmp = y_hist[:, :, 0] @ c.C
    assert rmse(zmp, d["y_hist"] @ c.C) <= 1e-9


@pytest.mark.parametrize("w", range(4))
def test_herdt_weights_vs_reference(w):
    """The Herdt QP at (alpha, beta, gamma) points beyond the class defaults (config.py:43-45;
    the jerk, velocity-tracking and ZMP-centring weights of zmp_controller.py:740-760):
    tests/golden/herdt_weights.npz holds the reference's own rollout of the default walk per
    point (recording cvxpy stand-in, exact answers; make_herdt_golden.py --weights) and six of
    its single steps.  CoM and ZMP RMSE ≤ 1e-9, footsteps ≤ 1e-9, steps ≤ 1e-9 relative."""
    d = golden("herdt_weights.npz")
    al, be, ga = (float(v) for v in d["weights"][w])
    cfg = MPCConfig(method="herdt", add_force=True, alpha=al, beta=be, gamma=ga)
    c = ZMPController(cfg)
    com, y_hist, foot = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                  v_ref=d[f"w{w}_v_ref"],
                                                  state_ref=d[f"w{w}_states"])
    assert rmse(com, d[f"w{w}_com"]) <= 1e-9
    assert np.abs(foot - d[f"w{w}_foot_hist"]).max() <= 1e-9
    assert rmse(y_hist[:, :, 0] @ c.C, d[f"w{w}_y_hist"] @ c.C) <= 1e-9
    A, B = c.A, c.B
    for k in range(int(d[f"w{w}_n_steps_saved"])):
        g = lambda key: d[f"w{w}_step{k}_{key}"]
        N, m = int(g("N")), int(g("m"))
        side = "left" if int(g("side")) == 0 else "right"
        xn, yn, fx, fy = c.predict_herdt_joint(g("x"), g("y"), g("v"), g("fx"), g("fy"),
                                               int(g("cur")), g("win"), N, (1, 1), None, None,
                                               side, k)
        sol = g("sol")
        # (relative to the state's size: at beta/gamma = 100 the acceleration row is ≈10 m/s²
        # and the exact QP is conditioned so that two exact FP64 solves agree to ≈5e-10 of it)
        xr = A @ g("x").reshape(3, 1) + B * sol[0]
        yr = A @ g("y").reshape(3, 1) + B * sol[N + m]
        assert np.abs(xn - xr).max() <= 1e-9 * max(1.0, np.abs(xr).max()), k
        assert np.abs(yn - yr).max() <= 1e-9 * max(1.0, np.abs(yr).max()), k
        if m > 0:
            assert abs(fx - sol[N]) <= 1e-9 and abs(fy - sol[2 * N + m]) <= 1e-9, k


def test_herdt_steps_vs_reference():
    """predict_herdt_joint on the saved steps (footsteps in the window: m = 0 .. 7)."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt"))
    A, B = c.A, c.B
    for k in range(int(d["n_steps_saved"])):
        g = lambda key: d[f"step{k}_{key}"]
        N, m = int(g("N")), int(g("m"))
        side = "left" if int(g("side")) == 0 else "right"
        xn, yn, fx, fy = c.predict_herdt_joint(g("x"), g("y"), g("v"), g("fx"), g("fy"),
                                               int(g("cur")), g("win"), N, (1, 1), None, None,
                                               side, k)
        sol = g("sol")
        assert np.abs(xn - (A @ g("x").reshape(3, 1) + B * sol[0])).max() <= 1e-9, k
        assert np.abs(yn - (A @ g("y").reshape(3, 1) + B * sol[N + m])).max() <= 1e-9, k
        if m == 0:
            assert fx is None and fy is None
        else:
            assert abs(fx - sol[N]) <= 1e-9 and abs(fy - sol[2 * N + m]) <= 1e-9, k


def test_herdt_batch_force_sweep():
    """Batched rollout of one walk under an F_ext sweep (shared v_ref/states): the 400 N walk
    equals the single-walk reference rollout, F = 0 equals the oracle without force (short
    walk), every walk converges."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt", add_force=True))
    F = np.array([0.0, 200.0, 400.0, 800.0] * 16)
    com, hist, foot = c.generate_com_trajectory_herdt_batch(None, d["v_ref"], d["states"],
                                                            F_ext=F)
    com = com.cpu().numpy()
    assert com.shape == (64,) + d["com"].shape
    assert rmse(com[2], d["com"]) <= 1e-9 and rmse(com[62], d["com"]) <= 1e-9
    assert np.array_equal(com[0], com[4]) and np.array_equal(com[3], com[63])
    # no force: x axis identical to the forced walks' x axis until the kick
    n = d["com"].shape[0]
    assert np.abs(com[0, : n // 2 + 1] - com[2, : n // 2 + 1]).max() <= 1e-12


def test_herdt_short_walk_vs_oracle():
    """A short ragged walk (a stepping window of the default schedule, velocities 0.2 m/s,
    start mid-walk at rest) against the oracle's own rollout."""
    d = golden("herdt_default.npz")
    st = d["states"][100:190].copy()
    v = np.zeros((len(st), 2))
    v[:, 0] = np.where(st == 0, 0.0, 0.2)
    cfg = MPCConfig(method="herdt", add_force=True, F_ext=300.0)
    com_o, y_o, foot_o, _ = HO.herdt_rollout(cfg, np.zeros(3), np.zeros(3), v, st)
    c = ZMPController(cfg)
    com, y_hist, foot = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                  v_ref=v, state_ref=st)
    assert rmse(com, com_o) <= 1e-9
    assert np.abs(foot - foot_o).max() <= 1e-9


def test_herdt_find_nb_steps_drop_in():
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt"))
    st = d["states"]
    pad = np.concatenate([st, np.repeat(st[-1:], 150)])
    assert np.array_equal(np.array(c.find_nb_steps(pad)), d["nb_steps"])
    A, b = c._polytope_halfspace(np.array(MPCConfig().left_foot_polytope))
    assert np.array_equal(A, d["poly_left_A"])


def test_herdt_work_counters():
    """zmpc_plan_counters [4..7]: every solve of both axes takes at least one active-set pass,
    and the footstep sums match the windows' counts of the default walk."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt", add_force=True))
    plan = c._plan()
    plan.counters(reset=True)
    B = 32
    F = np.linspace(0.0, 800.0, B)
    c.generate_com_trajectory_herdt_batch(None, d["v_ref"], d["states"], F_ext=F)
    k = plan.counters(reset=True)
    n = len(d["states"])
    assert k["herdt_instance_passes"] >= 2 * B * (n - 1)
    assert k["herdt_wave_passes"] * 64 >= k["herdt_instance_passes"]
    assert k["herdt_footsteps_sq"] >= k["herdt_footsteps"] >= 0
    # [9]: the most passes of one solve — at least the mean, at most the cap
    assert k["herdt_instance_passes"] / (2 * B * (n - 1)) <= k["herdt_max_passes_per_solve"] <= 64


def _ragged_schedules(B, n=90):
    """B walks of n samples cut from the default schedule at staggered offsets (the footstep
    count m of the windows differs between the walks of one 32-walk wave), each with its own
    forward speed."""
    d = golden("herdt_default.npz")
    states = np.stack([d["states"][40 + 3 * b: 40 + 3 * b + n] for b in range(B)])
    v = np.zeros((B, n, 2))
    v[:, :, 0] = np.where(states == 0, 0.0, (0.12 + 0.004 * np.arange(B))[:, None])
    return states, v


def test_herdt_per_walk_schedules_equal_single_walks():
    """Per-walk [B,n] states and [B,n,2] v_ref with B = 37 (not a multiple of the 32 walks of a
    wave: invalid-lane clamping), footstep counts differing inside a wave (zero-padded footstep
    columns): every walk equals the same walk launched alone (whose path is pinned to the
    reference-driven golden and to the oracle by the tests above)."""
    B = 37
    states, v = _ragged_schedules(B)
    cfg = MPCConfig(method="herdt", add_force=True, F_ext=300.0)
    c = ZMPController(cfg)
    rng = np.random.default_rng(9)
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    F = rng.uniform(0.0, 600.0, B)
    com, hist, foot = c.generate_com_trajectory_herdt_batch(x0, v, states, F_ext=F)
    com, foot = com.cpu().numpy(), foot.cpu().numpy()
    n = states.shape[1]
    # the windows really differ in footstep count inside the first wave
    pad = np.concatenate([states, np.repeat(states[:, -1:], cfg.horizon, axis=1)], axis=1)
    ms = {H.max_footsteps(pad[b:b + 1], cfg.horizon, n) for b in range(32)}
    assert len(ms) > 1
    for b in range(B):
        cb, _, fb = c.generate_com_trajectory_herdt_batch(x0[b:b + 1], v[b], states[b],
                                                          F_ext=F[b:b + 1])
        assert rmse(com[b], cb[0].cpu().numpy()) <= 1e-9, b
        assert np.abs(foot[b] - fb[0].cpu().numpy()).max() <= 1e-9, b


def test_herdt_rollout_rejects_mismatched_batches():
    """states / nb_next / v_ref given per walk must carry one row per walk."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt"))
    plan = c._plan()
    n = len(d["states"])
    prm = H.make_params(c.config, 7)
    x0 = np.zeros((3, 2, 3))
    nb = np.zeros(n, np.int32)
    with pytest.raises(ValueError, match="states"):
        plan.herdt_rollout(prm, d["v_ref"], np.stack([d["states"]] * 2), nb, x0)
    with pytest.raises(ValueError, match="nb_next"):
        plan.herdt_rollout(prm, d["v_ref"], d["states"], np.zeros((1, n), np.int32), x0)
    with pytest.raises(ValueError, match="v_ref"):
        plan.herdt_rollout(prm, np.stack([d["v_ref"]] * 2), d["states"], nb, x0)
    with pytest.raises(ValueError, match="v_ref"):
        plan.herdt_rollout(prm, np.zeros((n, 3)), d["states"], nb, x0)


def test_herdt_too_many_footsteps_flags_the_wave():
    """A batch whose windows hold more footsteps than params.max_footsteps: every walk of the
    affected wave reports a non-zero status — including a standing walk (no footsteps) that
    shares the wave (no walk reports success from a truncated solve)."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt"))
    plan = c._plan()
    n = len(d["states"])
    states = np.stack([d["states"]] * 3 + [np.zeros(n, np.int8)])
    pad = np.concatenate([states, np.repeat(states[:, -1:], plan.N, axis=1)], axis=1)
    nb = np.array([[t[0] for t in H.find_nb_steps(p)][:n] for p in pad], np.int32)
    assert H.max_footsteps(pad[:1], plan.N, n) >= 3 and H.max_footsteps(pad[3:], plan.N, n) == 0
    prm = H.make_params(c.config, 2)  # too small on purpose
    _, _, st = plan.herdt_rollout(prm, d["v_ref"], states, nb, np.zeros((4, 2, 3)))
    assert np.all(st.cpu().numpy() != 0)


def test_herdt_pass_cap_keeps_last_iterate():
    """zmpc_herdt_params.max_passes = 1 forces the pass cap on every cold solve that needs a
    second pass: those report ZMPC_ST_MAXITER and keep the last iterate (OSQP returns its
    iterate at its own iteration limit; the reference's zero-jerk fallback of
    zmp_controller.py:796-802 is for a solve with no solution, ZMPC_ST_INFEASIBLE) — a finite
    state that is not the zero-jerk one; solves that converge in one pass equal the
    reference-driven golden.  A capped rollout stays finite and flags only the pass cap."""
    d = golden("herdt_default.npz")
    c = ZMPController(MPCConfig(method="herdt"))
    A = c.A
    capped = 0
    for k in range(int(d["n_steps_saved"])):
        g = lambda key: d[f"step{k}_{key}"]
        N, m = int(g("N")), int(g("m"))
        plan = c._plan(N)
        win = H.encode_states(g("win")).reshape(1, N)
        cur = H.encode_states([int(g("cur"))])
        prm = H.make_params(c.config, 8)
        prm.max_passes = 1
        x = np.stack([g("x").reshape(3), g("y").reshape(3)])[None]
        foot = np.array([[float(g("fx")), float(g("fy"))]])
        xn, step, st = plan.herdt_step(prm, x, g("v").reshape(1, N, 2), win, cur, foot,
                                       np.array([int(g("side"))], np.int8))
        stv = int(st[0])
        xn, step = xn[0].cpu().numpy(), step[0].cpu().numpy()
        assert (stv & ~1) == 0, (k, stv)
        assert np.all(np.isfinite(xn)), k
        if stv & 1:
            capped += 1
            # the first pass's iterate, not the zero-jerk fallback.  A cold step's first pass
            # pins no ZMP row and solves the footstep problem exactly, so its iterate is the
            # optimum of the reference's QP with the swing-polytope rows only (the rows on the
            # first footstep's (f_x0, f_y0) alone): pinned against the oracle's exact solve
            side = "left" if int(g("side")) == 0 else "right"
            Q, p, G, h, Nq, mq = HO.herdt_qp(c.config, g("x"), g("y"), g("v"), float(g("fx")),
                                             float(g("fy")), int(g("cur")), g("win"), side)
            n1 = Nq + mq
            poly = (np.abs(np.delete(G, [Nq, n1 + Nq], axis=1)).sum(axis=1) == 0) if mq else \
                np.zeros(len(h), bool)
            u1, _ = HO.herdt_solve(Q, p, G[poly], h[poly], Nq, mq)
            ex = A @ x[0, 0] + c.B[:, 0] * u1[0]
            ey = A @ x[0, 1] + c.B[:, 0] * u1[n1]
            assert np.abs(xn[0] - ex).max() <= 1e-9 * max(1.0, np.abs(ex).max()), k
            assert np.abs(xn[1] - ey).max() <= 1e-9 * max(1.0, np.abs(ey).max()), k
            if mq:
                assert abs(step[0] - u1[Nq]) <= 1e-9 and abs(step[1] - u1[n1 + Nq]) <= 1e-9, k
            assert np.abs(xn[0] - A @ x[0, 0]).max() > 0 or np.abs(xn[1] - A @ x[0, 1]).max() > 0
        else:
            sol = g("sol")
            assert np.abs(xn[0] - (A @ x[0, 0] + c.B[:, 0] * sol[0])).max() <= 1e-9, k
    assert capped > 0
    # capped rollout: finite, only the pass-cap bit
    plan = c._plan()
    n = len(d["states"])
    pad = np.concatenate([d["states"], np.repeat(d["states"][-1:], plan.N)])
    nb = np.array([t[0] for t in H.find_nb_steps(pad)][:n], np.int32)
    prm = H.make_params(c.config, H.max_footsteps(pad[None], plan.N, n))
    prm.max_passes = 1
    hist, foot, st = plan.herdt_rollout(prm, d["v_ref"], d["states"], nb, np.zeros((4, 2, 3)))
    stv = st.cpu().numpy()
    assert np.all((stv & ~1) == 0) and np.any(stv & 1)
    assert bool(torch.isfinite(hist).all()) and bool(torch.isfinite(foot).all())
