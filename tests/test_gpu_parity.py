"""Parity of the HIP path (through the C-ABI) with the oracle and the reference's golden vectors.

Tolerances: north_star's bar is CoM/ZMP RMSE <= 1e-6 against the reference NumPy solve; the
unconstrained path is held to 1e-9 here (the reference's own BLAS noise floor is ~7e-13), the
strict path to 1e-6 against the exact KKT-certified oracle (parity with OSQP unpinned).
"""
import os

import numpy as np
import pytest
import torch

from conftest import PKG, golden, rmse
from oracle import zmp_oracle as O

pytestmark = pytest.mark.gpu

from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.controllers import ZMPController  # noqa: E402
from mpc_bipedal.solver import Plan, get_plan  # noqa: E402
from mpc_bipedal import _native  # noqa: E402

H, G, Q, R, M = 0.75, 9.81, 1.0, 1e-6, 40.0


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    _native.load()


def plan(N, strict=False, Qv=Q, Rv=R, h=H, dt=None):
    dt = 1.5 / N if dt is None else dt
    return Plan(torch.cuda.current_device(), N, dt, h, G, Qv, Rv, strict)


# --------------------------------------------------------------------------- plan


@pytest.mark.parametrize("N", (1, 10, 32, 64, 150, 512))
def test_plan_matrices(N):
    p = plan(N, strict=(N <= 512))
    dt = 1.5 / N
    Px, Pu = O.prediction_matrices(N, dt, H, G)
    assert np.array_equal(p.export(_native.EXPORT_P), Pu[:, 0])      # bit-exact vs reference
    assert np.array_equal(p.export(_native.EXPORT_PX), Px)
    Mref = Pu.T @ Pu + R / Q * np.eye(N)
    Md = p.export(_native.EXPORT_M)
    assert np.abs(Md - Mref).max() <= 1e-13 * np.abs(Mref).max()    # MFMA (N>=64) / FMA
    k, kx = O.gain_row(N, dt, H, G, Q, R)
    assert np.abs(p.export(_native.EXPORT_K) - k).max() <= 1e-9 * np.abs(k).max()
    assert np.allclose(p.export(_native.EXPORT_KX), kx, rtol=1e-9, atol=0)
    Gd = p.export(_native.EXPORT_G)
    Hz, V, _, _ = O.strict_matrices(N, dt, H, G, Q, R)
    Gref = np.linalg.inv(Hz)
    assert np.abs(Gd - Gref).max() <= 1e-10 * np.abs(Gref).max()
    Hd = p.export(_native.EXPORT_HZ)
    assert np.abs(Hd - Hz).max() <= 1e-10 * np.abs(Hz).max()


@pytest.mark.parametrize("N", (10, 64, 150, 512))
def test_plan_gain_vs_reference_inverse(N):
    d = golden(f"predict_n{N}.npz")
    p = plan(N, dt=float(d["dt"]))
    k = p.export(_native.EXPORT_K)
    assert np.abs(k - d["gain_k"]).max() <= 1e-9 * np.abs(d["gain_k"]).max()
    assert np.allclose(p.export(_native.EXPORT_KX), d["gain_kPx"], rtol=1e-9, atol=0)


# --------------------------------------------------------------------------- drop-in API


@pytest.mark.parametrize("N", (10, 64, 150, 512))
def test_controller_com_trajectory_vs_reference(N):
    d = golden(f"walk_n{N}.npz")
    cfg = MPCConfig(horizon=N, strict=False, add_force=True)
    c = ZMPController(cfg)
    com, y_hist = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)), d["zmax"],
                                            d["zmin"])
    assert com.shape == d["com_force"].shape and y_hist.shape == d["y_hist_force"].shape
    assert rmse(com, d["com_force"]) <= 1e-9
    zmp = np.tensordot(y_hist[:, :, 0], c.C, axes=([1], [0]))   # run_mpc.py:294
    assert rmse(zmp, d["zmp_y_force"]) <= 1e-9
    assert np.abs(y_hist - d["y_hist_force"]).max() <= 1e-7
    xs, ys = c.generate_state_trajectory_wieber(np.zeros((3, 1)), np.zeros((3, 1)), d["zmax"],
                                                d["zmin"])
    assert np.abs(xs - d["state_x_hist"]).max() <= 1e-7
    assert np.abs(ys - d["state_y_hist"]).max() <= 1e-7
    if "com_noforce" in d:
        c2 = ZMPController(MPCConfig(horizon=N, strict=False, add_force=False))
        com2, _ = c2.generate_com_trajectory_wieber(np.zeros((3, 1)), np.zeros((3, 1)),
                                                    d["zmax"], d["zmin"])
        assert rmse(com2, d["com_noforce"]) <= 1e-9
        xs, ys = c2.generate_state_trajectory_wieber(d["state_x0"], d["state_y0"], d["zmax"],
                                                     d["zmin"])
        assert np.abs(xs - d["state_x_hist_x0"]).max() <= 1e-7
        assert np.abs(ys - d["state_y_hist_x0"]).max() <= 1e-7


@pytest.mark.parametrize("N", (10, 64, 150, 512))
def test_predict_wieber_axis_vs_reference(N):
    d = golden(f"predict_n{N}.npz")
    for c in range(len(d["x"])):
        cfg = MPCConfig(horizon=N, strict=False, Q=float(d["Q"][c]), R=float(d["R"][c]),
                        h=float(d["h"][c]), g=float(d["g"][c]))
        out = ZMPController(cfg).predict_wieber_axis(d["x"][c], N, d["zmax"][c], d["zmin"][c])
        ref = d["out"][c]
        assert out.shape == (3, 1)
        assert np.abs(out - ref).max() <= 1e-9 * max(1.0, np.abs(ref).max()), c


def test_batched_step_vs_reference():
    d = golden("predict_n150.npz")
    p = plan(150, dt=float(d["dt"]))
    out, st = p.step(d["x"][:64, :, 0], d["zmax"][:64, :, 0], d["zmin"][:64, :, 0])
    assert np.abs(out.cpu().numpy() - d["out"][:64, :, 0]).max() <= 1e-9 * np.abs(d["out"]).max()
    assert int(st.abs().max()) == 0


def test_speed_generator_wieber_vs_reference():
    """SpeedTrajectoryGenerator wieber mode (speed_generation.py:55-67):
    velocity rows of the reference's own zero-start state rollout (walk_n150 fixture), and
    the batched form on the same walk."""
    from mpc_bipedal.generators import SpeedTrajectoryGenerator
    d = golden("walk_n150.npz")
    dj = dict(ssp_duration=0.24, dsp_duration=0.03, standing_duration=1.0, distance=2.1,
              step_length=0.3, foot_spread=0.1, horizon=150, Q=1.0, R=1e-6, S=1.0, h=0.75,
              g=9.81, m=40.0, F_ext=400.0, strict=False, add_force=True,
              speed_generation="wieber")
    g = SpeedTrajectoryGenerator(MPCConfig(**dj))
    vx, vy, st = g.generate_speed_and_state(save_footsteps=False)
    assert np.abs(vx - d["state_x_hist"][:, 1, 0]).max() <= 1e-9
    assert np.abs(vy - d["state_y_hist"][:, 1, 0]).max() <= 1e-9
    bx, by = g.generate_speed_batch(np.repeat(d["zmax"][None], 3, 0),
                                    np.repeat(d["zmin"][None], 3, 0))
    assert bx.shape == (3, len(vx))
    assert np.abs(bx.cpu().numpy() - vx[None]).max() <= 1e-12
    assert np.abs(by.cpu().numpy() - vy[None]).max() <= 1e-12


def test_cli_matches_reference_walk(tmp_path):
    """mpc_bipedal.cli (run_mpc.py semantics) on default.json, unconstrained: the saved CoM
    equals the reference walk; --batch sweeps F_ext over [0, 2·F_ext] in one rollout
    (the middle walk of an odd batch is the F_ext walk)."""
    import json
    from mpc_bipedal import cli
    d = golden("walk_n150.npz")
    cfgf = tmp_path / "default.json"
    cfgf.write_text(json.dumps({"mpc": dict(
        ssp_duration=0.24, dsp_duration=0.03, standing_duration=1.0, distance=2.1,
        step_length=0.3, foot_spread=0.1, horizon=150, Q=1.0, R=1e-6, S=1.0, h=0.75, g=9.81,
        m=40.0, F_ext=400.0, strict=True, add_force=True)}))
    out = tmp_path / "o.npz"
    assert cli.main(["--config", str(cfgf), "--no-strict", "--save", str(out)]) == 0
    r = np.load(out)
    assert rmse(r["com"][0], d["com_force"]) <= 1e-9
    out3 = tmp_path / "o3.npz"
    assert cli.main(["--config", str(cfgf), "--no-strict", "--batch", "3", "--save",
                     str(out3)]) == 0
    r3 = np.load(out3)
    assert r3["com"].shape == (3,) + d["com_force"].shape
    assert rmse(r3["com"][1], d["com_force"]) <= 1e-9


def _cop_cases():
    """The 7 golden CoP configurations + seeded random walk parameters (ragged n)."""
    from mpc_bipedal.generators import cop_params
    cases = []
    for tag in ("default_n150", "default_n10", "default_n64", "default_n512",
                "classdefaults_n150", "long_n100", "short_n200"):
        d = golden(f"cop_{tag}.npz")
        cases.append(MPCConfig(horizon=int(d["horizon"]), dt=float(d["dt"]),
                               distance=float(d["distance"]),
                               step_length=float(d["step_length"]),
                               foot_spread=float(d["foot_spread"]),
                               ssp_duration=float(d["ssp_duration"]),
                               dsp_duration=float(d["dsp_duration"]),
                               standing_duration=float(d["standing_duration"])))
    rng = np.random.default_rng(8)
    for _ in range(25):
        cases.append(MPCConfig(horizon=150, distance=float(rng.uniform(0.2, 4.0)),
                               step_length=float(rng.uniform(0.1, 0.45)),
                               foot_spread=float(rng.uniform(0.05, 0.15)),
                               ssp_duration=float(rng.uniform(0.1, 0.5)),
                               dsp_duration=float(rng.uniform(0.01, 0.1)),
                               standing_duration=float(rng.uniform(0.2, 1.5))))
    return cases, np.array([cop_params(c) for c in cases])


def test_device_cop_producer_bit_exact():
    """zmpc_cop_generate vs the host generator (itself bit-exact vs the
    reference fixtures): every walk's bounds, states and sample count, padding rows."""
    from mpc_bipedal.generators import CoPGenerator, State, generate_cop_batch
    cases, params = _cop_cases()
    zx, zn, n, st = generate_cop_batch(params)
    zx, zn, n, st = zx.cpu().numpy(), zn.cpu().numpy(), n.cpu().numpy(), st.cpu().numpy()
    code = {State.STANDING: 0, State.DOUBLE_SUPPORT: 1, State.SINGLE_SUPPORT: 2}
    for b, c in enumerate(cases):
        hx, hn, hs = CoPGenerator(c).generate_cop_trajectory()
        nb = len(hx)
        assert n[b] == nb, b
        assert np.array_equal(zx[b, :nb], hx) and np.array_equal(zn[b, :nb], hn), b
        assert np.array_equal(st[b, :nb], [code[s] for s in hs]), b
        assert (zx[b, nb:] == hx[-1]).all() and (zn[b, nb:] == hn[-1]).all()
        assert (st[b, nb:] == -1).all()


def test_ragged_batch_rollout_equals_single_walks():
    """Ragged walks from the device producer, padded to the longest, in ONE rollout with a
    per-walk force step (n_b // 2, zmp_controller.py:90) == each walk run alone through the
    drop-in API (generate_com_trajectory_wieber)."""
    from mpc_bipedal.generators import CoPGenerator, generate_cop_batch
    cases, params = _cop_cases()
    cases = [c for c in cases if abs(c.dt - 0.01) < 1e-15][:12]
    params = params[[i for i, c in enumerate(_cop_cases()[0]) if abs(c.dt - 0.01) < 1e-15][:12]]
    zx, zn, n, _ = generate_cop_batch(params)
    B = len(cases)
    F = np.linspace(100.0, 800.0, B)
    cfg = MPCConfig(horizon=150, strict=False, add_force=True)
    ctl = ZMPController(cfg)
    com, hist = ctl.generate_com_trajectory_batch(np.zeros((B, 2, 3)), zx, zn, F_ext=F,
                                                  walk_lengths=n)
    com = com.cpu().numpy()
    for b, c in enumerate(cases):
        hx, hn, _ = CoPGenerator(c).generate_cop_trajectory()
        one = ZMPController(MPCConfig(horizon=150, strict=False, add_force=True,
                                      F_ext=float(F[b])))
        ref, _ = one.generate_com_trajectory_wieber(np.zeros((3, 1)), np.zeros((3, 1)), hx, hn)
        nb = int(n[b])
        assert np.abs(com[b, :nb] - ref).max() <= 1e-12, b


# --------------------------------------------------------------------------- batches


def synthetic_batch(B, N, seed=20251226, F_max=800.0):
    """SURVEY §8d config-2 style batch: default CoP + rigid offsets, random x0 and F_ext."""
    cop = golden(f"walk_n{N}.npz")
    rng = np.random.default_rng(seed)
    off = rng.uniform(-0.02, 0.02, (B, 1, 2))
    zmax = cop["zmax"][None] + off
    zmin = cop["zmin"][None] + off
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    F = rng.uniform(0.0, F_max, B)
    return zmax, zmin, x0, F, float(cop["dt"])


@pytest.mark.parametrize("N", (64, 150))
def test_batch_unconstrained_vs_oracle(N):
    zmax, zmin, x0, F, dt = synthetic_batch(256, N)
    n = zmax.shape[1]
    kick = dt * F / M
    p = plan(N, dt=dt)
    hist, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, n // 2)
    h = hist.cpu().numpy()
    assert np.abs(h - ref).max() <= 1e-8
    assert rmse(h[..., 0], ref[..., 0]) <= 1e-10
    assert int(st.abs().max()) == 0


def test_shared_cop_equals_dense():
    zmax, zmin, x0, F, dt = synthetic_batch(64, 150)
    n = zmax.shape[1]
    cop = golden("walk_n150.npz")
    p = plan(150, dt=dt)
    kick = dt * F / M
    h_shared, _ = p.rollout(cop["zmax"], cop["zmin"], x0, kick=kick, kick_step=n // 2)
    dense_x = np.repeat(cop["zmax"][None], 64, 0)
    dense_n = np.repeat(cop["zmin"][None], 64, 0)
    h_dense, _ = p.rollout(dense_x, dense_n, x0, kick=kick, kick_step=n // 2)
    # the shared CoP's correlation runs in its own kernel: equal to rounding
    assert (h_shared - h_dense).abs().max().item() <= 1e-13


@pytest.mark.parametrize("n", (2, 3, 65, 300, 513, 514, 900))
def test_shared_cop_equals_dense_lengths(n):
    """A shared CoP (bounds stride 0) takes the once-per-launch correlation
    (zmpc_shared_f_kernel) on single-pass geometries and the per-walk kernels beyond: both
    equal, to rounding (1e-13 abs on O(0.1) states), to the same CoP repeated per walk, with
    per-walk kicks and x0."""
    rng = np.random.default_rng(n)
    dt = 0.01
    zc = np.cumsum(rng.uniform(-0.01, 0.01, (n, 2)), axis=0)
    zmax, zmin = zc + 0.05, zc - 0.05
    B = 96
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    kick = dt * rng.uniform(0, 800, B) / M
    p = plan(150, dt=dt)
    h_shared, _ = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    h_dense, _ = p.rollout(np.repeat(zmax[None], B, 0), np.repeat(zmin[None], B, 0), x0,
                           kick=kick, kick_step=n // 2)
    assert (h_shared - h_dense).abs().max().item() <= 1e-13


@pytest.mark.parametrize("n", (1, 2, 3, 65, 130, 513, 514, 700, 1100, 2500, 4097, 4098, 6000))
def test_walk_lengths(n):
    """Ragged lengths: n=1 (no solve), chunk boundaries of the lane scan, the single-pass /
    wide (2, 4, 8 waves per axis) kernel boundaries (513 | 514, 1025, 2049, 4097) and the
    chunked kernel beyond (4098: one full 1024-step chunk plus a partial one, 6000)."""
    rng = np.random.default_rng(n)
    N = 40
    dt = 1.5 / N
    ctr = np.cumsum(rng.normal(0, 0.01, (3, n, 2)), 1)
    zmax, zmin = ctr + 0.05, ctr - 0.05
    x0 = rng.normal(0, 0.01, (3, 2, 3))
    kick = np.array([0.1, 0.0, -0.2])
    p = plan(N, dt=dt)
    hist, _ = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, n // 2)
    assert np.abs(hist.cpu().numpy() - ref).max() <= 1e-8


@pytest.mark.parametrize("N", (1, 2, 3, 5, 150, 512))
@pytest.mark.parametrize("n", (40, 130, 300, 420))
def test_fast_fir_correlation_odd_chunk_widths(N, n):
    """The fast-FIR correlation (rollout.hip axis_correlate_ffa) runs for odd chunk widths:
    n = 40 / 130 / 300 / 420 give CW = 1 / 3 / 5 / 7; horizons from one tap (no pair sums) to
    512 (tap table and window padding past the unrolled steps).  Every walk vs the oracle;
    horizons below ≈10 samples do not stabilise the walk (states reach 1e6 by n = 420), so the
    bound is relative to the largest state."""
    rng = np.random.default_rng(10 * N + n)
    dt = 0.01
    ctr = np.cumsum(rng.normal(0, 0.01, (3, n, 2)), 1)
    zmax, zmin = ctr + 0.05, ctr - 0.05
    x0 = rng.normal(0, 0.01, (3, 2, 3))
    kick = np.array([0.1, 0.0, -0.2])
    p = plan(N, dt=dt)
    hist, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    assert int(st.abs().max()) == 0
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, n // 2)
    assert np.abs(hist.cpu().numpy() - ref).max() <= 1e-8 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("N,n", ((512, 3649), (512, 3650), (512, 5000), (150, 6001)))
def test_long_walks_any_length(N, n):
    """Walks longer than one LDS-resident pass (n > 3649 at N = 512 was rejected before the
    chunked kernel): every walk vs the oracle, kick in the second chunk."""
    rng = np.random.default_rng(N + n)
    dt = 1.5 / N
    ctr = np.cumsum(rng.normal(0, 0.004, (2, n, 2)), 1)
    zmax, zmin = ctr + 0.05, ctr - 0.05
    x0 = rng.normal(0, 0.01, (2, 2, 3))
    kick = np.array([0.05, -0.1])
    p = plan(N, dt=dt)
    hist, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=1500)
    assert int(st.abs().max()) == 0
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, 1500)
    assert np.abs(hist.cpu().numpy() - ref).max() <= 1e-8


def test_chunk_kernel_equals_wide_kernel():
    """The chunked kernel (ZMPC_OPT_LONG_WALK = 3) and the wide kernel agree on walks the wide
    kernel covers (514 <= n <= 4097)."""
    rng = np.random.default_rng(9)
    for n in (700, 3000):
        ctr = np.cumsum(rng.normal(0, 0.004, (5, n, 2)), 1)
        zmax, zmin = ctr + 0.05, ctr - 0.05
        x0 = rng.normal(0, 0.01, (5, 2, 3))
        kick = rng.uniform(0, 0.1, 5)
        res = []
        for form in (0, 3):
            p = plan(150, dt=0.01).set_option("long_walk", form)
            h, _ = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
            res.append(h.cpu().numpy())
        assert np.abs(res[0] - res[1]).max() <= 1e-12


@pytest.mark.parametrize("N,n", ((920, 2570), (700, 4097)))
def test_wide_kernel_past_64k_lds(N, n):
    """Walks whose wide-kernel geometry needs more than 64 KiB of LDS (8-wave axes, 75 / 86 KiB:
    rollout.hip wide_lds_cap) take the wide kernel instead of the chunked one: equal to the
    chunked kernel (ZMPC_OPT_LONG_WALK = 3) to 1e-12 and to the oracle to 1e-8."""
    rng = np.random.default_rng(N + n)
    dt = 1.5 / N
    B = 3
    ctr = np.cumsum(rng.normal(0, 0.004, (B, n, 2)), 1)
    zmax, zmin = ctr + 0.05, ctr - 0.05
    x0 = rng.normal(0, 0.01, (B, 2, 3))
    kick = rng.uniform(0, 0.1, B)
    res = []
    for form in (0, 3):
        p = plan(N, dt=dt).set_option("long_walk", form)
        h, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
        assert int(st.abs().max()) == 0
        res.append(h.cpu().numpy())
    assert np.abs(res[0] - res[1]).max() <= 1e-12
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, n // 2)
    assert np.abs(res[0] - ref).max() <= 1e-8


def test_kick_step_out_of_range_is_no_kick():
    zmax, zmin, x0, F, dt = synthetic_batch(8, 64)
    p = plan(64, dt=dt)
    a, _ = p.rollout(zmax, zmin, x0, kick=np.full(8, 3.0), kick_step=10 ** 6)
    b, _ = p.rollout(zmax, zmin, x0)
    assert torch.equal(a, b)


def test_empty_batch():
    p = plan(64)
    hist, st = p.rollout(np.zeros((0, 10, 2)), np.zeros((0, 10, 2)), np.zeros((0, 2, 3)))
    assert hist.shape == (0, 10, 2, 3)


@pytest.mark.parametrize("n", (65, 420))
def test_multi_walk_workgroups_vs_oracle(n):
    """More walks than resident workgroups (B > 16 per CU x CUs, several dispatch rounds),
    every walk distinct, all checked."""
    B = 2 * 16 * torch.cuda.get_device_properties(0).multi_processor_count + 37
    rng = np.random.default_rng(n + 7)
    N = 150
    dt = 1.5 / N
    ctr = np.cumsum(rng.normal(0, 0.01, (B, n, 2)), 1)
    zmax, zmin = ctr + rng.uniform(0.02, 0.08, (B, 1, 2)), ctr - 0.05
    x0 = rng.normal(0, 0.01, (B, 2, 3))
    kick = rng.uniform(-0.2, 0.2, B)
    p = plan(N, dt=dt)
    hist, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 3)
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, n // 3)
    assert np.abs(hist.cpu().numpy() - ref).max() <= 1e-8
    assert int(st.abs().max()) == 0


def test_rollout_kernel_variants_agree():
    """The default single-pass kernels (split per axis: one walk per workgroup, the fast-FIR or
    sparse correlation; persistent for even chunk widths) and the cross-check kernel (one wave
    per walk, direct correlation: ZMPC_OPT_ROLLOUT_KERNEL = 1) agree, at an odd (n = 420: 7)
    and an even (n = 360: 6) chunk width, and at n = 480 (chunk width 8: per-walk bounds take
    the wide kernel), with per-walk and shared CoP."""
    for Nn, n_cut in ((150, None), (150, 360), (512, 480)):
        zmax, zmin, x0, F, dt = synthetic_batch(4133 if Nn == 150 else 1031, Nn)
        if n_cut:
            zmax, zmin = zmax[:, :n_cut], zmin[:, :n_cut]
        n = zmax.shape[1]
        kick = dt * F / M
        outs = []
        for kern in (0, 1):
            p = plan(Nn, dt=dt).set_option("rollout_kernel", kern)
            h, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
            assert int(st.abs().max()) == 0
            outs.append(h.cpu().numpy())
            hs, _ = p.rollout(zmax[0], zmin[0], x0, kick=kick, kick_step=n // 2)  # shared CoP
            outs.append(hs.cpu().numpy())
        assert np.abs(outs[0] - outs[2]).max() <= 1e-12
        assert np.abs(outs[1] - outs[3]).max() <= 1e-12


def test_mixed_sparse_dense_batch_between_rounds():
    """A batch between one and two dispatch rounds of the split kernel (B = 3001: walks 2048+
    run in a second round on the slots the first round frees, with the first round's next-round
    prefetch) that mixes the default CoP walks (sparse correlation) with random-walk bounds
    (dense correlation), at chunk widths 7 (n = 420) and 6 (n = 360): the default kernels equal
    the cross-check kernel (ZMPC_OPT_ROLLOUT_KERNEL = 1), and walks at both ends of each round
    match the gain-form oracle.  (Round 6 measured a two-walks-per-workgroup form of this case,
    the second walk's bounds held in registers: slower, 28.5-29.1 vs 27.4-27.5 us at B = 4096,
    profiles/r6e/; not kept.)"""
    rng = np.random.default_rng(5)
    for n_cut in (None, 360):
        zmax, zmin, x0, F, dt = synthetic_batch(3001, 150)
        if n_cut:
            zmax, zmin = zmax[:, :n_cut], zmin[:, :n_cut]
        zmax, zmin = zmax.copy(), zmin.copy()
        n = zmax.shape[1]
        dense = rng.random(3001) < 0.3
        zc = np.cumsum(rng.normal(0, 0.005, (int(dense.sum()), n, 2)), 1)
        zmax[dense], zmin[dense] = zc + 0.05, zc - 0.05
        kick = dt * F / M
        outs = []
        for kern in (0, 1):
            p = plan(150, dt=dt).set_option("rollout_kernel", kern)
            h, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
            assert int(st.abs().max()) == 0
            outs.append(h.cpu().numpy())
        assert np.abs(outs[0] - outs[1]).max() <= 1e-11, n
        idx = np.array([0, 1, 952, 953, 2047, 2048, 2049, 3000])
        ref = O.rollout_gain(zmax[idx], zmin[idx], x0[idx], 150, dt, H, G, Q, R, kick[idx],
                             n // 2)
        assert np.abs(outs[0][idx] - ref).max() <= 1e-8, n


SPARSE_MAX = 40  # rollout.hip kSparseMax: more z_ref changes per axis take the dense form
SPARSE_MAX_WIDE = 64  # kSparseMaxWide: the wide kernel (walks of more than 513 samples)


def _piecewise_walks(rng, B, n, changes):
    """Piecewise-constant bounds with `changes` z_ref changes per axis at distinct random
    samples (always including the first and the last possible one, m = 0 and m = n − 2)."""
    zmax = np.empty((B, n, 2))
    for b in range(B):
        for ax in range(2):
            k = min(changes, n - 1)
            pos = rng.choice(np.arange(1, n - 2), size=max(k - 2, 0), replace=False) \
                if n > 3 else np.array([], int)
            pos = np.unique(np.concatenate([pos, [0, n - 2]]))[:k]
            steps = np.zeros(n)
            steps[pos + 1] = rng.uniform(-0.05, 0.05, pos.size)
            zmax[b, :, ax] = 0.1 + np.cumsum(steps)
    return zmax + 0.05, zmax - 0.05


@pytest.mark.parametrize("N,n", ((150, 2), (150, 65), (150, 350), (150, 420), (150, 513),
                                 (512, 1431), (150, 1100), (256, 1000), (150, 2500)))
def test_sparse_correlation_equals_dense(N, n):
    """The sparse-difference correlation (rollout.hip axis_correlate_sparse, the default for
    piecewise-constant CoP bounds) against the dense forms (ZMPC_OPT_CORRELATION = 1)
    and the oracle, on one batch that mixes default.json walks with rigid offsets, random-walk
    bounds (dense: the fallback), and piecewise-constant bounds with SPARSE_MAX − 1, SPARSE_MAX
    and SPARSE_MAX + 1 changes per axis at random samples including m = 0 and m = n − 2, so
    waves on both sides of the switch sit in one launch.  n covers odd and even chunk widths,
    the split kernels (n ≤ 513) and the wide kernel's FFT and direct forms (longer walks, where
    the limit is SPARSE_MAX_WIDE per axis and a walk is sparse only if both axes are)."""
    rng = np.random.default_rng(n + N)
    cop = golden("walk_n150.npz")
    dt = 1.5 / N if N != 150 else float(cop["dt"])
    lim = SPARSE_MAX if n <= 513 else SPARSE_MAX_WIDE
    parts_hi, parts_lo = [], []
    base = min(n, cop["zmax"].shape[0])
    for _ in range(24):  # default CoP (its first n samples), rigid offsets
        off = rng.uniform(-0.02, 0.02, (1, 2))
        parts_hi.append(np.concatenate([cop["zmax"][:base], np.repeat(cop["zmax"][base - 1:base],
                                                                      n - base, 0)]) + off)
        parts_lo.append(np.concatenate([cop["zmin"][:base], np.repeat(cop["zmin"][base - 1:base],
                                                                      n - base, 0)]) + off)
    hi, lo = np.stack(parts_hi), np.stack(parts_lo)
    ctr = np.cumsum(rng.normal(0, 0.01, (24, n, 2)), 1)  # dense
    hi, lo = np.concatenate([hi, ctr + 0.05]), np.concatenate([lo, ctr - 0.05])
    for c in (1, 2, lim - 1, lim, lim + 1):
        a, b = _piecewise_walks(rng, 8, n, c)
        hi, lo = np.concatenate([hi, a]), np.concatenate([lo, b])
    mixed_hi, mixed_lo = _piecewise_walks(rng, 8, n, 3)  # x sparse, y dense
    mixed_hi[:, :, 1] = ctr[:8, :, 1] + 0.05
    mixed_lo[:, :, 1] = ctr[:8, :, 1] - 0.05
    zmax, zmin = np.concatenate([hi, mixed_hi]), np.concatenate([lo, mixed_lo])
    B = zmax.shape[0]
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    kick = rng.uniform(0, 0.2, B)
    ks = max(n // 3, 0)
    outs = {}
    for mode in ("1", "0"):  # sparse where it applies (default) / dense only
        p = plan(N, dt=dt).set_option("correlation", 0 if mode == "1" else 1)
        h, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=ks)
        assert int(st.abs().max()) == 0
        outs[mode] = h.cpu().numpy()
    scale = np.abs(outs["0"]).max(axis=1, keepdims=True) + 1.0
    assert (np.abs(outs["1"] - outs["0"]) / scale).max() <= 1e-12
    ref = O.rollout_gain(zmax, zmin, x0, N, dt, H, G, Q, R, kick, ks)
    assert np.abs(outs["1"] - ref).max() <= 1e-8


def test_full_size_config2_properties():
    """BASELINE config 2 size (B=4096, N=150): oracle on a sample + translation invariance
    over the whole batch (x0 + δe0 and bounds + δ shift every position by δ exactly)."""
    B = 4096
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150)
    n = zmax.shape[1]
    kick = dt * F / M
    p = plan(150, dt=dt)
    hist, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    assert int(st.abs().max()) == 0
    idx = np.arange(0, B, 64)
    ref = O.rollout_gain(zmax[idx], zmin[idx], x0[idx], 150, dt, H, G, Q, R, kick[idx], n // 2)
    assert np.abs(hist.cpu().numpy()[idx] - ref).max() <= 1e-8
    delta = 0.0625  # exactly representable: the shifted problem is exact in FP64
    x1 = x0.copy()
    x1[:, :, 0] += delta
    h2, _ = p.rollout(zmax + delta, zmin + delta, x1, kick=kick, kick_step=n // 2)
    diff = (h2 - hist).cpu().numpy()
    assert np.abs(diff[..., 0] - delta).max() <= 1e-9
    assert np.abs(diff[..., 1:]).max() <= 1e-7


# --------------------------------------------------------------------------- strict


@pytest.mark.parametrize("N", (16, 64, 150))
def test_strict_step_vs_reference(N):
    """Cold strict predict_wieber_axis calls with heavily active bounds vs the state the
    reference's own strict branch returned (tests/golden/strict_ref.npz: the reference's QP,
    captured by a recording cvxpy stand-in and answered exactly — make_strict_ref_golden.py)."""
    d = golden("strict_ref.npz")
    p = plan(N, strict=True)
    out, st = p.step(d[f"step{N}_x"], d[f"step{N}_zmax"], d[f"step{N}_zmin"])
    ref = d[f"step{N}_out"]
    assert int(st.abs().max()) == 0
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("N", (64, 150))
@pytest.mark.parametrize("F", (0, 400, 800))
def test_strict_rollout_vs_reference(N, F):
    """generate_com_trajectory(strict=True) on the default walk vs the reference-driven strict
    rollout (strict_ref.npz): CoM and ZMP RMSE <= 1e-9 for every F_ext (north star: 1e-6)."""
    d = golden("strict_ref.npz")
    zx, zn = d[f"n{N}_zmax"], d[f"n{N}_zmin"]
    cfg = MPCConfig(horizon=N, strict=True, add_force=F > 0, F_ext=float(F))
    c = ZMPController(cfg)
    com, y_hist = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)), zx, zn)
    assert rmse(com, d[f"n{N}_F{F}_com"]) <= 1e-9
    zmp = y_hist[:, :, 0] @ c.C
    assert rmse(zmp, d[f"n{N}_F{F}_yhist"] @ c.C) <= 1e-9
    assert np.abs(y_hist[:, :, 0] - d[f"n{N}_F{F}_yhist"]).max() <= 1e-6
    # the planned ZMP respects the bounds (strict semantics)
    assert np.all(zmp[1:] <= zx[1:, 1] + 1e-9) and np.all(zmp[1:] >= zn[1:, 1] - 1e-9)


@pytest.mark.parametrize("N", (64, 150))
def test_strict_state_trajectory_x0_vs_reference(N):
    d = golden("strict_ref.npz")
    c = ZMPController(MPCConfig(horizon=N, strict=True))
    xs, ys = c.generate_state_trajectory_wieber(d[f"n{N}_x0"].reshape(3, 1),
                                                d[f"n{N}_y0"].reshape(3, 1), d[f"n{N}_zmax"],
                                                d[f"n{N}_zmin"])
    assert rmse(xs[:, 0, 0], d[f"n{N}_x0_xhist"][:, 0]) <= 1e-9
    assert rmse(ys[:, 0, 0], d[f"n{N}_x0_yhist"][:, 0]) <= 1e-9
    assert np.abs(xs[:, :, 0] - d[f"n{N}_x0_xhist"]).max() <= 1e-6
    assert np.abs(ys[:, :, 0] - d[f"n{N}_x0_yhist"]).max() <= 1e-6


def test_strict_equals_unconstrained_when_inactive():
    zmax, zmin, x0, F, dt = synthetic_batch(32, 64, F_max=50.0)
    n = zmax.shape[1]
    zx, zn = zmax + 5.0, zmin - 5.0
    kick = dt * F / M
    hs, st = plan(64, strict=True, dt=dt).rollout(zx, zn, x0, kick=kick, kick_step=n // 2)
    hu, _ = plan(64, dt=dt).rollout(zx, zn, x0, kick=kick, kick_step=n // 2)
    assert int(st.abs().max()) == 0
    assert np.abs((hs - hu).cpu().numpy()).max() <= 1e-8


def test_strict_batch_vs_oracle_sample():
    """Config-3 style batch (offsets, F_ext ~ U(0,800)): a sample of walks vs the oracle."""
    B = 64
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150, seed=3)
    n = zmax.shape[1]
    kick = dt * F / M
    hist, st = plan(150, strict=True, dt=dt).rollout(zmax, zmin, x0, kick=kick,
                                                     kick_step=n // 2)
    assert int(st.abs().max()) == 0
    h = hist.cpu().numpy()
    for b in (0, 7, 31, 63):
        ref = O.rollout_strict(x0[b, 0], x0[b, 1], zmax[b], zmin[b], 150, dt, H, G, Q, R,
                               kick=kick[b], kick_step=n // 2)
        assert rmse(h[b, :, :, 0], ref[:, :, 0]) <= 1e-6, b


def test_strict_translation_invariance_full_batch():
    B = 2048
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150, seed=5)
    n = zmax.shape[1]
    kick = dt * F / M
    p = plan(150, strict=True, dt=dt)
    h1, s1 = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    x1 = x0.copy()
    x1[:, :, 0] += 0.0625
    h2, s2 = p.rollout(zmax + 0.0625, zmin + 0.0625, x1, kick=kick, kick_step=n // 2)
    assert int(s1.abs().max()) == 0 and int(s2.abs().max()) == 0
    d = (h2 - h1).cpu().numpy()
    assert np.abs(d[..., 0] - 0.0625).max() <= 1e-7


@pytest.mark.parametrize("shared", (False, True))
def test_strict_kick_order_same_results(shared):
    """order.hip: walks with per-walk kicks are mapped to lanes sorted by (kick step, kick).
    The schedule changes, the results do not: the default run and one in input order
    (ZMPC_OPT_KICK_ORDER = 0) give bitwise the same histories — per-walk bounds and the shared
    CoP, per-walk kick steps, a batch that is not a multiple of 64 — and the sorted run needs no
    more wave passes for the same instance passes."""
    B = 1000
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150, seed=21)
    n = zmax.shape[1]
    rng = np.random.default_rng(22)
    F = rng.uniform(-800.0, 800.0, B)
    ks = rng.integers(n // 4, 3 * n // 4, B).astype(np.int64)
    if shared:  # one [n, 2] CoP for every walk (bounds stride 0)
        zmax, zmin, x0 = zmax[0], zmin[0], np.zeros_like(x0)
    outs = []
    for mode in (1, 0):
        p = plan(150, strict=True, dt=dt).set_option("kick_order", mode)
        p.set_option("strict_solver", 3)  # (the kick order is the LQ kernel's lane order)
        h, st = p.rollout(zmax, zmin, x0, kick=dt * F / M, kick_step=ks)
        c = p.counters()
        assert int(st.abs().max()) == 0
        outs.append((h.cpu().numpy(), c["wave_passes"], c["instance_passes"]))
    (hs, wps, ips), (hi, wpi, ipi) = outs
    assert np.array_equal(hs, hi)
    assert ips == ipi and wps <= wpi
    # one walk of the batch against the oracle (per-walk kick step)
    b = 777
    zb, nb = (zmax, zmin) if shared else (zmax[b], zmin[b])
    ref = O.rollout_strict(x0[b, 0], x0[b, 1], zb, nb, 150, dt, H, G, Q, R,
                           kick=dt * F[b] / M, kick_step=int(ks[b]))
    assert rmse(hs[b, :, :, 0], ref[:, :, 0]) <= 1e-9


@pytest.mark.parametrize("shared,N", ((False, 150), (True, 150), (False, 10)))
def test_strict_run_length_bounds_same_results(shared, N):
    """ZMPC_OPT_STRICT_BOUNDS: the LQ kernel reading the bounds as runs of equal values (2)
    and as one staged row per sample (1) give bitwise the same histories and work — per-walk
    bounds (kick-ordered lanes, a batch that is not a multiple of 64, walks whose bounds
    change every sample in part) and the shared CoP, a horizon that is not a multiple of the
    segment."""
    B = 333
    zmax, zmin, x0, F, dt = synthetic_batch(B, N, seed=31)
    n = zmax.shape[1]
    rng = np.random.default_rng(32)
    F = rng.uniform(-800.0, 800.0, B)
    ks = rng.integers(n // 4, 3 * n // 4, B).astype(np.int64)
    if shared:
        zmax, zmin, x0 = zmax[0], zmin[0], np.zeros_like(x0)
    else:  # a few walks with a ramp in their bounds: one run per sample
        ramp = 0.01 * np.sin(np.arange(n) * 0.3)
        zmax[5:9, :, 0] += ramp
        zmin[5:9, :, 0] += ramp
    outs = []
    for mode in (1, 2):
        p = plan(N, strict=True, dt=dt).set_option("strict_solver", 3)
        p.set_option("strict_bounds", mode)
        h, st = p.rollout(zmax, zmin, x0, kick=dt * F / M, kick_step=ks)
        outs.append((h.cpu().numpy(), st.cpu().numpy(), p.counters()["instance_passes"]))
    (h1, s1, c1), (h2, s2, c2) = outs
    assert np.array_equal(h1, h2) and np.array_equal(s1, s2) and c1 == c2


def test_strict_work_counters():
    """zmpc_plan_counters: every solve takes at least one active-set pass; the working-set
    slots are a part of all pass-slots; reset zeroes them."""
    B = 128
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150, seed=11)
    n = zmax.shape[1]
    p = plan(150, strict=True, dt=dt).set_option("strict_solver", 3)  # the LQ kernel counts
    p.counters(reset=True)
    _, st = p.rollout(zmax, zmin, x0, kick=dt * F / M, kick_step=n // 2)
    c = p.counters(reset=True)
    assert int(st.abs().max()) == 0
    assert c["launches"] == 1
    solves = B * (n - 1) * 2
    assert solves <= c["instance_passes"] <= 3 * solves
    assert 0 < c["working_set_slots"] < c["instance_passes"] * 150
    assert c["wave_passes"] * 64 >= c["instance_passes"]
    # [8]: the most passes of one solve — at least the mean, at most the cap
    assert c["instance_passes"] / solves <= c["max_passes_per_solve"] <= 64
    assert p.counters()["launches"] == 0


def _oracle_strict_walk(job):
    """Spawned worker: oracle.rollout_strict of one shared-CoP scenario (1 BLAS thread)."""
    zx, zn, kick, n = job
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        return O.rollout_strict(np.zeros(3), np.zeros(3), zx, zn, 150, 1.5 / 150, H, G, Q, R,
                                kick=kick, kick_step=n // 2)


def test_strict_shared_cop_config4():
    """BASELINE config 4 (run_compare_resistance.py:87-169 scaled up): one shared default.json
    CoP for every scenario (bounds stride 0: strict_lq.hip stages one group's lanes for the
    whole launch and keeps cached checkpoints), x0 = 0, F_ext ~ U(0, 800) N, B = 4096.
    The F = 0/400/800 N scenarios equal the reference-driven strict rollouts
    (strict_ref.npz); 8 more scenarios equal the oracle's rollout; the x axis (no kick) is
    the same for every scenario."""
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    d = golden("strict_ref.npz")
    zx, zn = d["n150_zmax"], d["n150_zmin"]
    n, dt = len(zx), 1.5 / 150
    B = 4096
    F = np.random.default_rng(404).uniform(0.0, 800.0, B)
    F[0], F[1], F[2] = 400.0, 0.0, 800.0
    kick = dt * F / M
    p = plan(150, strict=True)
    hist, st = p.rollout(zx, zn, np.zeros((B, 2, 3)), kick=kick, kick_step=n // 2)
    assert int(st.abs().max()) == 0
    h = hist.cpu().numpy()
    for b, Fv in ((0, 400), (1, 0), (2, 800)):
        assert rmse(h[b, :, :, 0], d[f"n150_F{Fv}_com"]) <= 1e-9, Fv
        assert rmse(h[b, :, 1] @ np.array([1.0, 0.0, -H / G]),
                    d[f"n150_F{Fv}_yhist"] @ np.array([1.0, 0.0, -H / G])) <= 1e-9, Fv
    pick = (3, 17, 500, 1023, 2048, 3001, 4000, 4095)
    with ProcessPoolExecutor(max_workers=len(pick),
                             mp_context=multiprocessing.get_context("spawn")) as ex:
        refs = list(ex.map(_oracle_strict_walk, [(zx, zn, kick[b], n) for b in pick]))
    for b, ref in zip(pick, refs):
        assert rmse(h[b, :, :, 0], ref[:, :, 0]) <= 1e-9, b
    assert np.abs(h[:, :, 0] - h[0:1, :, 0]).max() <= 1e-12


def _oracle_strict_walk_b(job):
    """Spawned worker: oracle.rollout_strict of one per-walk config-3 walk (1 BLAS thread)."""
    x0, zx, zn, kick, ks, dt = job
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        return O.rollout_strict(x0[0], x0[1], zx, zn, 150, dt, H, G, Q, R, kick=kick,
                                kick_step=ks)


def test_strict_config3_full_size():
    """BASELINE config 3 at its full per-GPU size: B = 65 536 default.json walks with per-walk
    rigid offsets (seed 20251226), x0 ~ U(−0.01, 0.01), F_ext ~ U(0, 800) N at
    n//2, strict (zmp_controller.py:173-195).  Every status is 0; translating CoP and x0 by
    δ = 0.0625 translates every CoM position by δ; 44 walks spread over the whole launch —
    lane positions of the first and the last workgroups and one walk of every 8th workgroup
    in the kernel's kick order (order.hip: walks sorted by (kick step, float32 kick), stable)
    — equal the oracle's exact rollout at ≤ 1e-9 CoM RMSE."""
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    B = 65536
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150)
    n = zmax.shape[1]
    kick = dt * F / M
    p = plan(150, strict=True, dt=dt)
    zx_d = torch.as_tensor(zmax, device="cuda")
    zn_d = torch.as_tensor(zmin, device="cuda")
    x0_d = torch.as_tensor(x0, device="cuda")
    kick_d = torch.as_tensor(kick, device="cuda")
    h1, s1 = p.rollout(zx_d, zn_d, x0_d, kick=kick_d, kick_step=n // 2)
    assert int(s1.abs().max()) == 0
    delta = 0.0625
    x1 = x0_d.clone()
    x1[:, :, 0] += delta
    h2, s2 = p.rollout(zx_d + delta, zn_d + delta, x1, kick=kick_d, kick_step=n // 2)
    assert int(s2.abs().max()) == 0
    assert float(((h2 - h1)[..., 0] - delta).abs().max()) <= 1e-7
    del h2, x1
    order = np.argsort(kick.astype(np.float32), kind="stable")   # lane position -> walk
    wg = 256  # lane positions per 8-wave workgroup
    pos = [0, 1, 63, 64, 127, 200, 255, B - 256, B - 193, B - 64, B - 2, B - 1]
    pos += [w * wg + (w * 37) % wg for w in range(0, B // wg, 8)]
    walks = [int(order[q]) for q in pos]
    h = h1[walks].cpu().numpy()
    jobs = [(x0[b], zmax[b], zmin[b], float(kick[b]), n // 2, dt) for b in walks]
    with ProcessPoolExecutor(max_workers=16,
                             mp_context=multiprocessing.get_context("spawn")) as ex:
        refs = list(ex.map(_oracle_strict_walk_b, jobs))
    for i, (b, ref) in enumerate(zip(walks, refs)):
        assert rmse(h[i, :, :, 0], ref[:, :, 0]) <= 1e-9, b
        assert np.abs(h[i] - ref).max() <= 1e-6, b


def test_strict_shared_cop_full_size_properties():
    """Config 4 at its full per-GPU size (125 000 scenarios, shared CoP): every scenario's
    status is 0, the x-axis rows are the same for every scenario, translating the CoP and the
    initial CoM by δ translates every CoM position by δ, and 16 scenarios chosen by their lane
    position — resident and queued tasks, the last block — equal the oracle's rollout."""
    d = golden("strict_ref.npz")
    zx, zn = d["n150_zmax"], d["n150_zmin"]
    n, dt = len(zx), 1.5 / 150
    B = 125_000
    F = np.random.default_rng(405).uniform(0.0, 800.0, B)
    kick = torch.as_tensor(dt * F / M, device="cuda")
    p = plan(150, strict=True)
    x0 = torch.zeros((B, 2, 3), dtype=torch.float64, device="cuda")
    h1, s1 = p.rollout(zx, zn, x0, kick=kick, kick_step=n // 2)
    delta = 0.0625
    x1 = x0.clone()
    x1[:, :, 0] += delta
    h2, s2 = p.rollout(zx + delta, zn + delta, x1, kick=kick, kick_step=n // 2)
    assert int(s1.abs().max()) == 0 and int(s2.abs().max()) == 0
    assert float((h1[:, :, 0] - h1[0:1, :, 0]).abs().max()) <= 1e-12
    assert float(((h2 - h1)[..., 0] - delta).abs().max()) <= 1e-7
    assert float((h2 - h1)[..., 1:].abs().max()) <= 1e-5
    # scenarios by lane position in the kernel's kick order (order.hip: (kick step, float32
    # kick), stable): the launch is 489 8-wave blocks (4 groups of 64 walks), the grid the
    # resident blocks, the rest run as queued tasks — y waves first, then x waves.  Positions
    # in the first and the last resident blocks, in queued blocks across the queue, and in the
    # last block (walks 124 928 .. 124 999), each rolled by the oracle on its own kick.
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    order = np.argsort((dt * F / M).astype(np.float32), kind="stable")  # position -> scenario
    blocks = (B + 255) // 256
    pos = [0, 255, 256 * 255 + 17, 256 * 256, 256 * 256 + 100, 256 * 300 + 63, 256 * 300 + 64,
           256 * 350 + 200, 256 * 400 + 1, 256 * 450 + 128, 256 * 470 + 255, 256 * 480 + 64,
           256 * (blocks - 2) + 190, 256 * (blocks - 1), 256 * (blocks - 1) + 37, B - 1]
    walks = [int(order[q]) for q in pos]
    h = h1[walks].cpu().numpy()
    with ProcessPoolExecutor(max_workers=16,
                             mp_context=multiprocessing.get_context("spawn")) as ex:
        refs = list(ex.map(_oracle_strict_walk, [(zx, zn, float(kick[b]), n) for b in walks]))
    for b, hb, ref in zip(walks, h, refs):
        assert rmse(hb[:, :, 0], ref[:, :, 0]) <= 1e-9, b
        assert np.abs(hb[:, 1] - ref[:, 1]).max() <= 1e-6, b


def test_config5_full_size():
    """BASELINE config 5 at its per-GPU size (16 384 walks over 8 GPUs = 2048 per GPU): N = 512,
    dt = 1.5/512, n = 1431, default.json walks + rigid offsets, x0 and F_ext as SURVEY §8d —
    the wide kernel with its launch geometry of the bench.  Translation invariance over the
    whole batch (CoP and x0 + δ ⇒ every CoM position + δ), and 32 walks spread over the batch
    equal the gain-form oracle (oracle.rollout_gain, zmp_controller.py:196-199)."""
    B = 2048
    zmax, zmin, x0, F, dt = synthetic_batch(B, 512)
    n = zmax.shape[1]
    assert n == 1431
    kick = dt * F / M
    p = plan(512, dt=dt)
    zx_d = torch.as_tensor(zmax, device="cuda")
    zn_d = torch.as_tensor(zmin, device="cuda")
    x0_d = torch.as_tensor(x0, device="cuda")
    kick_d = torch.as_tensor(kick, device="cuda")
    h1, s1 = p.rollout(zx_d, zn_d, x0_d, kick=kick_d, kick_step=n // 2)
    delta = 0.0625
    x1 = x0_d.clone()
    x1[:, :, 0] += delta
    h2, s2 = p.rollout(zx_d + delta, zn_d + delta, x1, kick=kick_d, kick_step=n // 2)
    assert int(s1.abs().max()) == 0 and int(s2.abs().max()) == 0
    assert float(((h2 - h1)[..., 0] - delta).abs().max()) <= 1e-7
    pick = np.unique(np.linspace(0, B - 1, 32).astype(int))
    ref = O.rollout_gain(zmax[pick], zmin[pick], x0[pick], 512, dt, H, G, Q, R, kick[pick],
                         n // 2)
    h = h1[torch.as_tensor(pick, device="cuda")].cpu().numpy()
    assert np.abs(h - ref).max() <= 1e-8
    assert rmse(h[..., 0], ref[..., 0]) <= 1e-10


# ------------------------------------------------ strict: long horizons, Cholesky cross-check


def test_strict_long_horizon_rollout_vs_oracle():
    """N = 400: the LQ kernel with 4 waves per workgroup (8 waves' slot flags exceed LDS);
    300 samples of the stepping phase, 800 N kick, vs the reference-driven strict rollout
    (tests/golden/strict_long_ref.npz)."""
    d = golden("strict_long_ref.npz")
    N = 400
    zx, zn = d["n400_zmax"], d["n400_zmin"]
    n = len(zx)
    x0 = np.stack([d["n400_x0"], d["n400_y0"]])[None]
    p = plan(N, strict=True)
    hist, st = p.rollout(zx, zn, x0, kick=np.array([float(d["n400_kick"])]), kick_step=n // 2)
    assert int(st.abs().max()) == 0
    h = hist.cpu().numpy()[0]
    assert rmse(h[:, :, 0], d["n400_com"]) <= 1e-9
    assert np.abs(h[:, 1] - d["n400_yhist"]).max() <= 1e-6


@pytest.mark.parametrize("N,solver", ((400, 3), (400, 4), (700, 3), (700, 4), (1300, 0)))
def test_strict_long_horizon_step_vs_oracle(N, solver):
    """Cold-start strict solves, vs the reference's own strict calls (strict_long_ref.npz): the
    LQ kernel (3) at horizons it runs with 4, 2 and 1 waves per workgroup, the parallel-in-time
    kernel (4) with whole-wave instances to N = 960 (C = 7 and 11 slots per lane), and the
    automatic choice beyond it (N = 1300: the LQ kernel)."""
    d = golden("strict_long_ref.npz")
    p = plan(N, strict=True)
    if solver:
        p.set_option("strict_solver", solver)
    out, st = p.step(d[f"step{N}_x"], d[f"step{N}_zmax"], d[f"step{N}_zmin"])
    ref = d[f"step{N}_out"]
    assert int(st.abs().max()) == 0
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())


def test_strict_horizon_limit():
    with pytest.raises(ValueError, match="strict horizon"):
        plan(2465, strict=True)


@pytest.mark.parametrize("solver", (1, 2, 3, 4))
def test_strict_solvers_vs_reference(solver):
    """Every strict solver forced through ZMPC_OPT_STRICT_SOLVER — 1 the reduced-Cholesky tile
    kernel (16 instances per workgroup, MFMA GEMM), 2 the reduced-Cholesky one-instance-per-
    wavefront kernel, 3 the LQ lane-per-instance kernel (the large-batch default), 4 the
    parallel-in-time one-instance-per-wavefront kernel (the small-batch default) — on
    the reference-driven strict walks (N = 64/150, F = 0/400/800 N), the cold single solves,
    and the N = 400 long-horizon fixtures: CoM RMSE ≤ 1e-9, single solves ≤ 1e-7 relative."""
    s = golden("strict_ref.npz")
    lg = golden("strict_long_ref.npz")
    for N in (64, 150):
        zx, zn = s[f"n{N}_zmax"], s[f"n{N}_zmin"]
        n, dt = len(zx), 1.5 / N
        p = plan(N, strict=True).set_option("strict_solver", solver)
        F = np.array([0.0, 400.0, 800.0])
        h, st = p.rollout(zx, zn, np.zeros((3, 2, 3)), kick=dt * F / M, kick_step=n // 2)
        assert int(st.abs().max()) == 0
        for b, Fv in enumerate((0, 400, 800)):
            assert rmse(h.cpu().numpy()[b][:, :, 0], s[f"n{N}_F{Fv}_com"]) <= 1e-9, (N, Fv)
        out, st = p.step(s[f"step{N}_x"], s[f"step{N}_zmax"], s[f"step{N}_zmin"])
        ref = s[f"step{N}_out"]
        assert int(st.abs().max()) == 0
        assert np.abs(out.cpu().numpy() - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())
    p = plan(400, strict=True).set_option("strict_solver", solver)
    zx, zn = lg["n400_zmax"], lg["n400_zmin"]
    n = len(zx)
    x0 = np.stack([lg["n400_x0"], lg["n400_y0"]])[None]
    h, st = p.rollout(zx, zn, x0, kick=np.array([float(lg["n400_kick"])]), kick_step=n // 2)
    assert int(st.abs().max()) == 0
    assert rmse(h.cpu().numpy()[0][:, :, 0], lg["n400_com"]) <= 1e-9
    out, st = p.step(lg["step400_x"], lg["step400_zmax"], lg["step400_zmin"])
    ref = lg["step400_out"]
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())
    if solver in (1, 2):
        with pytest.raises(ValueError, match="reduced-Cholesky"):
            plan(600, strict=True).set_option("strict_solver", solver)
    if solver == 4:
        with pytest.raises(ValueError, match="small-batch"):
            plan(961, strict=True).set_option("strict_solver", solver)


@pytest.mark.parametrize("solver", (3, 4))
@pytest.mark.parametrize("w", range(5))
def test_strict_weights_vs_reference(w, solver):
    """Strict parity beyond default.json's weights (the QP depends on Q, R, h and g:
    zmp_controller.py:174,184-188, config.py:31-35).  tests/golden/strict_weights_ref.npz holds,
    per (Q, R, h, g) point — R/Q from 1e-10 to 1e-2, Q 0.1 .. 100, h 0.5 .. 1.0, g 3.71 and
    9.81 — the reference's own strict branch (recording cvxpy stand-in, exact answers,
    make_strict_ref_golden.py --weights) on the default.json walk at N = 64 and 150 with a
    400 N kick, and 48 cold heavily-active predict_wieber_axis calls at N = 16, 64, 150.  The
    LQ kernel (3) and the parallel-in-time kernel (4): CoM and ZMP RMSE ≤ 1e-10 (round 6: was
    1e-9), single solves ≤ 1e-9 relative, every status 0."""
    d = golden("strict_weights_ref.npz")
    Qv, Rv, hv, gv = (float(v) for v in d["weights"][w])
    cz = np.array([1.0, 0.0, -hv / gv])
    for N in (64, 150):
        zx, zn = d[f"w{w}_n{N}_zmax"], d[f"w{w}_n{N}_zmin"]
        n, dt = len(zx), 1.5 / N
        p = Plan(torch.cuda.current_device(), N, dt, hv, gv, Qv, Rv, True)
        p.set_option("strict_solver", solver)
        h, st = p.rollout(zx, zn, np.zeros((1, 2, 3)), kick=np.array([dt * 400.0 / M]),
                          kick_step=n // 2)
        assert int(st.abs().max()) == 0
        h = h.cpu().numpy()[0]
        # (measured at every point, both kernels: CoM ≤ 1.1e-11, ZMP ≤ 6.1e-14 — profiles/r6b/
        # sw.log; the walks reach 2.4e3 m at the cheapest jerk)
        assert rmse(h[:, :, 0], d[f"w{w}_n{N}_com"]) <= 1e-10, N
        assert rmse(h[:, 1] @ cz, d[f"w{w}_n{N}_yhist"] @ cz) <= 1e-10, N
        assert np.abs(h[:, 1] - d[f"w{w}_n{N}_yhist"]).max() <= 1e-6, N
    for N in (16, 64, 150):
        p = Plan(torch.cuda.current_device(), N, 1.5 / N, hv, gv, Qv, Rv, True)
        p.set_option("strict_solver", solver)
        out, st = p.step(d[f"w{w}_step{N}_x"], d[f"w{w}_step{N}_zmax"], d[f"w{w}_step{N}_zmin"])
        ref = d[f"w{w}_step{N}_out"]
        assert int(st.abs().max()) == 0
        assert np.abs(out.cpu().numpy() - ref).max() <= 1e-9 * max(1.0, np.abs(ref).max()), N


@pytest.mark.parametrize("solver", (3, 4))
@pytest.mark.parametrize("w", range(5))
def test_strict_weights_long_horizon(w, solver):
    """The five (Q, R, h, g) points of test_strict_weights_vs_reference at long horizons
    (tests/golden/strict_weights_long_ref.npz, make_strict_ref_golden.py --weights-long): the
    reference's strict branch on 200 samples of the default walk's stepping phase at N = 400 with
    an 800 N kick, and 8 cold heavily-active calls at N = 700.  Both kernels (3: the LQ kernel
    with 4-wave workgroups at N = 400, 2 at 700; 4: whole-wave scan instances, 7 and 11 slots
    per lane): CoM RMSE ≤ 1e-9 and single solves ≤ 1e-7 relative, as the default-weight long
    fixtures (test_strict_long_horizon_*), every status 0."""
    d = golden("strict_weights_long_ref.npz")
    Qv, Rv, hv, gv = (float(v) for v in d["weights"][w])
    N = 400
    zx, zn = d[f"w{w}_n400_zmax"], d[f"w{w}_n400_zmin"]
    n = len(zx)
    p = Plan(torch.cuda.current_device(), N, 1.5 / N, hv, gv, Qv, Rv, True)
    p.set_option("strict_solver", solver)
    x0 = np.stack([d[f"w{w}_n400_x0"], d[f"w{w}_n400_y0"]])[None]
    h, st = p.rollout(zx, zn, x0, kick=np.array([float(d[f"w{w}_n400_kick"])]), kick_step=n // 2)
    assert int(st.abs().max()) == 0
    h = h.cpu().numpy()[0]
    assert rmse(h[:, :, 0], d[f"w{w}_n400_com"]) <= 1e-9
    assert np.abs(h[:, 1] - d[f"w{w}_n400_yhist"]).max() <= 1e-6
    N = 700
    p = Plan(torch.cuda.current_device(), N, 1.5 / N, hv, gv, Qv, Rv, True)
    p.set_option("strict_solver", solver)
    out, st = p.step(d[f"w{w}_step700_x"], d[f"w{w}_step700_zmax"], d[f"w{w}_step700_zmin"])
    ref = d[f"w{w}_step700_out"]
    assert int(st.abs().max()) == 0
    assert np.abs(out.cpu().numpy() - ref).max() <= 1e-7 * max(1.0, np.abs(ref).max())


@pytest.mark.parametrize("w", (0, 2))
def test_strict_weights_drop_in(w):
    """The drop-in at non-default weights: ZMPController(MPCConfig(Q, R, h, g, strict=True))
    .generate_com_trajectory on the default walk equals the reference-driven strict rollout
    (strict_weights_ref.npz) at ≤ 1e-9 CoM RMSE."""
    d = golden("strict_weights_ref.npz")
    Qv, Rv, hv, gv = (float(v) for v in d["weights"][w])
    c = ZMPController(MPCConfig(horizon=150, strict=True, add_force=True, F_ext=400.0, Q=Qv,
                                R=Rv, h=hv, g=gv))
    com, y_hist = c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                            d[f"w{w}_n150_zmax"], d[f"w{w}_n150_zmin"])
    assert rmse(com, d[f"w{w}_n150_com"]) <= 1e-9
    assert rmse(y_hist[:, :, 0] @ c.C, d[f"w{w}_n150_yhist"] @ c.C) <= 1e-9


@pytest.mark.parametrize("B,auto", ((2, 4), (300, 4), (2100, 4), (8192, 4), (8200, 3)))
def test_strict_small_and_large_batch_paths_agree(B, auto):
    """The automatic choice (ZMPC_OPT_STRICT_SOLVER = 0) takes the parallel-in-time kernel up to
    16384 instances (whole waves per instance up to one per SIMD, 32 lanes beyond) and the
    LQ kernel beyond; on config-3 style batches the small-batch kernels
    (forced) and the LQ kernel give the same histories to rounding, and the automatic one equals
    the chosen kernel's bitwise."""
    zmax, zmin, x0, F, dt = synthetic_batch(B, 150, seed=41)
    n = zmax.shape[1]
    kick = dt * F / M
    outs = {}
    for solver in ((0, 2, 3, 4) if B <= 300 else (0, 3, 4)):
        h, st = plan(150, strict=True, dt=dt).set_option("strict_solver", solver).rollout(
            zmax, zmin, x0, kick=kick, kick_step=n // 2)
        assert int(st.abs().max()) == 0
        outs[solver] = h.cpu().numpy()
    assert np.array_equal(outs[0], outs[auto])
    for sv in outs:
        assert np.abs(outs[sv] - outs[3]).max() <= 1e-9, sv
        assert rmse(outs[sv][..., 0], outs[3][..., 0]) <= 1e-12, sv


@pytest.mark.parametrize("N,B", ((1, 3), (2, 5), (63, 7), (65, 7), (20, 600), (40, 600),
                                 (129, 1100), (257, 5), (300, 600), (400, 600), (512, 3),
                                 (512, 600), (513, 3), (700, 1100), (960, 2)))
def test_strict_scan_kernel_chunk_widths(N, B):
    """The parallel-in-time kernel at the edges of its chunk widths (C = ⌈N/64⌉ = 1..15 slots
    per lane; N = 65/129/513 leave the last lane one slot, N = 1 a single lane, N = 960 the
    widest whole-wave chunk) and with 32 lanes per
    instance (beyond one instance per SIMD: B = 600 walks at N = 20 / 40, 1 and 2 slots per lane
    of 32; B = 1100 at N = 129; B = 600 at N = 300 / 400 / 512: 10 / 13 / 16 slots per lane of
    32; past N = 512 whole waves again, B = 1100 at N = 700 in two dispatch rounds) against the
    LQ kernel on
    the same kicked walks: CoM within 1e-9, same statuses; and one window-mode step."""
    zmax, zmin, x0, F, dt = synthetic_batch(B, 64 if N < 150 else 150, seed=N)
    n = zmax.shape[1]
    kick = dt * F / M
    outs = []
    for sv in (4, 3):
        p = plan(N, strict=True, dt=dt).set_option("strict_solver", sv)
        h, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
        outs.append((h.cpu().numpy(), st.cpu().numpy()))
        xw = x0[:, 1, :]
        idx = np.minimum(np.arange(N), n - 1)
        o, sts = p.step(xw, zmax[:, idx, 1], zmin[:, idx, 1])
        outs.append((o.cpu().numpy(), sts.cpu().numpy()))
    (h4, s4), (o4, t4), (h3, s3), (o3, t3) = outs
    assert np.array_equal(s4, s3) and int(np.abs(s4).max()) == 0
    assert np.abs(h4[..., 0] - h3[..., 0]).max() <= 1e-9
    assert np.array_equal(t4, t3)
    assert np.abs(o4 - o3).max() <= 1e-9 * max(1.0, np.abs(o3).max())


@pytest.mark.parametrize("N,n", ((512, 1431), (150, 1100), (150, 2500), (256, 1000),
                                 (200, 3000)))
def test_fft_correlation_equals_direct(N, n):
    """Long walks: the FFT correlation (rollout.hip, wide kernel; ZMPC_OPT_LONG_WALK = 2) and the
    direct form (= 1) on the same batch agree to rounding: max |Δ| ≤ 1e-11 on O(1) states
    (measured ≈1e-14); the automatic choice (FFT where (n − 1)·N ≥ 9·P·log2 P, e.g. N ≥ 200
    here) equals one of them exactly."""
    rng = np.random.default_rng(n)
    dt = 1.5 / N if N == 512 else 0.01
    B = 8
    zc = np.cumsum(rng.uniform(-0.01, 0.01, (B, n, 2)), axis=1)
    zmax, zmin = zc + 0.05, zc - 0.05
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    kick = dt * rng.uniform(0, 800, B) / M
    h = {}
    for form in (0, 1, 2):
        p = plan(N, dt=dt).set_option("long_walk", form)
        hh, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
        assert int(st.abs().max()) == 0
        h[form] = hh.cpu().numpy()
    assert np.abs(h[2] - h[1]).max() <= 1e-11
    assert np.array_equal(h[0], h[2]) or np.array_equal(h[0], h[1])


# ------------------------------------------------ plan build at long horizons


@pytest.mark.parametrize("N,strict", ((1000, False), (700, True), (2048, False)))
def test_plan_blocked_factorisation_long_horizon(N, strict):
    """The blocked Cholesky (16-column MFMA panels), the blocked gain solves and (strict) the
    blocked L⁻¹Puᵀ at horizons past a single panel row: L·Lᵀ = M, the gain row equals the
    oracle's dense solve, G = inv(Hz)."""
    dt = 1.5 / N
    p = plan(N, strict=strict)
    Px, Pu = O.prediction_matrices(N, dt, H, G)
    Mref = Pu.T @ Pu + R / Q * np.eye(N)
    M = p.export(_native.EXPORT_M)
    assert np.abs(M - Mref).max() <= 1e-13 * np.abs(Mref).max()
    Lf = p.export(_native.EXPORT_L)
    assert np.array_equal(np.triu(Lf, 1), np.zeros_like(Lf))
    assert np.abs(Lf @ Lf.T - Mref).max() <= 1e-12 * np.abs(Mref).max()
    k, kx = O.gain_row(N, dt, H, G, Q, R)
    assert np.abs(p.export(_native.EXPORT_K) - k).max() <= 1e-8 * np.abs(k).max()
    assert np.allclose(p.export(_native.EXPORT_KX), kx, rtol=1e-8, atol=0)
    t = p.timings()
    assert t["total"] > 0 and t["cholesky"] > 0 and t["gram_PuTPu"] > 0
    if strict:
        Hz, V, _, _ = O.strict_matrices(N, dt, H, G, Q, R)
        Gref = np.linalg.inv(Hz)
        assert np.abs(p.export(_native.EXPORT_G) - Gref).max() <= 1e-9 * np.abs(Gref).max()
        assert np.abs(p.export(_native.EXPORT_HZ) - Hz).max() <= 1e-9 * np.abs(Hz).max()


def test_plan_cache_bounded_and_destroy():
    from mpc_bipedal import solver
    solver.clear_plan_cache(destroy=True)
    for N in range(10, 10 + 10 * (solver.PLAN_CACHE_MAX + 3), 10):
        get_plan(MPCConfig(horizon=N))
    assert len(solver._PLAN_CACHE) == solver.PLAN_CACHE_MAX
    p = plan(32)
    p.destroy()
    p.destroy()  # idempotent
    with pytest.raises(RuntimeError, match="destroyed"):
        p.export(_native.EXPORT_K)


_ENV_CHILD = r"""
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
import torch
from mpc_bipedal.solver import Plan
d = np.load(sys.argv[2])
out = {}
for strict in (False, True):
    p = Plan(0, 150, float(d["dt"]), 0.75, 9.81, 1.0, 1e-6, strict)
    h, st = p.rollout(d["zmax"], d["zmin"], d["x0"], kick=d["kick"], kick_step=int(d["ks"]))
    out[f"h{int(strict)}"] = h.cpu().numpy()
    out[f"s{int(strict)}"] = st.cpu().numpy()
np.savez(sys.argv[3], **out)
"""


def test_environment_does_not_change_results(tmp_path):
    """Every environment switch earlier libraries read (diagnostic ablations that changed results
    while reporting success, A/B kernel variants) set to a non-default value in a subprocess:
    the product library's unconstrained and strict rollouts are bitwise those of a clean
    environment (the switches exist only in the diagnostics build)."""
    import subprocess
    import sys
    from test_host import _DIAG_ENV
    zmax, zmin, x0, F, dt = synthetic_batch(300, 150, seed=31)
    n = zmax.shape[1]
    inp = tmp_path / "in.npz"
    np.savez(inp, zmax=zmax, zmin=zmin, x0=x0, kick=dt * F / M, ks=n // 2, dt=dt)
    res = []
    for dirty in (False, True):
        env = {k: v for k, v in os.environ.items() if not k.startswith("ZMPC_")}
        if dirty:
            env.update({k: "7" for k in _DIAG_ENV})
            env.update(ZMPC_STRICT_LQ="4x3x4", ZMPC_STRICT_VARIANT="chol", ZMPC_FFT="1")
        out = tmp_path / f"o{int(dirty)}.npz"
        subprocess.run([sys.executable, "-c", _ENV_CHILD, PKG, str(inp), str(out)], env=env,
                       check=True, timeout=300)
        res.append(np.load(out))
    for k in ("h0", "s0", "h1", "s1"):
        assert np.array_equal(res[0][k], res[1][k]), k
    assert int(np.abs(res[0]["s1"]).max()) == 0
