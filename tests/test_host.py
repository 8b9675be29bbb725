"""Host-side logic that needs no GPU: config, model, input producer, C-ABI symbol table,
controller argument handling."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, PKG, golden

from mpc_bipedal.config import MPCConfig
from mpc_bipedal.generators import CoPGenerator, generate_footsteps
from mpc_bipedal.models.lipm_model import LIPMModel, lipm_matrices, prediction_matrices
from mpc_bipedal import _native

STATE_CODE = {"STANDING": 0, "DOUBLE_SUPPORT": 1, "SINGLE_SUPPORT": 2}


def test_config_defaults_match_reference():
    """Field defaults of config.py:13-87 and the dt rule of :84-87."""
    c = MPCConfig()
    assert c.horizon == 150 and c.dt == 1.5 / 150
    assert (c.Q, c.R, c.S, c.h, c.g, c.m, c.F_ext) == (1.0, 1e-6, 1.0, 0.75, 9.81, 40.0, 400.0)
    assert c.strict is True and c.add_force is True and c.method == "wieber"
    assert (c.ssp_duration, c.dsp_duration, c.standing_duration) == (0.24, 0.01, 0.5)
    assert (c.distance, c.step_length, c.foot_spread) == (2.1, 0.3, 0.1)
    assert len(c.left_foot_polytope) == 11 and len(c.right_foot_polytope) == 11
    assert MPCConfig(horizon=64).dt == 1.5 / 64
    assert MPCConfig(dt=0.02).dt == 0.02


@pytest.mark.parametrize("tag", ["default_n150", "default_n10", "default_n64", "default_n512",
                                 "classdefaults_n150", "long_n100", "short_n200"])
def test_cop_generator_bit_exact(tag):
    d = golden(f"cop_{tag}.npz")
    cfg = MPCConfig(horizon=int(d["horizon"]), dt=float(d["dt"]), distance=float(d["distance"]),
                    step_length=float(d["step_length"]), foot_spread=float(d["foot_spread"]),
                    ssp_duration=float(d["ssp_duration"]), dsp_duration=float(d["dsp_duration"]),
                    standing_duration=float(d["standing_duration"]))
    zx, zn, st = CoPGenerator(cfg).generate_cop_trajectory()
    assert np.array_equal(zx, d["zmax"]) and np.array_equal(zn, d["zmin"])
    assert np.array_equal(np.array([STATE_CODE[s.value] for s in st]), d["states"])


def test_footsteps():
    f = generate_footsteps(2.1, 0.3, 0.1)
    assert len(f) == 10
    assert f[0].y == -0.1 and f[1].y == 0.1 and f[-1].x == f[-2].x
    assert np.isclose(f[2].z_max[0] - f[2].z_min[0], 0.11)


@pytest.mark.parametrize("N", (10, 64, 150, 512))
def test_model_prediction_matrices_bit_exact(N):
    d = golden(f"predict_n{N}.npz")
    Px, Pu = prediction_matrices(N, float(d["dt"]), 0.75, 9.81)
    assert np.array_equal(Px, d["Px"]) and np.array_equal(Pu[:, 0], d["Pu_col0"])


def test_lipm_model():
    cfg = MPCConfig()
    m = LIPMModel(cfg)
    A, B, C = lipm_matrices(cfg.dt, cfg.h, cfg.g)
    assert m.get_state_dimension() == 3
    x = np.array([[0.1], [0.2], [0.3]])
    assert np.array_equal(m.step(x, 2.0), A @ x + B * 2.0)
    assert np.allclose(m.get_zmp(x[:, 0]), 0.1 - 0.75 / 9.81 * 0.3)


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "zmpc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zmpc_[a-z_]+)\s*\(", src)))


def test_header_and_binding_agree():
    syms = _header_symbols()
    assert set(syms) == set(_native.SIGNATURES), syms


def test_library_loads_and_exports_every_symbol():
    """The C-ABI library loads without a GPU and exports every declared entry point."""
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libzmpc.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_native.LIB_PATH)
    for s in _header_symbols():
        assert hasattr(lib, s), s
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True,
                         text=True).stdout
    exported = set(re.findall(r" T (zmpc_\w+)", out))
    assert set(_header_symbols()) <= exported
    lib = _native.load()
    assert lib.zmpc_abi_version() == _native.ABI_VERSION == 7
    assert lib.zmpc_last_error() == b""


def test_argument_errors_without_gpu():
    """Argument validation happens before any device call and reports through last_error."""
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libzmpc.so not built")
    lib = _native.load()
    h = ctypes.c_void_p()
    rc = lib.zmpc_plan_create(0, 0, 0.01, 5e-5, 1.6e-7, 0.07, 7e-4, 1.0, 1e-6, 0, None,
                              ctypes.byref(h))
    assert rc == _native.ZMPC_EINVAL and b"horizon" in lib.zmpc_last_error()
    rc = lib.zmpc_rollout(None, 1, 10, None, None, 20, None, None, -1, None, None, None)
    assert rc == _native.ZMPC_EINVAL
    rc = lib.zmpc_step(None, 1, None, None, None, None, None, None)
    assert rc == _native.ZMPC_EINVAL
    rc = lib.zmpc_rollout_kicks(None, 1, 10, None, None, 20, None, None, None, None, None, None)
    assert rc == _native.ZMPC_EINVAL and b"kick_steps" in lib.zmpc_last_error()
    rc = lib.zmpc_cop_generate(0, -1, None, 0, None, None, None, None, None)
    assert rc == _native.ZMPC_EINVAL
    rc = lib.zmpc_cop_generate(0, 4, None, 0, None, None, None, None, None)
    assert rc == _native.ZMPC_EINVAL and b"params" in lib.zmpc_last_error()
    buf = (ctypes.c_uint64 * _native.NCOUNTERS)()
    rc = lib.zmpc_plan_counters(None, buf, _native.NCOUNTERS, 0)
    assert rc == _native.ZMPC_EINVAL and b"NULL" in lib.zmpc_last_error()
    rc = lib.zmpc_herdt_rollout(None, None, 1, 10, None, 0, None, 0, None, 0, None, None, -1,
                                None, None, None, None)
    assert rc == _native.ZMPC_EINVAL and b"NULL" in lib.zmpc_last_error()
    rc = lib.zmpc_herdt_step(None, None, 1, None, None, None, None, None, None, None, None,
                             None, None)
    assert rc == _native.ZMPC_EINVAL
    tbuf = (ctypes.c_float * _native.PLAN_STAGES)()
    rc = lib.zmpc_plan_timings(None, tbuf, _native.PLAN_STAGES)
    assert rc == _native.ZMPC_EINVAL and b"NULL" in lib.zmpc_last_error()
    rc = lib.zmpc_plan_set_option(None, 0, 0)
    assert rc == _native.ZMPC_EINVAL and b"NULL" in lib.zmpc_last_error()


# environment variables that earlier libraries read to select A/B variants or diagnostic
# ablations (some of which changed results while reporting success)
_DIAG_ENV = ("ZMPC_DEBUG_LQ", "ZMPC_DEBUG_ROLLOUT", "ZMPC_DEBUG_PLAN", "ZMPC_DEBUG_STRICT",
             "ZMPC_ROLLOUT_VARIANT", "ZMPC_STRICT_LQ", "ZMPC_STRICT_NT", "ZMPC_STRICT_WARM",
             "ZMPC_STRICT_LQ_DRIFT", "ZMPC_STRICT_ORDER", "ZMPC_STRICT_VARIANT", "ZMPC_SPARSE_CORR",
             "ZMPC_FFT", "ZMPC_NO_FFT", "ZMPC_ROLLOUT_NO_WIDE", "ZMPC_NO_SHARED_F",
             "ZMPC_PREFETCH", "ZMPC_PF_ROUNDS", "ZMPC_PERS_PER_CU", "ZMPC_HERDT_WARM",
             "ZMPC_HERDT_PROF", "ZMPC_STRICT_LDS_G", "ZMPC_STRICT_LDS_CHOL")


def test_product_library_reads_no_result_changing_environment():
    """The product libzmpc.so contains no diagnostic / variant switch: the only environment
    variable it names is ZMPC_POOL_KEEP_MB (memory retention of the stream-ordered pool).
    Algorithm choices are explicit plan options (zmpc_plan_set_option); ablations live in the
    separate diagnostics build (make diag).  tests/test_gpu_parity.py
    test_environment_does_not_change_results runs a rollout with every old switch set."""
    if not os.path.exists(_native.LIB_PATH):
        pytest.skip("libzmpc.so not built")
    blob = open(_native.LIB_PATH, "rb").read()
    names = set(re.findall(rb"ZMPC_[A-Z0-9_]+", blob))
    assert names <= {b"ZMPC_POOL_KEEP_MB"}, names
    for v in _DIAG_ENV:
        assert v.encode() not in blob, v
    assert b"getenv" in blob  # (the one read above)


def test_router_errors():
    from mpc_bipedal.controllers import ZMPController
    c = ZMPController(MPCConfig())
    with pytest.raises(ValueError, match="z_max and z_min are required"):
        c.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)))
    c2 = ZMPController(MPCConfig(method="herdt"))
    with pytest.raises(ValueError, match="v_ref and state_ref"):
        c2.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)))
    if not __import__("torch").cuda.is_available():
        # the Herdt QP runs on the device only: no CPU fallback behind the drop-in
        with pytest.raises(RuntimeError, match="HIP device"):
            c2.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                       v_ref=np.zeros((5, 2)), state_ref=[0] * 5)
    c3 = ZMPController(MPCConfig(method="foo"))
    with pytest.raises(ValueError, match="Unknown method"):
        c3.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)))
    assert np.array_equal(c.C, np.array([1.0, 0.0, -0.75 / 9.81]))


def test_product_has_no_oracle_or_cpu_solver_import():
    """The product package never imports the oracle (test infrastructure only)."""
    for dirpath, _, files in os.walk(os.path.join(PKG, "mpc_bipedal")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in src.replace("no oracle", ""), f
                assert "linalg.inv" not in src and "linalg.solve" not in src, f


def test_speed_generator_classic_and_errors():
    """speed_generation.py:49-53 (classic: 0.3 m/s except STANDING) and :67 (unknown mode),
    on the golden CoP state timeline."""
    from mpc_bipedal.generators import SpeedTrajectoryGenerator, State
    d = golden("cop_default_n150.npz")
    cfg = MPCConfig(horizon=int(d["horizon"]), dt=float(d["dt"]), distance=float(d["distance"]),
                    step_length=float(d["step_length"]), foot_spread=float(d["foot_spread"]),
                    ssp_duration=float(d["ssp_duration"]), dsp_duration=float(d["dsp_duration"]),
                    standing_duration=float(d["standing_duration"]), speed_generation="classic")
    vx, vy, st = SpeedTrajectoryGenerator(cfg).generate_speed_and_state(save_footsteps=False)
    standing = d["states"] == STATE_CODE[State.STANDING.value]
    assert np.array_equal(vx, np.where(standing, 0.0, 0.3)) and not vy.any()
    assert len(st) == len(d["states"])
    bad = SpeedTrajectoryGenerator(MPCConfig(speed_generation="nope"))
    with pytest.raises(ValueError, match="Unknown speed_generation mode"):
        bad.generate_speed_and_state(save_footsteps=False)


def test_cli_config_semantics(tmp_path):
    """run_mpc.py:23-40,153-221 semantics in mpc_bipedal.cli: only the
    "mpc" section is read, a lone dt sets horizon = int(1.5/dt), dt is always 1.5/horizon,
    flags override the file, --no-strict / --no-add-force."""
    import json
    from mpc_bipedal import cli
    f = tmp_path / "c.json"
    f.write_text(json.dumps({"cop_generator": {"distance": 9.9},
                             "mpc": {"dt": 0.02, "Q": 2.0, "strict": True}}))
    c = cli.config_from_args(cli.build_parser().parse_args(["--config", str(f)]))
    assert c.horizon == 75 and c.dt == 1.5 / 75 and c.Q == 2.0 and c.distance == 2.1
    c = cli.config_from_args(cli.build_parser().parse_args(
        ["--config", str(f), "--horizon", "64", "--no-strict", "--no-add-force", "--F-ext", "7",
         "--distance", "3.0"]))
    assert c.horizon == 64 and c.dt == 1.5 / 64 and not c.strict and not c.add_force
    assert c.F_ext == 7.0 and c.distance == 3.0 and c.backend == "hip"
    c = cli.config_from_args(cli.build_parser().parse_args(["--config", str(f), "--dt", "0.05"]))
    assert c.horizon == 30 and c.dt == 1.5 / 30
