"""Command line driver with the reference's ``scripts/run_mpc.py`` semantics (SURVEY.md §8f
row 4): same flags, the same JSON loading (only the ``"mpc"`` section is read,
``run_mpc.py:23-40``), the same override rules (``:153-221`` — dt is always recomputed as
1.5/horizon), the same configuration printout, then the Wieber rollout on the device.

Additions: ``--backend`` (only ``hip``: there is no CPU solver in this build), ``--batch B``
(B walks in one device rollout, F_ext swept linearly over [0, 2·F_ext]) and ``--save FILE``
(npz with the CoP bounds, CoM and ZMP histories).  Plotting (plotly) is not part of this
build: ``--no-visualization`` is implied.

    python -m mpc_bipedal.cli --config configs/default.json --batch 4096 --save out.npz
"""
import argparse
import json
import os
import sys
import time

import numpy as np

from .config import MPCConfig


def load_config_from_json(config_file: str) -> MPCConfig:
    """run_mpc.py:23-40: the "mpc" section; a lone dt becomes horizon = int(1.5/dt)."""
    with open(config_file, "r") as f:
        config_dict = json.load(f)
    mpc_dict = config_dict.get("mpc", {}).copy()
    if "dt" in mpc_dict:
        dt_value = mpc_dict.pop("dt")
        if "horizon" not in mpc_dict:
            mpc_dict["horizon"] = int(1.5 / dt_value)
    return MPCConfig(**mpc_dict)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MPC bipedal locomotion (MI355X backend)")
    p.add_argument("--config", type=str, help="JSON configuration file")
    for name, dest in (("--distance", "distance"), ("--step-length", "step_length"),
                       ("--foot-spread", "foot_spread"), ("--ssp-duration", "ssp_duration"),
                       ("--dsp-duration", "dsp_duration"),
                       ("--standing-duration", "standing_duration"), ("--dt", "dt"),
                       ("--Q", "Q"), ("--R", "R"), ("--S", "S"), ("--h", "h"), ("--m", "m"),
                       ("--F-ext", "F_ext"), ("--alpha", "alpha"), ("--beta", "beta"),
                       ("--gamma", "gamma"), ("--vx-ref", "vx_ref"), ("--vy-ref", "vy_ref"),
                       ("--foot-length", "foot_length"), ("--foot-width", "foot_width")):
        p.add_argument(name, type=float, dest=dest)
    p.add_argument("--horizon", type=int)
    p.add_argument("--strict", action="store_true", default=None)
    p.add_argument("--no-strict", action="store_true", dest="no_strict")
    p.add_argument("--add-force", action="store_true", default=None)
    p.add_argument("--no-add-force", action="store_true", dest="no_add_force")
    p.add_argument("--method", type=str, choices=["wieber", "herdt"])
    p.add_argument("--no-visualization", action="store_true")
    p.add_argument("--output-dir", type=str, default="results")
    p.add_argument("--backend", type=str, default="hip", choices=["hip"])
    p.add_argument("--batch", type=int, default=1, help="walks per device rollout")
    p.add_argument("--save", type=str, default=None, help="npz output file")
    return p


def config_from_args(args) -> MPCConfig:
    """run_mpc.py:140-221 override semantics."""
    if args.config:
        config = load_config_from_json(args.config)
    elif os.path.exists("configs/default.json"):
        config = load_config_from_json("configs/default.json")
    else:
        config = MPCConfig()
    for k in ("distance", "step_length", "foot_spread", "ssp_duration", "dsp_duration",
              "standing_duration"):
        if getattr(args, k) is not None:
            setattr(config, k, getattr(args, k))
    if args.horizon is not None:
        config.horizon = args.horizon
        config.dt = 1.5 / config.horizon
    elif args.dt is not None:
        config.horizon = int(1.5 / args.dt)
        config.dt = 1.5 / config.horizon
    else:
        config.dt = 1.5 / config.horizon
    for k in ("Q", "R", "S", "h", "m", "F_ext", "alpha", "beta", "gamma", "vx_ref", "vy_ref",
              "foot_length", "foot_width"):
        if getattr(args, k) is not None:
            setattr(config, k, getattr(args, k))
    if args.strict:
        config.strict = True
    elif args.no_strict:
        config.strict = False
    if args.add_force:
        config.add_force = True
    elif args.no_add_force:
        config.add_force = False
    if args.method is not None:
        config.method = args.method
    config.backend = args.backend
    return config


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    config = config_from_args(args)
    from .controllers import ZMPController
    from .generators import CoPGenerator

    print("=" * 60)
    print("MPC configuration (MI355X backend)")
    print("=" * 60)
    print(f"  Distance: {config.distance} m   Step length: {config.step_length} m   "
          f"Foot spread: {config.foot_spread} m   dt: {config.dt} s")
    print(f"  Method: {config.method}   Horizon: {config.horizon}   Q: {config.Q}   "
          f"R: {config.R}   h: {config.h} m   m: {config.m} kg   F_ext: {config.F_ext} N")
    print(f"  Strict: {config.strict}   Add force: {config.add_force}   "
          f"Batch: {args.batch}")
    print("=" * 60)
    if config.method.lower() != "wieber":
        raise NotImplementedError("only the Wieber method runs on this backend")
    z_max, z_min, _ = CoPGenerator(config).generate_cop_trajectory(output_dir=args.output_dir)
    controller = ZMPController(config)
    t0 = time.perf_counter()
    if args.batch <= 1:
        com, y_hist = controller.generate_com_trajectory(np.zeros((3, 1)), np.zeros((3, 1)),
                                                         z_max, z_min)
        com_b = com[None]
        zmp_y = np.tensordot(y_hist[:, :, 0], controller.C, axes=([1], [0]))[None]
    else:
        F = np.linspace(0.0, 2.0 * config.F_ext, args.batch) if config.add_force else None
        x0 = np.zeros((args.batch, 2, 3))
        com_t, hist = controller.generate_com_trajectory_batch(x0, z_max, z_min, F_ext=F)
        com_b = com_t.cpu().numpy()
        zmp_y = controller.zmp(hist[:, :, 1, :]).cpu().numpy()
    dt_s = time.perf_counter() - t0
    n = z_max.shape[0]
    print(f"CoM trajectory: {com_b.shape} ({args.batch} walk(s) × {n} samples) in "
          f"{dt_s * 1e3:.1f} ms")
    if args.save:
        os.makedirs(os.path.dirname(os.path.abspath(args.save)), exist_ok=True)
        np.savez(args.save, z_max=z_max, z_min=z_min, com=com_b, zmp_y=zmp_y)
        print(f"saved {args.save}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
