#!/usr/bin/env python3
"""Benchmark: QP solves/s of the batched Wieber LIPM-ZMP MPC on MI355X.

Workload (BASELINE.json configs[1]): per GPU, a batch of B = 4096
default.json walks (n = 420 CoP samples, horizon N = 150, dt = 0.01, unconstrained solve),
each with a rigid CoP offset δ_b ~ U(−0.02, 0.02)² m, x0 position ~ U(−0.01, 0.01) and an
F_ext_b ~ U(0, 800) N kick at step n//2; walk 0 is the reference walk (δ = 0, x0 = 0,
F = 400 N).  One "step" of this bench = one batched rollout of every walk over all n−1
timesteps and both axes = B·(n−1)·2 QP solves, inputs already resident in HBM.

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling, each rank rolls out its own
4096-walk block with no data-path collective; the CoM all-gather that reassembles the full
trajectories is timed separately (allgather_ms), outside `value`.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "model-predictive-control-for-bipedal-locomotion_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from mpc_bipedal.config import MPCConfig  # noqa: E402
from mpc_bipedal.generators import CoPGenerator  # noqa: E402
from mpc_bipedal.solver import Plan  # noqa: E402
from mpc_bipedal.distributed import allgather_walks  # noqa: E402

# configs/default.json "mpc" section of the reference (the fields the CoP producer and the
# Wieber hot path read)
DEFAULT_JSON = dict(ssp_duration=0.24, dsp_duration=0.03, standing_duration=1.0, distance=2.1,
                    step_length=0.3, foot_spread=0.1, horizon=150, Q=1.0, R=1e-6, S=1.0, h=0.75,
                    g=9.81, m=40.0, F_ext=400.0, strict=True, add_force=True)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFS = 78.6    # FP64 vector = matrix peak (spec)
SEED = 20251226


def make_batch(B, rank, cfg, strict):
    zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory()
    rng = np.random.default_rng(SEED + 7919 * rank)
    off = rng.uniform(-0.02, 0.02, (B, 1, 2))
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    F = rng.uniform(0.0, 800.0, B)
    if rank == 0:
        off[0], x0[0], F[0] = 0.0, 0.0, 400.0   # the reference walk
    return zmax, zmin, zmax[None] + off, zmin[None] + off, x0, F


def cpu_baseline(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg, budget_s):
    """Reference-faithful NumPy port (oracle/zmp_oracle.py:predict_wieber_axis_ref: the
    interpreted Px/Pu build + np.linalg.inv of zmp_controller.py:162-199, per solve), one
    BLAS thread, on whole walks of the same batch until `budget_s` of CPU work is spent."""
    from oracle import zmp_oracle as O
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        return _cpu_baseline(O, zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg, budget_s)


def _cpu_baseline(O, zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg, budget_s):
    N, dt = cfg.horizon, cfg.dt
    solves, elapsed, walks, rms = 0, 0.0, 0, []
    b = 1
    while elapsed < budget_s and b < len(zmax_b):
        n = zmax_b.shape[1]
        zx = np.vstack([zmax_b[b], np.tile(zmax_b[b, -1:], (N, 1))])
        zn = np.vstack([zmin_b[b], np.tile(zmin_b[b, -1:], (N, 1))])
        x = x0_b[b, 0].reshape(3, 1).copy()
        y = x0_b[b, 1].reshape(3, 1).copy()
        com = [[x[0, 0], y[0, 0]]]
        t0 = time.perf_counter()
        for i in range(n - 1):
            x = O.predict_wieber_axis_ref(x, N, zx[i + 1:i + 1 + N, 0:1], zn[i + 1:i + 1 + N, 0:1],
                                          dt, cfg.h, cfg.g, cfg.Q, cfg.R)
            y = O.predict_wieber_axis_ref(y, N, zx[i + 1:i + 1 + N, 1:2], zn[i + 1:i + 1 + N, 1:2],
                                          dt, cfg.h, cfg.g, cfg.Q, cfg.R)
            if i == n // 2:
                y = y - np.array([[0.0, kick_b[b], 0.0]]).T
            com.append([x[0, 0], y[0, 0]])
        elapsed += time.perf_counter() - t0
        solves += 2 * (n - 1)
        rms.append(float(np.sqrt(np.mean((np.array(com) - hist_gpu[b, :, :, 0]) ** 2))))
        walks += 1
        b += 1
    return dict(value=solves / elapsed, unit="QP solves/s", cores=1, kind="port",
                sample=f"{walks} full walk(s) = {solves} solves of this batch (walks 1..{walks}), "
                       "reference-faithful NumPy port (interpreted Pu build + np.linalg.inv "
                       "per solve, zmp_controller.py:162-199), 1 BLAS thread",
                seconds=elapsed, com_rmse_gpu_vs_port=max(rms) if rms else None)


def pmc_traffic(workload):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_<workload>.json, written by profiles/collect_pmc.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="walks per GPU")
    ap.add_argument("--horizon", type=int, default=150)
    ap.add_argument("--strict", action="store_true", help="strict ZMP box constraints (config 3)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    d = dict(DEFAULT_JSON)
    d["horizon"] = args.horizon
    d["strict"] = bool(args.strict)
    cfg = MPCConfig(**d)  # dt = 1.5 / horizon
    B = args.batch
    cop_x, cop_n, zmax_h, zmin_h, x0_h, F_h = make_batch(B, rank, cfg, args.strict)
    n = zmax_h.shape[1]
    kick_h = cfg.dt * F_h / cfg.m
    plan = Plan(dev.index, cfg.horizon, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, cfg.strict)
    zmax = torch.as_tensor(zmax_h, device=dev)
    zmin = torch.as_tensor(zmin_h, device=dev)
    x0 = torch.as_tensor(x0_h, device=dev)
    kick = torch.as_tensor(kick_h, device=dev)
    hist = torch.empty((B, n, 2, 3), dtype=torch.float64, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    kstep = n // 2

    launch = plan.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=kstep, hist=hist,
                                   status=status)
    for _ in range(args.warmup):
        launch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        launch()
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    assert int(status.abs().max()) == 0, "solver reported a failed instance"

    solves_per_step = B * (n - 1) * 2 * world
    value = solves_per_step * args.steps / elapsed
    # algorithmic bytes of one launch: bounds in (2 × [B,n,2] f64) + history out ([B,n,2,3])
    alg_bytes = 2 * B * n * 2 * 8 + B * n * 6 * 8
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    flops = B * (n - 1) * 2 * (2 * cfg.horizon + 20)
    gemm_tf = B * (n - 1) * 2 * 2 * cfg.horizon ** 2 / (kern_ms * 1e-3) / 1e12
    workload = ("config3_strict" if args.strict else "config2") + f"_n{cfg.horizon}_b{B}"

    # parity in the same run: the reference walk (walk 0 of rank 0) vs the committed
    # reference fixture (tests/golden: produced by the reference itself)
    com_rmse_ref = None
    if rank == 0 and cfg.horizon == 150:
        fx = np.load(os.path.join(ROOT, "tests", "golden", "walk_n150.npz"))
        ref_com = fx["com_force"]
        if not args.strict and ref_com.shape[0] == n:
            com_rmse_ref = float(np.sqrt(np.mean(
                (hist[0, :, :, 0].cpu().numpy() - ref_com) ** 2)))

    gather_ms = None
    if world > 1:
        com = hist[..., 0].contiguous()
        torch.cuda.synchronize()
        dist.barrier()
        tg = time.perf_counter()
        full = allgather_walks(com, B * world)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        assert full.shape[0] == B * world

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.strict:
        cpu = cpu_baseline(zmax_h, zmin_h, x0_h, kick_h, hist.cpu().numpy(), cfg,
                           args.cpu_seconds)

    if rank == 0:
        traffic = pmc_traffic(workload)
        if not args.strict:
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS}
        else:
            # strict: the per-step z-space GEMM D = G·W (2N² FLOP per solve) bounds it
            roof = {"bound": "mfma", "achieved": gemm_tf, "peak": FP64_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": gemm_tf / FP64_PEAK_TFS}
        roof.update({
            "traffic": traffic,
            "kernel": "zmpc_strict_kernel" if args.strict else "zmpc_rollout_unc_kernel",
            "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes,
            "hbm_gbs": achieved, "alg_flops_per_launch": flops,
            "fp64_frac_alg": flops / (kern_ms * 1e-3) / (FP64_PEAK_TFS * 1e12)})
        line = {
            "metric": "QP solves/sec (horizon=150, batched) at 1/2/4/8 MI355X; CoM RMSE vs ref",
            "value": value,
            "unit": "QP solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (default.json CoP + seeded offsets/x0/F_ext, SURVEY.md §8d)",
            "config": {
                "workload": ("config3: B strict walks" if args.strict else
                             "config2: B default.json walks, unconstrained") +
                            f", horizon={cfg.horizon}, n={n}",
                "walks_per_gpu": B, "global_batch": B * world, "horizon": cfg.horizon,
                "samples_per_walk": n, "solves_per_step": solves_per_step,
                "parallelism": f"dp{world}", "strict": bool(args.strict),
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "com_rmse_vs_ref": com_rmse_ref,
            "allgather_ms": gather_ms,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
