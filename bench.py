#!/usr/bin/env python3
"""Benchmark: QP solves/s of the batched Wieber LIPM-ZMP MPC on MI355X.

Workloads (`--config`, default 2 = BASELINE.json's metric configuration):
  2  per GPU B = 4096 default.json walks (n = 420 CoP samples, horizon N = 150, dt = 0.01),
     unconstrained; each walk a rigid CoP offset δ_b ~ U(−0.02, 0.02)² m, x0 position
     ~ U(−0.01, 0.01), an F_ext_b ~ U(0, 800) N kick at step n//2; walk 0 is the reference
     walk (δ = 0, x0 = 0, F = 400 N).
  3  as 2 with strict = True (box-constrained QP), per GPU B = 65536.
  4  Monte-Carlo F_ext: one shared default.json CoP broadcast to every scenario
     (bounds_stride 0), x0 = 0, F ~ U(0, 800) N, strict; per GPU 125 000 scenarios
     (`--unconstrained` for the unconstrained variant).
  5  horizon N = 512 (dt = 1.5/512, n = 1431), offsets as 2, unconstrained, per GPU 2048.
  6  Herdt joint footstep QP (method = "herdt"): the reference's default
     Herdt walk (MPCConfig defaults, classic speed references, n = 302) shared by every walk,
     x0 position ~ U(−0.01, 0.01) per axis, F_ext ~ U(0, 800) N at n//2; per GPU B = 32768
     (one (walk, axis) per lane: 1024 waves, one per SIMD);
     one solve = one joint x/y QP (predict_herdt_joint).
One "step" = one batched rollout of every walk over all n−1 timesteps and both axes
= B·(n−1)·2 QP solves, inputs already resident in HBM.

Multi-GPU (torchrun, one process per GPU, RCCL): weak scaling, each rank rolls out its own
block of walks with no data-path collective; the CoM all-gather that reassembles the full
trajectories is timed separately (allgather_ms), outside `value`.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
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
from mpc_bipedal.distributed import allgather_walks, shard_range  # noqa: E402

# configs/default.json "mpc" section of the reference (the fields the CoP producer and the
# Wieber hot path read)
DEFAULT_JSON = dict(ssp_duration=0.24, dsp_duration=0.03, standing_duration=1.0, distance=2.1,
                    step_length=0.3, foot_spread=0.1, horizon=150, Q=1.0, R=1e-6, S=1.0, h=0.75,
                    g=9.81, m=40.0, F_ext=400.0, strict=True, add_force=True)
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFS = 78.6    # FP64 vector = matrix peak (spec)
FP64_SUSTAINED_TFS = 56.6  # profiles/r1_fp64_peak.log: register-only FMA chains, 8 waves/SIMD
SEED = 20251226
SPARSE_MAX = 40  # rollout.hip kSparseMax: z_ref changes per axis the sparse correlation takes
SPARSE_MAX_WIDE = 64  # kSparseMaxWide: the same for the wide kernel (walks > 513 samples)
# strict_lq.hip FLOP per instance-slot of one active-set pass (fma = 2, the z-input form of
# strict_eta.h, round 5): working-set slot = Riccati step 70 (its shared part 22, 1/Quu 9, the
# law 10, the P/s update 29) + forward 13 + costate and multiplier 13; free-tail slot = s
# recursion 13 + forward 13.  (The v-input form of rounds 1-4 counted 160 and 44.)
STRICT_FLOP_WS = 96
STRICT_FLOP_TAIL = 26


CONFIGS = {
    2: dict(batch=4096, horizon=150, strict=False, shared=False),
    3: dict(batch=65536, horizon=150, strict=True, shared=False),
    4: dict(batch=125000, horizon=150, strict=True, shared=True),
    5: dict(batch=2048, horizon=512, strict=False, shared=False),
    6: dict(batch=32768, horizon=150, strict=False, shared=True, herdt=True),
}


def fft_transform(n, N):
    """Transform size P of the FFT correlation if zmpc_rollout takes it for this shape (the wide
    kernel's rule in csrc/rollout.hip), else None."""
    ns = n - 1
    if ns <= 512 or ns > 4096:
        return None
    W = 2 if ns <= 1024 else (4 if ns <= 2048 else 8)
    cw = -(-ns // (64 * W))
    kc = -(-N // cw) * cw
    lz = W * 64 * cw + kc + 1
    lzp = ((lz + (1 if cw % 2 == 0 else 0) * (lz // cw) + 1) + 1) & ~1
    if 2 * lzp * 8 > 64 * 1024:
        return None
    P = 256
    while P < ns + N:
        P *= 2
    E = P // (128 * W) if P % (128 * W) == 0 else 0
    if E not in (4, 8) or P > 8192 or P * 16 > 64 * 1024:
        return None
    if ns * N < 9 * P * int(np.log2(P)):  # measured crossover: the direct form is faster
        return None
    return P


def rollout_kernel_name(B, n, N, strict, shared=False):
    """Which kernel zmpc_rollout launches for this shape (csrc/rollout.hip launch rules)."""
    if strict:
        return "zmpc_strict_lq_kernel"
    if shared and n - 1 <= 512 and 6 * n * 8 <= 64 * 1024:
        return "zmpc_rollout_unc_splitd_kernel<CW, true> (+ zmpc_shared_f_kernel)"
    if fft_transform(n, N):
        return ("zmpc_rollout_unc_wide_kernel<CW, W, E> (sparse-difference correlation; FFT "
                "for dense bounds)")
    if n - 1 <= 512:
        # chunk width as rollout.hip:pick_cw; odd widths take the fast-FIR correlation, one walk
        # per workgroup
        cw = min(range(8, 0, -1), key=lambda c: (-(-(n - 1) // (64 * c)) * c, -c))
        if cw % 2 == 1:
            return "zmpc_rollout_unc_splitd_kernel"
        slots = 8 * torch.cuda.get_device_properties(0).multi_processor_count
        return ("zmpc_rollout_unc_persd_kernel" if slots < B <= 3 * slots
                else "zmpc_rollout_unc_splitd_kernel")
    return "zmpc_rollout_unc_wide_kernel" if n - 1 <= 4096 else "zmpc_rollout_unc_chunk_kernel"


def herdt_bench(args, rank, world, dev, dist_on):
    """config 6: batched Herdt rollouts (csrc/herdt.hip); returns the JSON line (rank 0)."""
    from mpc_bipedal.controllers import herdt as H
    from mpc_bipedal.generators import SpeedTrajectoryGenerator
    cfg = MPCConfig(method="herdt", add_force=True, horizon=args.horizon or 150)
    B = args.batch or CONFIGS[6]["batch"]
    vx, vy, states = SpeedTrajectoryGenerator(cfg).generate_speed_and_state(save_footsteps=False)
    v_ref = np.stack([vx, vy], 1)
    st = H.encode_states(states)
    n, N = len(st), cfg.horizon
    pad = H.pad_states(st, N)
    nb = np.array([t[0] for t in H.find_nb_steps(pad)][:n], np.int32)
    mmax = H.max_footsteps(pad[None], N, n)
    prm = H.make_params(cfg, mmax)
    rng = np.random.default_rng(SEED + 7919 * rank)
    x0_h = np.zeros((B, 2, 3))
    x0_h[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    F_h = rng.uniform(0.0, 800.0, B)
    if rank == 0:
        x0_h[0], F_h[0] = 0.0, cfg.F_ext   # the reference walk
    kick_h = cfg.dt * F_h / cfg.m
    plan = Plan(dev.index, N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, False)
    v = torch.as_tensor(v_ref, device=dev)
    s_t = torch.as_tensor(st, device=dev)
    nb_t = torch.as_tensor(nb, device=dev)
    x0 = torch.as_tensor(x0_h, device=dev)
    kick = torch.as_tensor(kick_h, device=dev)

    last = {}

    def launch():
        last["out"] = plan.herdt_rollout(prm, v, s_t, nb_t, x0, kick=kick, kick_step=n // 2)
    for _ in range(args.warmup):
        launch()
    plan.counters(reset=True)
    elapsed, kern_ms = timed_region(launch, args.steps, dist_on, dev)
    cnt = plan.counters(reset=True)
    hist, foot, status = last["out"]
    assert int(status.abs().max()) == 0, "solver reported a failed instance"
    solves_per_step = B * (n - 1) * world
    value = solves_per_step * args.steps / elapsed
    # algorithmic FP64 work per active-set pass, row and axis at the window's footstep count m
    # (NA = 3 + m): 2·NA² + 14·NA + 40 FLOP for the value-function update, 60 for the forward
    # and costate sweeps = 160 + 26 m + 2 m²; summed over the executed passes with the kernel's
    # counters (zmpc_plan_counters [5..7]: passes, Σm, Σm²)
    P, Sm, Sm2 = cnt["herdt_instance_passes"], cnt["herdt_footsteps"], cnt["herdt_footsteps_sq"]
    flops = float(N * (160 * P + 26 * Sm + 2 * Sm2)) / args.steps
    tfs = flops / (kern_ms * 1e-3) / 1e12
    passes_per_solve = P / (args.steps * 2 * B * (n - 1))
    alg_bytes = B * n * (6 + 2) * 8 + B * (6 + 1) * 8 + n * (2 * 8 + 1 + 4)
    if rank != 0:
        return None
    com_rmse_ref = None
    gold = os.path.join(ROOT, "tests", "golden", "herdt_default.npz")
    if os.path.exists(gold):
        g = np.load(gold)
        if g["com"].shape[0] == n:
            com_rmse_ref = float(np.sqrt(np.mean((hist[0, :, :, 0].cpu().numpy() - g["com"])
                                                 ** 2)))
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = _herdt_cpu_baseline(cfg, v_ref, st, hist.cpu().numpy(), foot.cpu().numpy(),
                                  x0_h, kick_h, args.cpu_seconds)
    return {
        "metric": "QP solves/sec (horizon=150, batched) at 1/2/4/8 MI355X; CoM RMSE vs ref",
        "value": value, "unit": "QP solves/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (the reference's default Herdt walk shared by every walk, seeded "
                "x0/F_ext)",
        "config": {"workload": f"config6: Herdt joint footstep QP, default walk, horizon={N}, "
                               f"n={n}", "walks_per_gpu": B, "global_batch": B * world,
                   "horizon": N, "samples_per_walk": n, "solves_per_step": solves_per_step,
                   "parallelism": f"dp{world}", "max_footsteps_in_window": mmax,
                   "solve": "one joint x/y QP (predict_herdt_joint, zmp_controller.py:533-826)"},
        "roofline": {"bound": "fp64", "achieved": tfs, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": tfs / FP64_PEAK_TFS, "traffic": pmc_traffic(f"config6_n{N}_b{B}"),
                     "kernel": "zmpc_herdt_kernel", "kernel_ms": kern_ms,
                     "alg_flops_per_launch": flops,
                     # compulsory bytes: the history [B,n,2,3] and foot track [B,n,2] out, x0 and
                     # the kick in, the shared v_ref / states / footstep counters once
                     "alg_bytes_per_launch": alg_bytes,
                     "traffic_over_alg_bytes": (None if not pmc_traffic(f"config6_n{N}_b{B}")
                                                else pmc_traffic(f"config6_n{N}_b{B}") /
                                                alg_bytes),
                     "passes_per_solve": passes_per_solve,
                     "max_passes_per_solve": cnt["herdt_max_passes_per_solve"],
                     "wave_passes_per_launch": cnt["herdt_wave_passes"] / args.steps,
                     "engine": "FP64 VALU, one (walk, axis) per lane; FLOPs = minimal per-row "
                               "work x the executed active-set passes (kernel counters)"},
        "cpu_baseline": cpu, "com_rmse_vs_ref": com_rmse_ref}


def _herdt_port_qps(cfg, vpad, spad, hist_w, foot_w, kick, i0, budget_s):
    """The oracle's exact Herdt step (herdt_oracle.herdt_step, the reference's
    predict_herdt_joint restated; its cvxpy/OSQP is not installed) over consecutive timesteps
    of one GPU walk from timestep i0, each QP fed the GPU walk's own state and foot and checked
    against the GPU's next state, until budget_s: (QPs, seconds, max |Δstate|)."""
    from oracle import herdt_oracle as HO
    n = hist_w.shape[0]
    N = cfg.horizon
    # the support side at i0: flips after every single-support phase (zmp_controller.py:497-529)
    side = "left"
    for i in range(i0):
        if spad[i + 1] != spad[i] and spad[i] == 2:
            side = "left" if side == "right" else "right"
    cur = spad[i0]
    t0 = time.perf_counter()
    steps, err = 0, 0.0
    for i in range(i0, n - 1):
        if time.perf_counter() - t0 > budget_s and steps >= 2:
            break
        x, y = hist_w[i, 0], hist_w[i, 1]
        fx, fy = foot_w[i]
        xn, yn, _, _ = HO.herdt_step(cfg, x, y, vpad[i + 1: i + 1 + N], fx, fy, cur,
                                     spad[i + 1: i + 1 + N], side)
        if i == n // 2:
            yn = yn - np.array([0.0, kick, 0.0])
        err = max(err, float(np.abs(xn - hist_w[i + 1, 0]).max()),
                  float(np.abs(yn - hist_w[i + 1, 1]).max()))
        if spad[i + 1] != cur and cur == 2:
            side = "left" if side == "right" else "right"
        if spad[i + 1] != cur:
            cur = spad[i + 1]
        steps += 1
    return steps, time.perf_counter() - t0, err


def _herdt_port_worker(job):
    """One process of the multi-process Herdt CPU leg (spawned; numpy only, 1 BLAS thread)."""
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        return _herdt_port_qps(*job)


def _herdt_cpu_baseline(cfg, v_ref, st, hist_gpu, foot_gpu, x0_h, kick_h, budget_s):
    """CPU leg for config 6 (rank 0), §8d(ii): P processes x 1 BLAS thread (P = this process's
    CPU share), process p on GPU walk p from a timestep spread over the walk (so the sample
    covers standing, double and single support and every footstep count), each timing the
    oracle's exact joint QP for budget_s; the sum of their rates.  Also one process at the
    default BLAS threads on walk 0 (§8d(i)).  Parity: every timed QP against the GPU walk."""
    n = len(st)
    N = cfg.horizon
    vpad = np.vstack([v_ref, np.repeat(v_ref[-1:], N, axis=0)])
    spad = np.concatenate([st, np.repeat(st[-1:], N)])
    P = cpu_share()
    W = min(P, hist_gpu.shape[0])
    jobs = [(cfg, vpad, spad, hist_gpu[w], foot_gpu[w], float(kick_h[w]),
             int((n - 2) * w / max(1, W)), budget_s) for w in range(W)]
    import multiprocessing
    from concurrent.futures import ProcessPoolExecutor
    with ProcessPoolExecutor(max_workers=W,
                             mp_context=multiprocessing.get_context("spawn")) as ex:
        res = list(ex.map(_herdt_port_worker, jobs))
    qps = sum(r[0] for r in res)
    multi = {"value": sum(r[0] / r[1] for r in res if r[1] > 0), "unit": "QP solves/s",
             "cores": W, "kind": "port",
             "sample": f"{W} processes x 1 BLAS thread, {qps} joint QPs (process p: walk p from "
                       "timestep p(n-2)/P, exact Goldfarb-Idnani NumPy port of "
                       "predict_herdt_joint; the reference's cvxpy/OSQP is not installed), "
                       f"≈{budget_s:.0f} s each",
             "max_abs_state_gpu_vs_port": max(r[2] for r in res)}
    s_steps, s_el, s_err = _herdt_port_qps(cfg, vpad, spad, hist_gpu[0], foot_gpu[0],
                                           float(kick_h[0]), 0, budget_s)
    multi["single_process_default_blas"] = {
        "value": s_steps / s_el, "unit": "QP solves/s", "cores": P, "kind": "port",
        "sample": f"{s_steps} consecutive joint QPs of walk 0, 1 process at the default BLAS "
                  "threads", "seconds": s_el, "max_abs_state_gpu_vs_port": s_err}
    return multi


def plan_record(plan):
    """The batch-invariant plan build (charged once per plan, never per solve):
    zmpc_plan_timings stage durations (HIP events on the creation stream) and the FP64 MFMA
    Gram M = PuᵀPu + (R/Q)·I (zmp_controller.py:198): its algorithmic FLOPs — the lower
    triangle of the symmetric product of a lower-triangular Toeplitz Pu with itself,
    Σ_{a≥b} 2(N − a) = N(N+1)(N+2)/3 (the upper half is a copy; the reference's dense
    Pu.T @ Pu is 2N³) — over its event time, as a fraction of the FP64 dense peak.  The rocprofv3 kernel time and MFMA counters of the same kernel are in
    profiles/r3_plan_*.  The timings are those of a second build of the same plan: the
    first kernel launches of a process also load the code object (≈0.5 ms on the first)."""
    again = Plan(plan.device, plan.N, plan.dt, plan.h, plan.g, plan.Q, plan.R, plan.strict)
    t = again.timings()
    again.destroy()
    N = plan.N
    flops = N * (N + 1) * (N + 2) / 3.0
    g_ms = t["gram_PuTPu"]
    tf = flops / (g_ms * 1e-3) / 1e12 if g_ms > 0 else None
    return {"N": N, "strict": plan.strict, "build_ms": t["total"],
            "stages_ms": {k: v for k, v in t.items() if v > 0 and k != "total"},
            "gram": {"kernel": "zmpc_gram_mfma<ToeplitzOp>", "engine": "v_mfma_f64_16x16x4_f64",
                     "ms": g_ms, "alg_flops": flops, "dense_equiv_flops": 2.0 * N ** 3,
                     "tflops": tf, "frac_fp64_peak": tf / FP64_PEAK_TFS if tf else None},
            "cholesky_ms": t["cholesky"]}


def make_batch(B, rank, cfg, shared):
    """Bounds ([B,n,2] per walk, or the shared [n,2] CoP), x0 [B,2,3], F [B]."""
    zmax, zmin, _ = CoPGenerator(cfg).generate_cop_trajectory()
    rng = np.random.default_rng(SEED + 7919 * rank)
    if shared:  # config 4: x0 = 0, one CoP for every scenario
        F = rng.uniform(0.0, 800.0, B)
        if rank == 0:
            F[0] = 400.0
        return zmax, zmin, zmax, zmin, np.zeros((B, 2, 3)), F
    off = rng.uniform(-0.02, 0.02, (B, 1, 2))
    x0 = np.zeros((B, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (B, 2))
    F = rng.uniform(0.0, 800.0, B)
    if rank == 0:
        off[0], x0[0], F[0] = 0.0, 0.0, 400.0   # the reference walk
    return zmax, zmin, zmax[None] + off, zmin[None] + off, x0, F


def walk_bounds(zmax_b, zmin_b, b):
    """Walk b's [n,2] bounds from a per-walk [B,n,2] or a shared [n,2] array."""
    if zmax_b.ndim == 2:
        return zmax_b, zmin_b
    return zmax_b[b], zmin_b[b]


def cpu_share():
    """CPU cores this process may use: the affinity set, capped by the box's declared share
    (OMP_NUM_THREADS is set to the GPU's CPU share on the GPU boxes) and at 16."""
    n = len(os.sched_getaffinity(0))
    try:
        n = min(n, int(os.environ.get("OMP_NUM_THREADS", n)))
    except ValueError:
        pass
    return max(1, min(n, 16))


def cpu_baseline(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg, budget_s):
    """CPU path beside the GPU run (rank 0, N=1), SURVEY.md §8d.  This leg is the only place
    bench.py touches oracle/ — as the checker and the timed CPU baseline, never as the measured
    product.
      * value: the reference-faithful NumPy port (oracle predict_wieber_axis_ref: interpreted
        Px/Pu build + np.linalg.inv per solve, zmp_controller.py:162-199; strict: the exact
        active-set box-QP restatement — the reference's cvxpy/OSQP is not installed) in P
        processes x 1 BLAS thread (P = this process's CPU share), whole walks of this batch
        until `budget_s` of CPU work per process; the sum of the processes' rates;
      * single_process: the same port in this process, 1 BLAS thread;
      * optimized: the batched gain-form port (oracle rollout_gain, all BLAS threads) on the
        first walks (unconstrained configs);
      * parity: GPU vs port on those walks (CoM RMSE, max |Δstate|)."""
    from oracle import zmp_oracle as O
    from threadpoolctl import threadpool_limits
    P = cpu_share()
    first = 1 if len(x0_b) > 1 else 0
    per = 6  # walks handed to each process (more than its budget needs)
    jobs = []
    for w in range(P):
        idx = [first + w + P * m for m in range(per) if first + w + P * m < len(x0_b)]
        if idx:
            jobs.append((_walk_payload(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, idx), cfg,
                         budget_s))
    multi = None
    if jobs:
        import multiprocessing
        from concurrent.futures import ProcessPoolExecutor
        # spawned children (the parent holds a GPU context: no fork); each runs numpy only
        with ProcessPoolExecutor(max_workers=len(jobs),
                                 mp_context=multiprocessing.get_context("spawn")) as ex:
            res = list(ex.map(_port_worker, jobs))
        solves = sum(r[0] for r in res)
        multi = dict(value=sum(r[0] / r[1] for r in res if r[1] > 0), unit="QP solves/s",
                     cores=len(jobs), kind="port",
                     sample=f"{len(jobs)} processes x 1 BLAS thread, {solves} solves over "
                            f"{sum(r[2] for r in res)} walk(s) of this batch, "
                            f"{_port_what(cfg)}, ≈{budget_s:.0f} s of CPU work per process",
                     com_rmse_gpu_vs_port=max(r[3] for r in res))
    with threadpool_limits(1):
        single = _cpu_walks(O, _walk_payload(zmax_b, zmin_b, x0_b, kick_b, hist_gpu,
                                             range(first, len(x0_b))), cfg, budget_s)
    s_solves, s_el, s_walks, s_rms = single
    single = dict(value=s_solves / s_el, unit="QP solves/s", cores=1, kind="port",
                  sample=f"{s_walks} walk(s) = {s_solves} solves of this batch (walks "
                         f"{first}..{first + s_walks - 1}), {_port_what(cfg)}, 1 BLAS thread",
                  seconds=s_el, com_rmse_gpu_vs_port=s_rms)
    out = dict(multi) if multi else dict(single)
    out["single_process"] = single
    # §8d(i): one process at the default BLAS thread count (no thread limit)
    sd = _cpu_walks(O, _walk_payload(zmax_b, zmin_b, x0_b, kick_b, hist_gpu,
                                     range(first, len(x0_b))), cfg, budget_s)
    out["single_process_default_blas"] = dict(
        value=sd[0] / sd[1], unit="QP solves/s", cores=P, kind="port",
        sample=f"{sd[2]} walk(s) = {sd[0]} solves of this batch, {_port_what(cfg)}, 1 process "
               "at the default BLAS thread count", seconds=sd[1], com_rmse_gpu_vs_port=sd[3])
    if cfg.strict:
        out["optimized"] = _strict_optimized_leg(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg,
                                                 budget_s, P)
    if not cfg.strict:
        nb = min(64, len(x0_b))
        zx = zmax_b if zmax_b.ndim == 3 else np.broadcast_to(zmax_b, (nb,) + zmax_b.shape)
        zn = zmin_b if zmin_b.ndim == 3 else np.broadcast_to(zmin_b, (nb,) + zmin_b.shape)
        n = zx.shape[1]
        t0 = time.perf_counter()
        ref = O.rollout_gain(zx[:nb], zn[:nb], x0_b[:nb], cfg.horizon, cfg.dt, cfg.h, cfg.g,
                             cfg.Q, cfg.R, kick_b[:nb], n // 2)
        tg = time.perf_counter() - t0
        out["optimized"] = {"value": nb * (n - 1) * 2 / tg, "unit": "QP solves/s",
                            "cores": P, "kind": "port",
                            "sample": f"first {nb} walks, batched gain-form NumPy port "
                                      "(oracle rollout_gain), default BLAS threads"}
        out["parity_first_walks"] = {
            "walks": nb,
            "com_rmse": float(np.sqrt(np.mean((hist_gpu[:nb, :, :, 0] - ref[..., 0]) ** 2))),
            "max_abs_state": float(np.abs(hist_gpu[:nb] - ref).max())}
    return out


def _strict_optimized_leg(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, cfg, budget_s, P):
    """Optimized strict CPU leg: the device kernel's algorithm (LQ Riccati per working set +
    primal-dual active set, warm-started) restated in C (oracle/strict_lq_cpu.c), OpenMP over
    (walk, axis) instances on P cores, over whole walks of this batch — as many as ≈budget_s
    of wall time allows (a probe of P walks sizes the sample)."""
    from oracle import strict_cpu as SC
    n = zmax_b.shape[-2]
    Bt = len(x0_b)

    def run(idx):
        zx = zmax_b if zmax_b.ndim == 2 else zmax_b[idx]
        zn = zmin_b if zmin_b.ndim == 2 else zmin_b[idx]
        t0 = time.perf_counter()
        h, st, ps = SC.rollout_strict(zx, zn, x0_b[idx], cfg.horizon, cfg.dt, cfg.h, cfg.g,
                                      cfg.Q, cfg.R, kick=kick_b[idx], kick_step=n // 2,
                                      threads=P)
        return time.perf_counter() - t0, h, st, ps
    probe = np.arange(min(P, Bt))
    tp, _, _, _ = run(probe)
    m = int(min(Bt, max(len(probe), budget_s / max(tp, 1e-6) * len(probe))))
    idx = np.arange(m)
    el, h, st, ps = run(idx)
    solves = m * (n - 1) * 2
    com = hist_gpu[idx, :, :, 0]
    return {"value": solves / el, "unit": "QP solves/s", "cores": P, "kind": "port",
            "sample": f"walks 0..{m - 1} of this batch ({solves} solves), the kernel's LQ "
                      f"active-set algorithm in C (oracle/strict_lq_cpu.c), OpenMP on {P} "
                      "threads", "seconds": el,
            "passes_per_solve": float(ps.sum()) / solves, "status_max": int(st.max()),
            "com_rmse_gpu_vs_port": float(np.sqrt(np.mean((h[..., 0] - com) ** 2)))}


def _port_what(cfg):
    return ("exact active-set box-QP NumPy port (oracle rollout_strict; the reference's "
            "cvxpy/OSQP is not installed)" if cfg.strict else
            "reference-faithful NumPy port (interpreted Pu build + np.linalg.inv per solve, "
            "zmp_controller.py:162-199)")


def _walk_payload(zmax_b, zmin_b, x0_b, kick_b, hist_gpu, idx):
    """(bounds, x0, kick, GPU CoM) of the walks idx, as plain arrays for a CPU worker."""
    return [(*walk_bounds(zmax_b, zmin_b, b), x0_b[b], kick_b[b], hist_gpu[b, :, :, 0])
            for b in idx]


def _port_worker(job):
    """One process of the multi-process CPU baseline (spawned; numpy only, 1 BLAS thread)."""
    walks, cfg, budget_s = job
    from oracle import zmp_oracle as O
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        return _cpu_walks(O, walks, cfg, budget_s)


def _cpu_walks(O, walks, cfg, budget_s):
    """Time the CPU port over whole walks until budget_s; (solves, seconds, walks, max RMSE)."""
    N, dt = cfg.horizon, cfg.dt
    solves, elapsed, nw, rms = 0, 0.0, 0, []
    for zmx, zmn, x0, kick, com_gpu in walks:
        if elapsed >= budget_s:
            break
        n = zmx.shape[0]
        t0 = time.perf_counter()
        if cfg.strict:
            h = O.rollout_strict(x0[0], x0[1], zmx, zmn, N, dt, cfg.h, cfg.g, cfg.Q,
                                 cfg.R, kick=kick, kick_step=n // 2)
            com = h[:, :, 0]
        else:
            zx = np.vstack([zmx, np.tile(zmx[-1:], (N, 1))])
            zn = np.vstack([zmn, np.tile(zmn[-1:], (N, 1))])
            x = x0[0].reshape(3, 1).copy()
            y = x0[1].reshape(3, 1).copy()
            com = [[x[0, 0], y[0, 0]]]
            for i in range(n - 1):
                if elapsed + time.perf_counter() - t0 > budget_s and i >= 16:
                    break  # long walks (config 5): a timed prefix of the walk
                x = O.predict_wieber_axis_ref(x, N, zx[i + 1:i + 1 + N, 0:1],
                                              zn[i + 1:i + 1 + N, 0:1], dt, cfg.h, cfg.g,
                                              cfg.Q, cfg.R)
                y = O.predict_wieber_axis_ref(y, N, zx[i + 1:i + 1 + N, 1:2],
                                              zn[i + 1:i + 1 + N, 1:2], dt, cfg.h, cfg.g,
                                              cfg.Q, cfg.R)
                if i == n // 2:
                    y = y - np.array([[0.0, kick, 0.0]]).T
                com.append([x[0, 0], y[0, 0]])
            com = np.array(com)
        elapsed += time.perf_counter() - t0
        solves += 2 * (len(com) - 1)
        rms.append(float(np.sqrt(np.mean((com - com_gpu[:len(com)]) ** 2))))
        nw += 1
    return solves, elapsed, nw, (max(rms) if rms else None)


def pmc_traffic(workload):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary
    (profiles/pmc_<workload>.json, written by profiles/collect_pmc.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    try:
        with open(path) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(gpus, argv):
    """`bench.py --gpus N` without a launcher around it: start N ranks of this script (one
    process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* as torchrun sets them, rendezvous on
    127.0.0.1) and wait for them.  The parent never touches the GPU; it returns the first
    non-zero exit code, and stops the other ranks when one fails (they would wait in a
    collective forever)."""
    port = _free_port()
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus),
                   LOCAL_WORLD_SIZE=str(gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def timed_region(launch, steps, collective, dev):
    """The bench contract's timed region: barrier + sync on both sides of exactly `steps`
    launches, the job time = max over ranks (collective: the process group's barrier and MAX
    all-reduce — RCCL on device tensors with the nccl backend — run even at world size 1 under
    --force-dist).  Returns (elapsed seconds, average launch duration in ms from one HIP event
    pair on the launch stream — None on CPU)."""
    cuda = dev.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    sync()
    if collective:
        dist.barrier()
    sync()
    if cuda:
        # one event pair brackets the K back-to-back launches on their stream (per-launch
        # pairs would add a marker packet, and an idle gap, between consecutive kernels)
        stream = torch.cuda.current_stream()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if cuda:
        ev0.record(stream)
    for _ in range(steps):
        launch()
    if cuda:
        ev1.record(stream)
    sync()
    # this rank's time from the common start to its last launch finishing; the job time is the
    # max over ranks, so the closing barrier's own latency is not charged
    elapsed = time.perf_counter() - t0
    if collective:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, (ev0.elapsed_time(ev1) / steps if cuda else None)


def gather_com(com, total, world, dev):
    """All-gather of the per-rank CoM blocks (RCCL over xGMI on GPUs): (full [total, ...],
    milliseconds), timed separately from `value`."""
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()
    tg = time.perf_counter()
    if dist.get_backend() != "nccl":
        com = com.cpu()  # gloo rehearsal: host buffers
    full = allgather_walks(com, total)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return full, (time.perf_counter() - tg) * 1e3


def stub_bench(args, rank, world):
    """`--stub-solver`: the multi-rank plumbing of this script on CPU (gloo) with a stand-in
    per-rank solver — spawn → shard → timed region → all-gather → one JSON line — for the CPU
    test of the launcher (tests/test_distributed.py).  Walk w's "history" is w + t/1000 at
    timestep t, so the reassembled batch proves every shard landed in its place."""
    B = args.batch or 8
    n = 16
    dev = torch.device("cpu")
    total = B * world
    a, b = shard_range(total, world, rank)
    idx = torch.arange(a, b, dtype=torch.float64)[:, None]
    hist = torch.empty((b - a, n, 2, 3), dtype=torch.float64)

    def launch():
        hist[:] = (idx + torch.arange(n, dtype=torch.float64)[None] / 1000.0)[..., None, None]
    for _ in range(args.warmup):
        launch()
    elapsed, _ = timed_region(launch, args.steps, world > 1, dev)
    full, gather_ms = gather_com(hist[..., 0].contiguous(), total, world, dev)
    expect = (torch.arange(total, dtype=torch.float64)[:, None] +
              torch.arange(n, dtype=torch.float64)[None] / 1000.0)[..., None]
    ok = bool(torch.equal(full, expect.expand(total, n, 2)))
    if rank == 0:
        print(json.dumps({
            "metric": "launcher self-test (stub solver)", "value": total * (n - 1) * 2 *
            args.steps / elapsed, "unit": "stub solves/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "scaling": "weak", "world_size": dist.get_world_size(), "backend": "gloo",
            "config": {"walks_per_gpu": B, "global_batch": total, "parallelism": f"dp{world}"},
            "allgather_ms": gather_ms, "gather_ok": ok}))
    return ok


def harness_cpu_seconds(N, strict, n_steps=100):
    """The reference's own perf harness, run_compare_runtime.py:21-73, on the CPU port: a
    controller for MPCConfig(horizon=N, strict=..., add_force=False), dummy ±0.1 m bounds over
    n_steps samples padded by the horizon (:21-33), `_run_once` = one x-axis and one y-axis
    predict_wieber_axis on the window [1:1+N] (= 2 QP solves, :44-57), 3 warm-up calls, then
    the MEAN of 10 timed calls from a zero state (:59-73).  The port: oracle
    predict_wieber_axis_ref (interpreted Px/Pu loop + np.linalg.inv, zmp_controller.py:162-199);
    strict: the same loop build + the exact box-QP (the reference's cvxpy/OSQP is absent).
    Returns seconds per `_run_once`."""
    from oracle import zmp_oracle as O
    cfg = MPCConfig(horizon=N, strict=strict, add_force=False)
    zmax = np.vstack([np.ones((n_steps, 2)) * 0.1, np.ones((N, 2)) * 0.1])
    zmin = -zmax
    hi = zmax[1:1 + N]
    lo = zmin[1:1 + N]

    def axis(x, a):
        if not strict:
            return O.predict_wieber_axis_ref(x, N, hi[:, a:a + 1], lo[:, a:a + 1], cfg.dt, cfg.h,
                                             cfg.g, cfg.Q, cfg.R)
        A, Bv, _ = O.lipm(cfg.dt, cfg.h, cfg.g)
        Px, Pu = O.prediction_matrices_loop(N, cfg.dt, cfg.h, cfg.g)   # :162-171 per call
        V = np.linalg.solve(Pu, np.eye(N))
        Hz = cfg.Q * np.eye(N) + cfg.R * V.T @ V
        u0, _, _, _ = O.strict_u0(x.ravel(), hi[:, a], lo[:, a], Hz, Px, Pu[0, 0], cfg.Q)
        return A @ x + Bv * u0

    def run_once(x, y):
        return axis(x, 0), axis(y, 1)
    x, y = np.zeros((3, 1)), np.zeros((3, 1))
    for _ in range(3):
        x, y = run_once(x, y)
    times = []
    for _ in range(10):
        x, y = np.zeros((3, 1)), np.zeros((3, 1))
        t0 = time.perf_counter()
        run_once(x, y)
        times.append(time.perf_counter() - t0)
    return float(np.mean(times))


def sweep_horizon(args, dev):
    """`--sweep-horizon`: the reference harness's horizon sweep (run_compare_runtime.py:139,
    N = 10..300 step 10) on both sides, one JSON line per horizon plus a summary line.
      gpu_batched: B default.json walks (CoP at that horizon, dt = 1.5/N, rigid offsets as
        config 2) rolled out per launch — QP solves/s, inputs resident in HBM, HIP-event
        timed; unconstrained and strict;
      gpu_call_ms: the harness's own semantics on the drop-in (ZMPController.predict_wieber_axis
        with host NumPy arrays: H2D, one kernel, D2H) — mean of 10 `_run_once` after 3 warm-ups;
      cpu_call_ms: the same harness on the CPU port (harness_cpu_seconds), 1 process, 1 BLAS
        thread."""
    from threadpoolctl import threadpool_limits
    from mpc_bipedal.controllers import ZMPController
    lo, hi, step = (int(v) for v in args.sweep_horizon.split(":"))
    Bu = args.batch or 4096
    Bs = max(64, Bu // 4)
    rows = []
    for N in range(lo, hi + 1, step):
        row = {"N": N}
        for strict in (False, True):
            d = dict(DEFAULT_JSON, horizon=N, strict=strict)
            cfg = MPCConfig(**d)
            B = Bs if strict else Bu
            _, _, zmax_h, zmin_h, x0_h, F_h = make_batch(B, 0, cfg, False)
            n = zmax_h.shape[1]
            plan = Plan(dev.index, N, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, strict)
            zmax = torch.as_tensor(zmax_h, device=dev)
            zmin = torch.as_tensor(zmin_h, device=dev)
            x0 = torch.as_tensor(x0_h, device=dev)
            kick = torch.as_tensor(cfg.dt * F_h / cfg.m, device=dev)
            launch = plan.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=n // 2)
            launch()
            steps = 3 if strict else 10
            elapsed, kern_ms = timed_region(launch, steps, False, dev)
            assert int(launch.status.abs().max()) == 0
            tag = "strict" if strict else "unc"
            row[f"gpu_batched_{tag}"] = B * (n - 1) * 2 * steps / elapsed
            row[f"kernel_ms_{tag}"] = kern_ms
            row[f"walks_{tag}"] = B
            row["samples_per_walk"] = n
            row[f"plan_build_ms_{tag}"] = plan.timings()["total"]
            # the harness on the drop-in (host arrays in and out, one solve pair per call)
            c = ZMPController(MPCConfig(horizon=N, strict=strict, add_force=False))
            zx = np.ones((N, 1)) * 0.1
            zn = -zx

            def run_once(x, y):
                return (c.predict_wieber_axis(x, N, zx, zn), c.predict_wieber_axis(y, N, zx, zn))
            xs, ys = np.zeros((3, 1)), np.zeros((3, 1))
            for _ in range(3):
                xs, ys = run_once(xs, ys)
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                run_once(np.zeros((3, 1)), np.zeros((3, 1)))
                ts.append(time.perf_counter() - t0)
            row[f"gpu_call_ms_{tag}"] = float(np.mean(ts)) * 1e3
            if not args.no_cpu_baseline:
                with threadpool_limits(1):
                    row[f"cpu_call_ms_{tag}"] = harness_cpu_seconds(N, strict) * 1e3
                row[f"cpu_solves_per_s_{tag}"] = 2.0 / (row[f"cpu_call_ms_{tag}"] * 1e-3)
            plan.destroy()
        print(json.dumps(row), flush=True)
        rows.append(row)
    print(json.dumps({
        "metric": "horizon sweep (run_compare_runtime.py:139 semantics): QP solves/s vs N",
        "unit": "QP solves/s", "n_gpus": 1, "dtype": "f64", "cpu_cores": 1,
        "horizons": [r["N"] for r in rows],
        "gpu_batched_unc": [r["gpu_batched_unc"] for r in rows],
        "gpu_batched_strict": [r["gpu_batched_strict"] for r in rows],
        "cpu_solves_per_s_unc": [r.get("cpu_solves_per_s_unc") for r in rows],
        "cpu_solves_per_s_strict": [r.get("cpu_solves_per_s_strict") for r in rows],
        "config": {"walks_unc": Bu, "walks_strict": Bs, "workload": "default.json walks at each "
                   "horizon (dt = 1.5/N) + rigid offsets, F_ext ~ U(0, 800) N"}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="SURVEY.md §8d workload (2 = BASELINE.json metric config; 6 = Herdt)")
    ap.add_argument("--batch", type=int, default=None, help="walks per GPU (config default)")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--strict", action="store_true", help="alias of --config 3")
    ap.add_argument("--unconstrained", action="store_true", help="config 4 unconstrained variant")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse several ranks on fewer GPUs)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise the process group even at --gpus 1, so that the "
                         "multi-rank path (barrier, MAX all-reduce, CoM all-gather) runs through "
                         "RCCL on one GPU")
    ap.add_argument("--sweep-horizon", default=None, metavar="LO:HI:STEP",
                    help="horizon sweep of the reference harness (e.g. 10:300:10), "
                         "run_compare_runtime.py:139; prints one line per horizon")
    ap.add_argument("--stub-solver", action="store_true",
                    help="CPU/gloo self-test of the multi-rank launcher (no GPU, no solver)")
    ap.add_argument("--no-dense-leg", action="store_true",
                    help="skip timing the dense correlation beside the default (profiles: the "
                         "rocprof kernel average then covers the default launches only)")
    ap.add_argument("--pipelined", action="store_true",
                    help="also time batches pipelined two-deep on two streams (reported beside "
                         "value; off by default so a profile of the default command sees only "
                         "non-overlapped launches)")
    ap.add_argument("--strict-steps", type=int, default=3,
                    help="default line (config 2): timed launches of the config-3 strict "
                         "sub-record (0 = no sub-record)")
    ap.add_argument("--strict-cpu-seconds", type=float, default=4.0,
                    help="CPU-leg budget per process of the strict sub-record")
    ap.add_argument("--herdt-steps", type=int, default=3,
                    help="default line (config 2): timed launches of the config-6 Herdt "
                         "sub-record (0 = no sub-record)")
    ap.add_argument("--herdt-cpu-seconds", type=float, default=4.0,
                    help="CPU-leg budget per process of the Herdt sub-record")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="plan option (mpc_bipedal/_native.py OPTIONS, include/zmpc.h "
                         "ZMPC_OPT_*) for A/B timing of forms with the same results")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher around us (the driver's torchrun form sets WORLD_SIZE): start the ranks
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.stub_solver:
        if world > 1:
            dist.init_process_group("gloo")
            assert dist.get_world_size() == args.gpus
        ok = stub_bench(args, rank, world)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(0 if ok else 1)
    dist_on = world > 1 or args.force_dist
    if dist_on:
        ndev = torch.cuda.device_count()
        if local >= ndev and args.dist_backend == "nccl":
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} GPU(s) visible")
        local %= ndev  # gloo rehearsal may put several ranks on one GPU
        torch.cuda.set_device(local)
        if "MASTER_ADDR" not in os.environ:  # --force-dist without a launcher: a group of one
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                              RANK="0", WORLD_SIZE="1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
        assert dist.get_world_size() == args.gpus
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.sweep_horizon:
        if dist_on:
            raise SystemExit("--sweep-horizon runs on one GPU")
        sweep_horizon(args, dev)
        return

    conf = 3 if args.strict else args.config
    if CONFIGS[conf].get("herdt"):
        line = herdt_bench(args, rank, world, dev, dist_on)
    else:
        line = rollout_bench(args, conf, rank, world, dev, dist_on)
        if conf == 2 and args.strict_steps > 0 and not args.batch and not args.horizon:
            # the strict experiment (run_compare_resistance.py:87-169; default.json:18
            # "strict": true) beside the headline: config 3 in its own timed region
            sub = strict_subrecord(args, rank, world, dev, dist_on)
            if rank == 0:
                line["strict"] = sub
        if conf == 2 and args.herdt_steps > 0 and not args.batch and not args.horizon:
            # the Herdt experiment (zmp_controller.py:435-826, config 6) likewise
            sub = herdt_subrecord(args, rank, world, dev, dist_on)
            if rank == 0:
                line["herdt"] = sub
    if rank == 0:
        print(json.dumps(line))
    if dist_on:
        dist.destroy_process_group()


def strict_subrecord(args, rank, world, dev, dist_on):
    """Config 3 (B = 65 536 walks per GPU, N = 150, strict, f64) as a sub-record of the default
    line: its own warm-up and timed region (barrier + synchronize on both sides, max over
    ranks), roofline (counted FP64 work, algorithmic bytes, PMC traffic) and, at one GPU, the
    CPU legs with a shorter budget.  The headline `value` stays config 2's."""
    sa = argparse.Namespace(**vars(args))
    sa.steps, sa.warmup = args.strict_steps, 1
    sa.batch, sa.horizon, sa.option = None, None, []
    sa.unconstrained, sa.pipelined, sa.no_dense_leg = False, False, True
    sa.cpu_seconds = args.strict_cpu_seconds
    sub = rollout_bench(sa, 3, rank, world, dev, dist_on)
    if rank != 0:
        return None
    for k in ("metric", "higher_is_better", "vs_baseline", "correlation", "pipelined"):
        sub.pop(k, None)
    return sub


def herdt_subrecord(args, rank, world, dev, dist_on):
    """Config 6 (32 768 Herdt walks per GPU, N = 150, f64) as a second sub-record of the default
    line, built like `strict_subrecord`: its own warm-up and timed region, roofline and, at one
    GPU, the CPU legs with a shorter budget."""
    sa = argparse.Namespace(**vars(args))
    sa.steps, sa.warmup = args.herdt_steps, 1
    sa.batch, sa.horizon = None, None
    sa.cpu_seconds = args.herdt_cpu_seconds
    sub = herdt_bench(sa, rank, world, dev, dist_on)
    if rank != 0:
        return None
    for k in ("metric", "higher_is_better", "vs_baseline"):
        sub.pop(k, None)
    return sub


def rollout_bench(args, conf, rank, world, dev, dist_on):
    """Configs 2-5 (the rollout workloads): the JSON line (rank 0) or None."""
    wl = dict(CONFIGS[conf])
    if args.unconstrained:
        wl["strict"] = False
    d = dict(DEFAULT_JSON)
    d["horizon"] = args.horizon or wl["horizon"]
    d["strict"] = wl["strict"]
    cfg = MPCConfig(**d)  # dt = 1.5 / horizon
    B = args.batch or wl["batch"]
    cop_x, cop_n, zmax_h, zmin_h, x0_h, F_h = make_batch(B, rank, cfg, wl["shared"])
    n = zmax_h.shape[-2]
    kick_h = cfg.dt * F_h / cfg.m
    plan = Plan(dev.index, cfg.horizon, cfg.dt, cfg.h, cfg.g, cfg.Q, cfg.R, cfg.strict)
    plan_rec = plan_record(plan)
    for o in args.option:
        name, _, val = o.partition("=")
        plan.set_option(name, int(val))
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
    if cfg.strict:
        plan.counters(reset=True)  # count the timed launches only
    elapsed, kern_ms = timed_region(launch, args.steps, dist_on, dev)
    work = plan.counters() if cfg.strict else None
    assert int(status.abs().max()) == 0, "solver reported a failed instance"

    solves_per_step = B * (n - 1) * 2 * world
    value = solves_per_step * args.steps / elapsed
    # algorithmic bytes of one launch: bounds in (2 × [B,n,2] f64, or one shared [n,2] pair)
    # + history out ([B,n,2,3])
    alg_bytes = 2 * (1 if wl["shared"] else B) * n * 2 * 8 + B * n * 6 * 8
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    flops = B * (n - 1) * 2 * (2 * cfg.horizon + 20)
    if wl["shared"] and not cfg.strict:
        # one CoP for every walk: the gain dot k·z_ref (2N FLOP) of a (timestep, axis) is the
        # same for all walks and is evaluated once per launch; 20 FLOP per solve remain
        flops = B * (n - 1) * 2 * 20 + (n - 1) * 2 * 2 * cfg.horizon
    direct_flops = B * (n - 1) * 2 * (2 * cfg.horizon + 20)
    P_fft = None if cfg.strict else fft_transform(n, cfg.horizon)
    if P_fft:
        # FFT correlation (both axes in one complex signal): two P-point transforms
        # (5 P log2 P real FLOP each, radix-2 count), the spectrum product (8 P), 20 per solve
        flops = B * (2 * 5 * P_fft * int(np.log2(P_fft)) + 8 * P_fft + (n - 1) * 2 * 20)
    workload = (f"config{conf}" + ("_unc" if conf == 4 and not cfg.strict else "") +
                f"_n{cfg.horizon}_b{B}")

    # parity in the same run: the reference walk (walk 0 of rank 0) vs the committed
    # reference fixture (tests/golden: produced by the reference itself)
    com_rmse_ref = None
    if rank == 0 and cfg.horizon == 150:
        fx = np.load(os.path.join(ROOT, "tests", "golden", "walk_n150.npz"))
        ref_com = fx["com_force"]
        if cfg.strict and not wl["shared"]:
            # walk 0 = the default walk at F_ext = 400 N: the reference's own strict branch run
            # with the recording cvxpy stand-in (tests/golden/make_strict_ref_golden.py)
            ref_com = np.load(os.path.join(ROOT, "tests", "golden", "strict_ref.npz"))[
                "n150_F400_com"]
        if ref_com.shape[0] == n:
            com_rmse_ref = float(np.sqrt(np.mean(
                (hist[0, :, :, 0].cpu().numpy() - ref_com) ** 2)))

    # the correlation form the rollout took: the sparse-difference form (rollout.hip
    # axis_correlate_sparse) for waves whose axis has ≤ 40 z_ref changes, else dense.  The dense
    # form is timed on the same inputs beside it (plan option ZMPC_OPT_CORRELATION = 1)
    corr = None
    if rank == 0 and not cfg.strict and not wl["shared"] and not args.no_dense_leg:
        zr = (zmax_h + zmin_h) / 2
        ch = np.count_nonzero(np.diff(zr, axis=1), axis=1)  # [B, 2] changes per walk and axis
        wide = n - 1 > 512  # wide kernel: its own limit, and a walk is sparse if both axes are
        lim = SPARSE_MAX_WIDE if wide else SPARSE_MAX
        sparse_frac = float((ch.max(axis=1) <= lim).mean() if wide else (ch <= lim).mean())
        corr_opt = plan.get_option("correlation")  # (an --option correlation=1 run keeps it)
        dense_ms = None
        if corr_opt != 1:
            plan.set_option("correlation", 1)  # ZMPC_OPT_CORRELATION: dense forms only
            try:
                for _ in range(max(1, args.warmup)):
                    launch()
                torch.cuda.synchronize()
                _, dense_ms = timed_region(launch, args.steps, False, dev)
            finally:
                plan.set_option("correlation", corr_opt)
                launch()  # the history the rest of the run reads comes from the run's form
                torch.cuda.synchronize()
        corr = {"form": "dense (option correlation=1)" if corr_opt == 1 else "sparse-difference",
                "sparse_max_changes_per_axis": lim,
                "zref_changes_per_axis_mean": float(ch.mean()),
                "zref_changes_per_axis_max": int(ch.max()),
                "sparse_frac": sparse_frac,
                "dense_kernel_ms": dense_ms if dense_ms is not None else kern_ms,
                "dense_hbm_frac": alg_bytes / ((dense_ms if dense_ms is not None else kern_ms)
                                               * 1e-3) / 1e9 / HBM_PEAK_GBS}

    gather_ms = None
    gather_ok = None
    if dist_on:
        com_local = hist[..., 0].contiguous()
        full, gather_ms = gather_com(com_local, B * world, world, dev)
        assert full.shape[0] == B * world
        a0, a1 = shard_range(B * world, world, rank)
        gather_ok = bool(torch.equal(full[a0:a1].to(com_local.device), com_local))
        assert gather_ok, "all-gather did not reassemble this rank's block in place"

    # batches pipelined two-deep on two streams (separate history buffers): consecutive
    # rollouts overlap, so one's memory phases run under the other's FP64 phases — what a
    # many-batch driver gets; reported beside `value`, not as it
    pipelined = None
    if rank == 0 and world == 1 and not cfg.strict and args.pipelined:
        streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
        hist2 = torch.empty_like(hist)
        with torch.cuda.stream(streams[1]):
            launch2 = plan.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=kstep,
                                            hist=hist2)
        launches = [launch, launch2]
        torch.cuda.synchronize()
        tq = time.perf_counter()
        for k in range(args.steps):
            with torch.cuda.stream(streams[k % 2]):
                launches[k % 2]()
        torch.cuda.synchronize()
        tq = (time.perf_counter() - tq) / args.steps
        assert torch.equal(hist, hist2)
        pipelined = {"value": B * (n - 1) * 2 / tq, "unit": "QP solves/s",
                     "ms_per_step": tq * 1e3, "streams": 2,
                     "hbm_gbs_aggregate": alg_bytes / tq / 1e9}

    # the drop-in batch API hands host arrays over: PCIe-inclusive rate (never `value`)
    pcie = None
    if rank == 0 and world == 1:
        reps = 1 if cfg.strict else 3
        torch.cuda.synchronize()
        tp = time.perf_counter()
        for _ in range(reps):
            h, st = plan.rollout(zmax_h, zmin_h, x0_h, kick=kick_h, kick_step=kstep)
            h.cpu()
        torch.cuda.synchronize()
        tp = (time.perf_counter() - tp) / reps
        pcie = {"value": B * (n - 1) * 2 / tp, "unit": "QP solves/s", "ms_per_step": tp * 1e3,
                "path": "Plan.rollout(numpy in) + hist.cpu(): pageable H2D of bounds/x0/kick, "
                        "kernel, D2H of the history"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(zmax_h, zmin_h, x0_h, kick_h, hist.cpu().numpy(), cfg,
                           args.cpu_seconds)

    if rank == 0:
        traffic = pmc_traffic(workload)
        fp64_tfs = flops / (kern_ms * 1e-3) / 1e12
        if not cfg.strict and alg_bytes / HBM_PEAK_GBS / 1e9 >= flops / FP64_PEAK_TFS / 1e12:
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS}
        elif not cfg.strict:
            # long horizons (config 5: 2N+20 = 1044 FLOP per solve) are FP64-bound; the
            # dtype's dense peak (78.6 TF, vector = matrix); the kernel runs on the VALU
            roof = {"bound": "fp64", "achieved": fp64_tfs, "peak": FP64_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": fp64_tfs / FP64_PEAK_TFS,
                    "engine": "FP64 VALU (v_mfma_f64 measured slower, DESIGN.md §4)"}
        else:
            # strict (strict_lq.hip): FP64 VALU-bound.  Algorithmic FLOPs = the executed
            # active-set passes (kernel counters) x the minimal per-pass work: one backward
            # Riccati + forward + costate per working-set slot, one s-recursion + forward per
            # free-tail slot (the sweep-B recompute is not counted)
            per = max(1, work["launches"])
            slots = work["instance_passes"] * cfg.horizon
            ws = work["working_set_slots"]
            sflops = (ws * STRICT_FLOP_WS + (slots - ws) * STRICT_FLOP_TAIL) / per
            s_tf = sflops / (kern_ms * 1e-3) / 1e12
            roof = {"bound": "fp64", "achieved": s_tf, "peak": FP64_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": s_tf / FP64_PEAK_TFS,
                    "engine": "FP64 VALU (one instance per lane; no MFMA-shaped work)",
                    "strict_alg_flops_per_launch": sflops,
                    "passes_per_solve": work["instance_passes"] / per / (B * (n - 1) * 2),
                    "max_passes_per_solve": work["max_passes_per_solve"],
                    "lane_efficiency": work["instance_passes"] / max(1, 64 * work["wave_passes"]),
                    "working_set_slot_frac": ws / max(1, slots),
                    "traffic_over_alg_bytes": (traffic / alg_bytes if traffic else None)}
        roof.update({
            "traffic": traffic,
            "kernel": rollout_kernel_name(B, n, cfg.horizon, cfg.strict, wl["shared"]),
            "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes,
            "hbm_gbs": achieved, "alg_flops_per_launch": flops,
            "fp64_frac_alg": flops / (kern_ms * 1e-3) / (FP64_PEAK_TFS * 1e12),
            "fp64_sustained_peak_tfs": FP64_SUSTAINED_TFS})
        if P_fft:
            roof.update({"fft_points": P_fft, "direct_form_flops_per_launch": direct_flops,
                         "direct_form_equiv_tfs": direct_flops / (kern_ms * 1e-3) / 1e12})
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
                "workload": f"config{conf}: " + (
                    "shared default.json CoP, Monte-Carlo F_ext" if wl["shared"] else
                    "default.json walks + rigid offsets") +
                    (", strict" if cfg.strict else ", unconstrained") +
                    f", horizon={cfg.horizon}, n={n}",
                "walks_per_gpu": B, "global_batch": B * world, "horizon": cfg.horizon,
                "samples_per_walk": n, "solves_per_step": solves_per_step,
                "parallelism": f"dp{world}", "strict": bool(cfg.strict),
                "shared_cop": bool(wl["shared"]),
                **({"plan_options": args.option} if args.option else {}),
            },
            "roofline": roof,
            "cpu_baseline": cpu,
            "com_rmse_vs_ref": com_rmse_ref,
            "allgather_ms": gather_ms,
            "allgather_backend": dist.get_backend() if dist_on else None,
            "allgather_ok": gather_ok,
            "pcie_inclusive": pcie,
            "pipelined": pipelined,
            "correlation": corr,
            "plan": plan_rec,
        }
        plan.destroy()
        return line
    plan.destroy()
    return None


if __name__ == "__main__":
    main()
