"""Multi-process sharding + reassembly (world_size 2, gloo on CPU).

The device solve of each shard is stood in for by the oracle (CPU); what is under test is the
partition (shard_range) and the all-gather reassembly (allgather_walks) that bench.py and
multi-GPU callers use over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mpc_bipedal.distributed import allgather_walks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_range_partitions():
    for total in (0, 1, 7, 4096, 1000003):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, world, r) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            for (a, b), (c, d) in zip(parts, parts[1:]):
                assert b == c
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, total, out_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.dirname(here))
    from oracle import zmp_oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = np.load(os.path.join(here, "golden", "walk_n10.npz"))
    rng = np.random.default_rng(3)
    off = rng.uniform(-0.02, 0.02, (total, 1, 2))
    zmax, zmin = d["zmax"][None] + off, d["zmin"][None] + off
    x0 = np.zeros((total, 2, 3))
    kick = rng.uniform(0, 0.2, total)
    n = zmax.shape[1]
    a, b = shard_range(total, world, rank)
    hist = O.rollout_gain(zmax[a:b], zmin[a:b], x0[a:b], 10, float(d["dt"]), 0.75, 9.81, 1.0,
                          1e-6, kick[a:b], n // 2)
    com = torch.as_tensor(hist[..., 0]).contiguous()
    full = allgather_walks(com, total)
    if rank == 0:
        ref = O.rollout_gain(zmax, zmin, x0, 10, float(d["dt"]), 0.75, 9.81, 1.0, 1e-6, kick,
                             n // 2)
        np.save(out_path, np.abs(full.numpy() - ref[..., 0]).max())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", (9, 16))
def test_gloo_two_ranks_reassemble(tmp_path, total):
    out = str(tmp_path / "err.npy")
    mp.start_processes(_worker, args=(2, _free_port(), total, out), nprocs=2, join=True,
                       start_method="spawn")
    assert float(np.load(out)) == 0.0


def test_bench_launcher_two_ranks_stub():
    """`python bench.py --gpus 2` (no torchrun around it) starts two ranks itself: spawn →
    shard → timed region → all-gather → ONE JSON line from rank 0 with n_gpus 2 (gloo, stub
    per-rank solver; the GPU form runs the same code with RCCL)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--stub-solver", "--steps", "3", "--warmup", "1", "--batch", "5"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["world_size"] == 2
    assert line["config"]["global_batch"] == 10 and line["config"]["parallelism"] == "dp2"
    assert line["gather_ok"] is True and line["allgather_ms"] is not None
    assert line["steps"] == 3 and line["value"] > 0


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--stub-solver"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_harness_cpu_leg_semantics():
    """bench.harness_cpu_seconds follows run_compare_runtime.py:36-73 (3 warm-ups, mean of 10
    `_run_once` = 2 solves) on the CPU port, both branches."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    for strict in (False, True):
        t = bench.harness_cpu_seconds(10, strict)
        assert 0.0 < t < 1.0
