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
