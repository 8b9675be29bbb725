"""Two ranks drive the device solver (Plan → zmpc_rollout) on their own shards and reassemble
the batch with allgather_walks; the result equals one full-batch launch.

The 1-GPU box puts both ranks on cuda:0 with the gloo backend (RCCL needs one GPU per rank);
the sharding, the per-rank launches and the reassembly are the code the 8-GPU bench runs.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

N, TOTAL = 150, 9


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    here = os.path.dirname(os.path.abspath(__file__))
    d = np.load(os.path.join(here, "golden", "walk_n150.npz"))
    rng = np.random.default_rng(12)
    off = rng.uniform(-0.02, 0.02, (TOTAL, 1, 2))
    x0 = np.zeros((TOTAL, 2, 3))
    x0[:, :, 0] = rng.uniform(-0.01, 0.01, (TOTAL, 2))
    kick = 0.01 * rng.uniform(0, 800, TOTAL) / 40.0
    return d["zmax"][None] + off, d["zmin"][None] + off, x0, kick


def _rank(rank, world, port, strict, out):
    from mpc_bipedal.distributed import allgather_walks, shard_range
    from mpc_bipedal.solver import Plan
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    zmax, zmin, x0, kick = _batch()
    n = zmax.shape[1]
    a, b = shard_range(TOTAL, world, rank)
    p = Plan(0, N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, strict)
    hist, st = p.rollout(zmax[a:b], zmin[a:b], x0[a:b], kick=kick[a:b], kick_step=n // 2)
    assert int(st.abs().max()) == 0
    full = allgather_walks(hist.cpu().contiguous(), TOTAL)
    if rank == 0:
        np.save(out, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("strict", (False, True))
def test_two_ranks_device_shards_reassemble(tmp_path, strict):
    from mpc_bipedal.solver import Plan
    out = str(tmp_path / "full.npy")
    mp.start_processes(_rank, args=(2, _port(), strict, out), nprocs=2, join=True,
                       start_method="spawn")
    zmax, zmin, x0, kick = _batch()
    n = zmax.shape[1]
    p = Plan(torch.cuda.current_device(), N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, strict)
    ref, st = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    assert int(st.abs().max()) == 0
    assert np.abs(np.load(out) - ref.cpu().numpy()).max() <= 1e-12
