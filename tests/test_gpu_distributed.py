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


def _nccl_rank(rank, port, out):
    """World-size-1 RCCL group on cuda:0 (device_id bound, as bench.py:init does): the device
    all-gather, the bench's timed region (barrier + MAX all-reduce on a device tensor) and
    gather_com all run through the nccl backend."""
    import sys
    from mpc_bipedal.distributed import allgather_walks
    from mpc_bipedal.solver import Plan
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    zmax, zmin, x0, kick = _batch()
    n = zmax.shape[1]
    p = Plan(0, N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, False)
    launch = p.rollout_launcher(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    elapsed, kern_ms = bench.timed_region(launch, 3, True, dev)
    assert elapsed > 0 and kern_ms > 0
    com = launch.hist[..., 0].contiguous()
    full = allgather_walks(com, TOTAL)          # device tensors through RCCL
    assert full.device == dev and torch.equal(full, com)
    full2, ms = bench.gather_com(com, TOTAL, 1, dev)
    assert full2.device == dev and torch.equal(full2, com) and ms >= 0
    np.save(out, full.cpu().numpy())
    dist.destroy_process_group()


def test_nccl_group_of_one_device_collectives(tmp_path):
    """The RCCL path of the multi-GPU bench (bench.py init_process_group("nccl", device_id),
    timed_region's device all-reduce, gather_com / allgather_walks on device tensors) on the
    1-GPU box, with a group of one: the reassembled CoM equals the local rollout."""
    from mpc_bipedal.solver import Plan
    out = str(tmp_path / "com.npy")
    mp.start_processes(_nccl_rank, args=(_port(), out), nprocs=1, join=True,
                       start_method="spawn")
    zmax, zmin, x0, kick = _batch()
    n = zmax.shape[1]
    p = Plan(torch.cuda.current_device(), N, 1.5 / N, 0.75, 9.81, 1.0, 1e-6, False)
    ref, _ = p.rollout(zmax, zmin, x0, kick=kick, kick_step=n // 2)
    assert np.array_equal(np.load(out), ref[..., 0].cpu().numpy())


def test_bench_force_dist_nccl():
    """bench.py --gpus 1 --force-dist: the default workload with the RCCL process group live
    (the code path the 8-GPU driver run takes at every rank): one JSON line, the all-gather
    reassembled the rank's block in place, backend nccl."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1",
                        "--force-dist", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                        "--no-dense-leg"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["allgather_backend"] == "nccl" and line["allgather_ok"] is True
    assert line["allgather_ms"] is not None
