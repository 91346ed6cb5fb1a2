"""N > 1 path on CPU: two gloo ranks shard the problem ids (vboc_amd.dist.shard_ids), solve their
shards (the CPU oracle stands in for the GPU solver here) and all-gather the boundary states
(vboc_amd.dist.gather_boundary_states, the collective bench.py runs over RCCL).  The gathered
result must equal a single-process solve of all ids, bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _solve_x0(ids):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from vboc_amd.ics import data_generation_ics
    b = data_generation_ics(2, ids)
    xo, _, res = oracle.solve_batch(2, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                    b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"],
                                    opts=oracle.default_opts(max_iter=40), nthreads=1)
    return xo[:, 0, :], res["status"]


def _worker(rank, world, port, per_rank, steps, out_path):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vboc_amd.dist import gather_boundary_states, shard_ids
    gathered = []
    for step in range(steps):
        ids = shard_ids(step, world, rank, per_rank)
        x0, _ = _solve_x0(ids)
        gathered.append(gather_boundary_states(torch.as_tensor(x0)).numpy())
    if rank == 0:
        np.save(out_path, np.concatenate(gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ids_cover_every_problem_once():
    from vboc_amd.dist import shard_ids
    for world in (1, 2, 4, 8):
        ids = np.concatenate([shard_ids(s, world, r, 5) for s in range(3) for r in range(world)])
        np.testing.assert_array_equal(np.sort(ids), np.arange(3 * world * 5))


def test_two_rank_gather_equals_single_process(tmp_path):
    import torch.multiprocessing as mp
    world, per_rank, steps = 2, 3, 2
    out = str(tmp_path / "gathered.npy")
    mp.spawn(_worker, args=(world, _free_port(), per_rank, steps, out), nprocs=world, join=True)
    got = np.load(out)
    ref, status = _solve_x0(np.arange(world * per_rank * steps))
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)
    assert np.all(np.isin(status, [0, 2]))
