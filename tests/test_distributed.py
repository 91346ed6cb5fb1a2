"""N > 1 path on CPU: two gloo ranks shard the problem ids (vboc_amd.dist.shard_ids), solve their
shards (the CPU oracle stands in for the GPU solver here) and all-gather the boundary states
(vboc_amd.dist.gather_boundary_states, the collective bench.py runs over RCCL).  The gathered
result must equal a single-process solve of all ids, bit for bit.  bench.run itself (step loop, barrier,
rank-max timing, flop / solve all-reduce, all-gather of the samples) runs at world size 2 on gloo with the
oracle as its engine."""
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


# ------------------------------------------------------------------------------------------------
# bench.py's N > 1 path (run(args, engine_factory)) on gloo, the oracle as the engine
# ------------------------------------------------------------------------------------------------
class OracleEngine:
    """bench.GpuEngine's interface on the CPU oracle (test infrastructure)."""
    kernel = "oracle"

    def __init__(self, nq, args, local):
        import torch
        self.torch, self.nq = torch, nq
        self.device = torch.device("cpu")
        self.ms = 0.0

    def sync(self):
        pass

    def first_solve_batch(self, nq, ids):
        from vboc_amd.ics import data_generation_ics
        return data_generation_ics(nq, ids)

    def first_solve(self, b):
        import time
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        t0 = time.perf_counter()
        xo, _, r = oracle.solve_batch(self.nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                      b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"],
                                      opts=oracle.default_opts(max_iter=40), nthreads=1)
        self.ms = (time.perf_counter() - t0) * 1e3
        T = self.torch.as_tensor
        return dict(x0=T(xo[:, 0, :].copy()), status=T(r["status"].copy()), sqp_iter=T(r["sqp_iter"].copy()),
                    qp_iter=T(r["qp_iter"].copy()))

    def dg(self, ids):
        import time
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        from vboc_amd.drivers import data_generation_batch
        t0 = time.perf_counter()
        res, st = data_generation_batch(self.nq, ids, oracle.DriverBackend(self.nq, 1))
        self.ms = (time.perf_counter() - t0) * 1e3
        samples = [r[0] if self.nq == 2 else r for r in res]
        cnt = np.array([-1 if s is None else len(s) for s in samples])
        rows = np.array([row for s in samples if s for row in s], dtype=np.float64).reshape(-1, 2 * self.nq)
        off = np.concatenate([[0], np.cumsum(np.maximum(cnt, 0))[:-1]])
        from vboc_amd.lib import DG_STATS
        stats = np.zeros((len(ids), len(DG_STATS)))
        stats[0, 0], stats[0, 1] = st["solves"], st["rk4"]
        T = self.torch.as_tensor
        return dict(rows_all=T(rows), row_off=T(off.astype(np.int64)), row_cnt=T(cnt.astype(np.int32)), stats=T(stats))

    def kernel_ms(self):
        return self.ms


def _bench_worker(rank, world, port, argv, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import json
    import bench
    from test_distributed import OracleEngine
    line = bench.run(bench.parse(argv), engine_factory=OracleEngine)
    if rank == 0:
        json.dump(line, open(out_path, "w"))


@pytest.mark.parametrize("workload", ["dg-loop", "first-solve"])
def test_bench_runs_at_world_two_on_gloo(tmp_path, workload):
    import json
    import torch.multiprocessing as mp
    from vboc_amd.dist import shard_ids
    B, steps = 3, 2
    argv = ["--gpus", "2", "--nq", "2", "--batch", str(B), "--steps", str(steps), "--warmup", "1",
            "--workload", workload, "--no-cpu"]
    out = str(tmp_path / "line.json")
    mp.spawn(_bench_worker, args=(2, _free_port(), argv, out), nprocs=2, join=True)
    line = json.load(open(out))
    assert line["n_gpus"] == 2 and line["steps"] == steps and line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0 and line["ms_per_step"] > 0
    eng = OracleEngine(2, None, 0)
    ids = [shard_ids(s, 2, r, B) for s in range(1, 1 + steps) for r in range(2)]   # the timed steps
    if workload == "dg-loop":
        outs = [eng.dg(i) for i in ids]
        solves = sum(float(o["stats"][:, 0].sum()) for o in outs)
        rows = sum(int(o["rows_all"].shape[0]) for o in outs)
        # every rank's samples were all-gathered; solves all-reduced; value = all solves / max-over-ranks time
        assert line["loop"]["samples"] == rows
        assert abs(line["loop"]["solves_per_problem"] - solves / (2 * steps * B)) < 1e-3
        assert abs(line["value"] - solves / (line["ms_per_step"] * steps / 1e3)) < 0.01 * line["value"] + 0.01
    else:
        assert abs(line["value"] - 2 * steps * B / (line["ms_per_step"] * steps / 1e3)) < 0.01 * line["value"] + 0.01


def test_bench_gpus_two_starts_two_ranks_without_a_launcher(tmp_path):
    """`python bench.py --gpus 2` with no torch.distributed.run environment starts the two rank processes itself
    (the driver's N-GPU command), and the line's n_gpus is the process group's size.  The oracle engine stands
    in for the GPU (--engine, a test hook); everything else is the product's launcher and step loop."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["PYTHONPATH"] = os.pathsep.join([os.path.dirname(os.path.abspath(__file__)), ROOT])
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "dg-loop", "--nq", "2",
           "--batch", "2", "--steps", "1", "--warmup", "1", "--no-cpu", "--engine", "test_distributed:OracleEngine"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout          # rank 0 prints the only line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["library"] == {"engine": "test_distributed:OracleEngine"}
    assert line["value"] > 0 and line["loop"]["samples"] >= 0


def test_bench_refuses_a_world_that_differs_from_gpus():
    """A single process asked for --gpus 2 under a launcher environment of world size 1 exits non-zero instead
    of printing a one-rank line labelled as two."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               PYTHONPATH=os.pathsep.join([os.path.dirname(os.path.abspath(__file__)), ROOT]))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "first-solve", "--nq", "2",
           "--batch", "2", "--steps", "1", "--warmup", "0", "--no-cpu", "--engine", "test_distributed:OracleEngine"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "process group has 1 rank" in r.stderr


# ------------------------------------------------------------------------------------------------
# the VBOC loop (streamed segments) and the UR5 / Cartesian main blocks at world size 2 on gloo
# ------------------------------------------------------------------------------------------------
class _RankSegment:
    """A streamed segment whose round r is this rank's shard of iteration first + r (pipeline._rank_ids, what the
    product's StreamedRounds launches), solved by the host driver on the oracle."""

    def __init__(self, first, n, nq, num_prob):
        self.first, self.n, self.nq, self.num_prob = first, n, nq, num_prob

    def round(self, r):
        from oracle_backend import OracleBackend
        from vboc_amd.pipeline import _generate, _rank_ids
        return _generate(self.nq, OracleBackend(self.nq), _rank_ids(self.first + r, self.num_prob), None, 20250124)

    def cancel(self):
        pass

    def close(self):
        return dict(seconds=0.0, spec_solves=0, spec_used=0, waited_s=0.0)


def _main_blocks_worker(rank, world, port, out_dir):
    import pickle
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle_backend import OracleBackend
    from vboc_amd.pipeline import cartesian_run, ur5_run, vboc_run
    from vboc_amd.systems import cartesian_constraint
    X_test = np.tile([np.pi, np.pi, 1.0, 1.0], (4, 1))
    loop = vboc_run(2, OracleBackend(2), X_test, stop_time=1e9, num_prob=5, max_iterations=2, stream_rounds=2,
                    segment_factory=lambda f, k: _RankSegment(f, k, 2, 5),
                    trainer_kw=dict(hidden=8, minibatch=16, stop_val=1e9))
    u = ur5_run(OracleBackend(4), num_test=2, num_train=3, device="cpu", minibatch=8, hidden=16)
    c = cartesian_run(OracleBackend(2, path_constraint=cartesian_constraint()), num_test=2, num_train=3,
                      device="cpu", minibatch=8, hidden=16)
    res = dict(loop=loop["X_save"], loop_rmse=loop["rmse"], ur5_test=u["X_test"], ur5_train=u["X_train"],
               ur5_fit=u["fit"], cart_test=c["X_test"], cart_train=c["X_train"], cart_fit=c["fit"])
    with open(os.path.join(out_dir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def test_main_blocks_at_world_two_equal_one_process(tmp_path):
    """configs[3] / config 4's sharding on gloo: the streamed VBOC loop (each rank streams its shard of every
    iteration, the samples all-gathered per iteration), ur5_run and cartesian_run (each rank one contiguous share
    of the test and training ids, rows all-gathered) give every rank the single-process rows in problem order;
    only rank 0 fits."""
    import pickle
    import torch.multiprocessing as mp
    from oracle_backend import OracleBackend
    from vboc_amd.pipeline import _generate, cartesian_run, samples_array, ur5_run
    from vboc_amd.systems import cartesian_constraint
    mp.spawn(_main_blocks_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = [pickle.load(open(tmp_path / f"rank{r}.pkl", "rb")) for r in range(2)]
    loop_ref = np.concatenate([samples_array(2, _generate(2, OracleBackend(2), np.arange(i * 5, (i + 1) * 5), None,
                                                           20250124)[0]) for i in range(3)])
    u = ur5_run(OracleBackend(4), num_test=2, num_train=3, device="cpu", minibatch=8, hidden=16)
    c = cartesian_run(OracleBackend(2, path_constraint=cartesian_constraint()), num_test=2, num_train=3,
                      device="cpu", minibatch=8, hidden=16)
    for r in (r0, r1):
        np.testing.assert_array_equal(r["loop"], loop_ref)
        np.testing.assert_array_equal(r["ur5_test"], u["X_test"])
        np.testing.assert_array_equal(r["ur5_train"], u["X_train"])
        np.testing.assert_array_equal(r["cart_test"], c["X_test"])
        np.testing.assert_array_equal(r["cart_train"], c["X_train"])
    assert len(r0["loop_rmse"]) == 3 and r1["loop_rmse"] == []
    assert r0["ur5_fit"] is not None and r1["ur5_fit"] is None and r1["cart_fit"] is None
