"""The VBOC main loop: batched boundary data generation, NN fit, RMSE on the held-out set, repeated
until the time budget is spent, and the reference's artefact files.

Reference: VBOC/triplependulum_vboc.py:372-585 (the double VBOC/doublependulum_vboc.py:404-620).
  iteration 0: data_generation over num_prob problems (:399-405), X_save = all saved rows (:404-405),
               mean/std (:50), first fit (:77-99), times/rmse (:102-120);
  iteration i: more data (:127-134), X_save grows, refit half old / half new (:152-184), times/rmse
               appended (:187-197), until stop_time (:122);
  artefacts:   times_/rmse_/data_<n>dof_vboc.npy, mean_/std_<n>dof_vboc (torch.save of a float),
               model_<n>dof_vboc (state_dict) (:50-52, :204-215).
The held-out set comes from `drivers.testing_batch` (triplependulum_testdata.py, saved as
data<n>_test.npy, :145).

Quirk kept (documented in DESIGN.md): the triple driver recomputes the refit's "new" feature rows
from the WHOLE X_save (:140-150) rather than from X_new as the double does (doublependulum :138-146),
so old rows are duplicated into the new half; `triple_refit_quirk=False` uses X_new.

Problem ids: iteration i solves ids [i*num_prob, (i+1)*num_prob) (the reference's forked workers draw
fresh unseeded ICs every iteration); with torch.distributed initialised, each rank solves a
contiguous shard and the saved rows are all-gathered (vboc_amd.dist.gather_samples); rank 0 trains.
"""
import os
import time

import numpy as np

from .drivers import data_generation_batch, heldout_set, testing_batch
from .ics import SEED
from .learn import dir_features, make_trainer, position_stats
from .systems import system


def samples_array(nq, results):
    """Saved rows of one data-generation round: flatten the non-None sample lists (:404-405; the
    double unpacks its 3-tuples first, doublependulum_vboc.py:436-438)."""
    traj = results if nq != 2 else [r[0] for r in results]
    rows = [row for t in traj if t is not None for row in t]
    return np.array(rows, dtype=np.float64).reshape(len(rows), 2 * nq)


def save_artifacts(out_dir, nq, X_save, mean, std, model, times, rmse):
    """The reference's file names and formats (VBOC/triplependulum_vboc.py:51-52,204-215)."""
    import torch
    os.makedirs(out_dir, exist_ok=True)
    tag = f"{nq}dof_vboc"
    np.save(os.path.join(out_dir, f"times_{tag}.npy"), np.asarray(times))
    np.save(os.path.join(out_dir, f"rmse_{tag}.npy"), np.asarray(rmse))
    np.save(os.path.join(out_dir, f"data_{tag}.npy"), np.asarray(X_save))
    torch.save(mean, os.path.join(out_dir, f"mean_{tag}"))
    torch.save(std, os.path.join(out_dir, f"std_{tag}"))
    torch.save({k: v.detach().cpu() for k, v in model.state_dict().items()}, os.path.join(out_dir, f"model_{tag}"))


def load_artifacts(out_dir, nq, device="cpu"):
    """Read the artefacts back the way triplependulum_comparison.py:31-36 does (weights_only loads)."""
    import torch
    from .learn import NeuralNetDIR
    tag = f"{nq}dof_vboc"
    sd = torch.load(os.path.join(out_dir, f"model_{tag}"), weights_only=True)
    model = NeuralNetDIR(2 * nq, sd["linear_relu_stack.0.weight"].shape[0], 1).to(device)
    model.load_state_dict(sd)
    return dict(model=model, data=np.load(os.path.join(out_dir, f"data_{tag}.npy")),
                mean=torch.load(os.path.join(out_dir, f"mean_{tag}"), weights_only=True),
                std=torch.load(os.path.join(out_dir, f"std_{tag}"), weights_only=True),
                times=np.load(os.path.join(out_dir, f"times_{tag}.npy")),
                rmse=np.load(os.path.join(out_dir, f"rmse_{tag}.npy")))


def _device_solver(backend, nmin):
    """The backend's lib.Solver when the state machines can run on the device (the product GPU backend with a
    horizon capacity of at least nmin), else None (the oracle backends of the CPU tests)."""
    solver = getattr(backend, "solver", None)
    if solver is not None and hasattr(solver, "testing_device") and solver.nmax >= nmin:
        return solver
    return None


def make_test_set(nq, backend, num_prob=1000, first_id=0, out_dir=None, seed=SEED):
    """`testing` over num_prob problems -> X_test (data<n>_test.npy, triplependulum_testdata.py:137-145).  On the
    product GPU backend the whole state machine runs on the device (drivers.testing_device, one launch)."""
    from .drivers import testing_device
    ids = np.arange(first_id, first_id + num_prob)
    solver = _device_solver(backend, system(nq).N + 12) if nq in (2, 3) else None
    if solver is not None:
        res, stats = testing_device(nq, ids, solver, seed=seed)
    else:
        res, stats = testing_batch(nq, ids, backend, seed=seed)
    X = heldout_set(nq, res)
    if out_dir is not None:
        os.makedirs(out_dir, exist_ok=True)
        np.save(os.path.join(out_dir, f"data{nq}_test.npy"), X)
    return X, stats


def _generate(nq, backend, ids, N_start, seed):
    """data_generation for `ids`: on the product GPU backend the whole state machine runs on the device
    (drivers.data_generation_device, vboc_data_generation); other backends (the oracle in the tests) go
    through the host driver.  Both return the reference's per-problem results in problem order."""
    from .drivers import data_generation_device
    solver = getattr(backend, "solver", None)
    if solver is not None and hasattr(solver, "data_generation_device") and \
            solver.nmax >= (N_start or system(nq).N) + 12:
        return data_generation_device(nq, ids, solver, N_start=N_start, seed=seed)
    return data_generation_batch(nq, ids, backend, N_start=N_start, seed=seed)


def _round(nq, backend, iteration, num_prob, N_start, seed):
    """One synchronous data-generation round over the problem ids [iteration * num_prob, (iteration + 1) * num_prob),
    this rank's contiguous shard of them under torch.distributed; the samples are all-gathered in rank (= problem)
    order."""
    res, stats = _generate(nq, backend, _rank_ids(iteration, num_prob), N_start, seed)
    return _gather_rows(samples_array(nq, res)), stats


def _rank_ids(iteration, num_prob):
    """This rank's ids of VBOC iteration `iteration`: [iteration * num_prob, (iteration + 1) * num_prob) split into
    contiguous per-rank shards (np.array_split) under torch.distributed, so every world size solves the same ids and
    the rank-ordered gather is the problem order."""
    return _shard(np.arange(iteration * num_prob, (iteration + 1) * num_prob))


def _shard(ids):
    """This rank's contiguous share of `ids` under torch.distributed (np.array_split), else all of them."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return np.array_split(np.asarray(ids), dist.get_world_size())[dist.get_rank()]
    return np.asarray(ids)


def _is_rank0():
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def _gather_rows(X):
    """All ranks' rows in rank (= problem) order (dist.gather_samples: RCCL under nccl, gloo on the CPU); the local
    rows when torch.distributed is not initialised."""
    import torch
    import torch.distributed as dist
    from .dist import gather_samples
    if not (dist.is_available() and dist.is_initialized()):
        return X
    local = torch.from_numpy(np.ascontiguousarray(X))
    if dist.get_backend() == "nccl":
        local = local.cuda()
    return gather_samples(local).cpu().numpy()


# row pool of one streamed segment: at most this many bytes (the segment then covers fewer rounds)
STREAM_POOL_BYTES = 16 << 30


class StreamedRounds:
    """The data generation of many VBOC iterations as ONE persistent device launch (vboc_data_generation_async).

    The reference regenerates num_prob problems per iteration with a synchronous Pool.map and refits in
    between (VBOC/triplependulum_vboc.py:493-568); `data_generation` never reads the model, so the ids of every
    iteration are known up front.  One producer launch on its own stream works through the ids of its rounds
    in order, and the host takes round r once all of its problems are finished (per-problem done flags, released
    to memory by the kernel, polled on a side stream) - while round r is being fitted on the default stream, the
    GPU keeps generating r + 1, r + 2, ...; no round pays its own tail.  `cancel()` skips the problems not yet
    started (the time budget is spent); `close()` ends the launch.

    round_ids: one id array per round (this rank's shard under torch.distributed; default: `rounds` rounds of
    num_prob consecutive ids from first_id).  The row pool holds the most a problem can save (2 (N_start + 12) + 2
    rows, quirk A.3 included), so it cannot overflow; a segment whose pool would pass STREAM_POOL_BYTES is the
    caller's to split (vboc_run's segments)."""

    def __init__(self, nq, solver, rounds=None, num_prob=None, first_id=0, N_start=None, seed=SEED, poll_s=0.005,
                 round_ids=None):
        import torch
        self.torch, self.nq, self.poll_s = torch, nq, poll_s
        self.solver = solver
        dev = torch.device("cuda", solver.device)
        if round_ids is None:
            round_ids = [np.arange(first_id + r * num_prob, first_id + (r + 1) * num_prob) for r in range(rounds)]
        self.sizes = [len(r) for r in round_ids]
        self.offs = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        B = int(self.offs[-1])
        N_start = int(N_start or system(nq).N)
        rpp = 2 * (N_start + 12) + 2
        self.ids = torch.as_tensor(np.concatenate(round_ids).astype(np.int64), device=dev)
        self.flags = torch.zeros(B, dtype=torch.int32, device=dev)
        self.cancel_word = torch.zeros(1, dtype=torch.int32, device=dev)
        self.producer = torch.cuda.Stream(dev)
        self.side = torch.cuda.Stream(dev)
        self.host_flags = torch.zeros(max(self.sizes + [1]), dtype=torch.int32).pin_memory()
        torch.cuda.synchronize(dev)
        self.t_start = time.time()
        # jobs in round order: a round's restart chains and parked resumes go before a later round's new problems
        # (dg.h round gate), so the rounds complete in order while the launch keeps every wave busy
        solver.set_option("dg_round", max(self.sizes))
        self.out = solver.data_generation_device(self.ids, N_start=N_start, seed=seed, rows_cap=B * rpp,
                                                 stream=self.producer, done_flag=self.flags, cancel=self.cancel_word,
                                                 wait=False)
        self.waited = 0.0
        self.closed = False

    @staticmethod
    def rounds_within(num_prob, nq, N_start=None, budget=STREAM_POOL_BYTES):
        """How many rounds of num_prob problems one segment's row pool holds within `budget` bytes (>= 1)."""
        rpp = 2 * (int(N_start or system(nq).N) + 12) + 2
        return max(1, int(budget // max(1, num_prob * rpp * 2 * nq * 8)))

    def round(self, r):
        """Results of round r in problem order (drivers.data_generation_batch's format) and its stats."""
        torch = self.torch
        sl = slice(int(self.offs[r]), int(self.offs[r + 1]))
        n = self.sizes[r]
        t = time.time()
        while n:
            with torch.cuda.stream(self.side):
                self.host_flags[:n].copy_(self.flags[sl], non_blocking=True)
            self.side.synchronize()
            if bool(self.host_flags[:n].all()):
                break
            time.sleep(self.poll_s)
        self.waited += time.time() - t
        out = self.out
        with torch.cuda.stream(self.side):
            cnt = out["row_cnt"][sl].to("cpu", non_blocking=True)
            off = out["row_off"][sl].to("cpu", non_blocking=True)
            st = out["stats"][sl].to("cpu", non_blocking=True)
            ic, slot = out["ic"][sl].to("cpu", non_blocking=True), out["ic_slot"][sl].to("cpu", non_blocking=True)
        self.side.synchronize()
        cnt, off, st, ic, slot = cnt.numpy(), off.numpy(), st.numpy(), ic.numpy(), slot.numpy()
        if (cnt < -1).any():
            raise RuntimeError(f"round {r}: row pool overflow (-2) or cancelled problems (-3): {np.unique(cnt[cnt < -1])}")
        used = cnt > 0
        lo = int(off[used].min()) if used.any() else 0
        hi = int((off + np.maximum(cnt, 0))[used].max()) if used.any() else 0
        with torch.cuda.stream(self.side):
            block = out["rows_all"][lo:hi].to("cpu", non_blocking=True)   # the round's blocks (released)
        self.side.synchronize()
        block = block.numpy()
        results = []
        for b in range(n):
            samples = None if cnt[b] < 0 else block[off[b] - lo:off[b] - lo + cnt[b]].tolist()
            if self.nq == 2:
                icb = [int(ic[b, 0])] + ic[b, 1:].tolist()
                results.append((samples, icb, None) if slot[b] == 1 else (None, None, icb))
            else:
                results.append(samples)
        return results, dict(solves=int(st[:, 0].sum()), rk4=int(st[:, 1].sum()), sqp_iter=int(st[:, 2].sum()),
                             rounds=1, per_problem=st)

    def cancel(self):
        with self.torch.cuda.stream(self.side):
            self.cancel_word.fill_(1)
        self.side.synchronize()

    def close(self):
        if self.closed:
            return None
        self.closed = True
        out = self.solver.data_generation_wait(self.out)
        return dict(seconds=time.time() - self.t_start, spec_solves=out["spec_solves"], spec_used=out["spec_used"],
                    waited_s=self.waited)


class SegmentedProducer:
    """The VBOC loop's data generation as consecutive streamed segments of `R` rounds each: round `it` comes from
    the segment that covers it; once the loop passes a segment's last round (all of its problems consumed) the
    next segment starts at `it`.  So the time budget stays the only stop rule of a run without an iteration limit
    (the reference's `while time.time() - start_time < stop_time`, VBOC/triplependulum_vboc.py:493).
    make_segment(first_round, rounds) -> an object with round(r), cancel(), close() (StreamedRounds)."""

    def __init__(self, make_segment, R, last_round=None):
        self.make, self.R, self.last = make_segment, int(R), last_round
        self.seg, self.first, self.infos = None, 0, []

    def round(self, it):
        if self.seg is None or it >= self.first + self.R:
            if self.seg is not None:
                self.infos.append(self.seg.close())
            n = self.R if self.last is None else max(1, min(self.R, self.last + 1 - it))
            self.seg, self.first = self.make(it, n), it
        return self.seg.round(it - self.first)

    def close(self, cancel=True):
        if self.seg is not None:
            if cancel:
                self.seg.cancel()
            self.infos.append(self.seg.close())
            self.seg = None
        infos = [i for i in self.infos if i]
        if not infos:
            return None
        return dict(segments=len(infos), seconds=sum(i["seconds"] for i in infos),
                    spec_solves=sum(i["spec_solves"] for i in infos), spec_used=sum(i["spec_used"] for i in infos),
                    waited_s=sum(i["waited_s"] for i in infos))


def _agree(flag):
    """Rank 0's decision on every rank (the time budget must not split the ranks' loop counts)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return flag
    t = torch.tensor([int(flag)], dtype=torch.int64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    dist.broadcast(t, 0)
    return bool(t.item())


def vboc_run(nq, backend, X_test, stop_time, num_prob=1000, max_iterations=None, N_start=None, seed=SEED,
             out_dir=None, device=None, trainer_kw=None, triple_refit_quirk=True, log=None, stream=None,
             stream_rounds=None, segment_factory=None):
    """Run the VBOC loop; returns dict(X_save, mean, std, trainer, times, rmse, stats).
    stream (default: on the GPU backend): the iterations' data generation runs as producer launches ahead of the
    fits (StreamedRounds), each over stream_rounds iterations (default: max_iterations + 1, else 64, capped by the
    row-pool budget STREAM_POOL_BYTES); when the loop passes a launch's last iteration the next launch starts
    (SegmentedProducer), so without an iteration limit the time budget is the only stop rule, as in the reference.
    Under torch.distributed every rank streams its own shard of each iteration's ids (np.array_split, the same
    shards as the synchronous rounds) and each iteration's samples are all-gathered (RCCL) in problem order; rank 0
    fits, and rank 0's stop decision is broadcast.  Problems not reached when the loop stops are cancelled.
    segment_factory(first_round, rounds) replaces StreamedRounds (tests)."""
    import torch
    import torch.distributed as dist
    if nq not in (2, 3):
        raise NotImplementedError("the pendulum VBOC driver uses the free-time OCP (pendulum_vboc.py:54), "
                                  "which the boundary solver does not implement")
    log = log or (lambda *a: None)
    rank0 = not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0
    device = device or ("cuda" if torch.cuda.is_available() else "cpu")
    t0 = time.time()
    iteration = 0
    solver = getattr(backend, "solver", None)
    if stream is None:
        stream = segment_factory is not None or (
            solver is not None and hasattr(solver, "data_generation_device") and
            solver.nmax >= (N_start or system(nq).N) + 12)
    producer = None
    if stream:
        R = stream_rounds or ((max_iterations + 1) if max_iterations is not None else 64)
        R = min(R, StreamedRounds.rounds_within(num_prob, nq, N_start))
        make = segment_factory or (lambda first, n: StreamedRounds(
            nq, solver, N_start=N_start, seed=seed, round_ids=[_rank_ids(first + r, num_prob) for r in range(n)]))
        producer = SegmentedProducer(make, R, last_round=max_iterations)

        def get_round(it):
            res, st = producer.round(it)
            return _gather_rows(samples_array(nq, res)), st
    else:
        get_round = lambda it: _round(nq, backend, it, num_prob, N_start, seed)
    times, rmse, fits, stats = [], [], [], []
    trainer = None
    try:
        X_save, st = get_round(iteration)
        stats.append(st)
        log(f"iteration 0: {X_save.shape[0]} rows")
        mean, std = position_stats(X_save, nq)
        F = dir_features(X_save, mean, std, nq)
        F_test = dir_features(X_test, mean, std, nq)
        trainer = make_trainer(nq, device, **(trainer_kw or {})) if rank0 else None
        if rank0:
            fits.append(trainer.fit(F))
            times.append(time.time() - t0)
            rmse.append(trainer.rmse(F_test))
            log(f"fit: {fits[-1]}  rmse {rmse[-1]:.4g}")
        while _agree(time.time() - t0 < stop_time and (max_iterations is None or iteration < max_iterations)):
            iteration += 1
            X_new, st = get_round(iteration)
            stats.append(st)
            X_save = np.concatenate((X_save, X_new))
            if rank0:
                src = X_save if (nq == 3 and triple_refit_quirk) else X_new
                F_new = dir_features(src, mean, std, nq)
                F = np.concatenate((F, F_new))
                fits.append(trainer.fit(F, n_new=F_new.shape[0]))
                times.append(time.time() - t0)
                rmse.append(trainer.rmse(F_test))
                log(f"iteration {iteration}: {X_save.shape[0]} rows, fit {fits[-1]}, rmse {rmse[-1]:.4g}")
    finally:
        # an exception anywhere above must not leave a producer launch running on the handle
        producer_info = producer.close(cancel=True) if producer is not None else None
    if rank0 and out_dir is not None:
        save_artifacts(out_dir, nq, X_save, mean, std, trainer.model, times, rmse)
    return dict(X_save=X_save, mean=mean, std=std, trainer=trainer, times=times, rmse=rmse, stats=stats, fits=fits,
                producer=producer_info)


def pendulum_vboc_run(out_dir=None, device="cuda", seed=0, backend=None, it_max=None):
    """VBOC/pendulum_vboc.py's main block: the simplified data generation (two free-time sweeps,
    :52-223, drivers.pendulum_data_generation), features [(q - mean) / std, sign(dq), |dq|] (:226-236),
    the 2-100-1 fit (Adam lr 1e-3, minibatch 64, EMA beta 0.8, stop at val <= 1e-4 or it_max =
    100 * int(n * 100 / 64) steps, :241-277), the RMSE on the training data (:296-301) and the
    artefacts data_1dof_vboc_10.npy, model_/mean_/std_1dof_vboc_10 (:239, :290-292).
    Difference kept explicit: rows with dq = 0 get direction 0 here; the reference leaves that entry
    of an np.empty array uninitialised (:230-235).  Returns dict(X, rmse, fit, stats)."""
    import torch
    from .drivers import GpuBackend, pendulum_data_generation
    backend = backend or GpuBackend(1, nmax=200)
    X, stats = pendulum_data_generation(backend)
    mean, std = position_stats(X, 1)
    F = dir_features(X, mean, std, 1)
    tr = make_trainer(1, device=device, beta=0.8, stop_val=1e-4, seed=seed)
    B = int(X.shape[0] * 100 / tr.k)
    # the reference counts it from 0 (`while val > 1e-4 and it < it_max`), the trainer from 1
    fit = tr.fit(F, it_max=(it_max or B * 100) + 1)
    rmse = tr.rmse(F)
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        np.save(os.path.join(out_dir, "data_1dof_vboc_10.npy"), np.asarray(X))
        torch.save({k: v.detach().cpu() for k, v in tr.model.state_dict().items()},
                   os.path.join(out_dir, "model_1dof_vboc_10"))
        torch.save(mean, os.path.join(out_dir, "mean_1dof_vboc_10"))
        torch.save(std, os.path.join(out_dir, "std_1dof_vboc_10"))
    return dict(X=X, rmse=rmse, fit=fit, stats=stats, mean=mean, std=std)


def ur5_run(backend=None, num_test=10000, num_train=100000, out_dir=None, device="cuda", seed=0,
            minibatch=1 << 15, hidden=1000, log=None, resume=False):
    """VBOC/UR5/vboc_multiprocessing_ur5.py's main block (config 5), on one GPU or sharded over the ranks of
    torch.distributed (config 5's 8 MI355X: each rank one contiguous share of every id range, rows all-gathered):
      test set      `testing_test` over ids [0, num_test) (:487-498)      -> data_4dof_vboc_test.npy
      training set  `testing_test` over ids [num_test, + num_train) (:506-528) -> data_4dof_vboc_train.npy
      features      [(q - mean) / std, qdot / |qdot|, |qdot|] with the position mean / std of the training set
                    (the reference's commented-out computation, :546-548; it loads them from files)
      fit           NeuralNetDIR(8, 1000, 1), Adam lr 1e-3, minibatch 2^15, EMA beta 0.95, stop at val <= 1e-3
                    or it_max = 20 * int(n * 100 / 2^15) steps (:530-595), on the HIP-graph trainer
      RMSE          on the training and the test data (:597-625); artefacts model_/mean_/std_4dof_vboc.
    resume: the reference appends the new rows to the training set of a previous run (X_old = np.load of
    data_4dof_vboc_train.npy, :501; X_tot = concatenate((X_old, X_save)), :530) and fits on all of it.  With
    resume=True and out_dir holding a previous run, X_old is loaded the same way and the new problems continue
    after the previous run's ids (data_4dof_vboc_train.next_id, written by every run), so a resumed run adds
    new initial states instead of repeating the Philox-keyed ones.  Returns dict(X_test, X_train, fit,
    rmse_train, rmse_test, stats)."""
    import torch
    from .drivers import GpuBackend, ur5_set, ur5_testing_batch, ur5_testing_device
    log = log or (lambda *a: None)
    backend = backend or GpuBackend(4, nmax=400)   # some arm problems extend past 100 stages (tools/testing_probe.py)
    t0 = time.time()
    dev = _device_solver(backend, 112)
    tt = (lambda ids: ur5_testing_device(ids, dev)) if dev is not None else (lambda ids: ur5_testing_batch(ids, backend))
    # under torch.distributed every rank runs a contiguous shard of each id range and the rows are all-gathered in
    # rank (= problem) order (the reference's Pool.map over range(num_prob), :487-528); rank 0 fits and writes
    res, st_test = tt(_shard(np.arange(num_test)))
    X_test = _gather_rows(ur5_set(res).reshape(-1, 8))
    log(f"test set: {X_test.shape[0]} rows of {num_test} in {time.time() - t0:.1f} s")
    t1 = time.time()
    first, X_old = num_test, np.zeros((0, 8))
    old_path = os.path.join(out_dir, "data_4dof_vboc_train.npy") if out_dir else None
    if resume:
        if not (old_path and os.path.exists(old_path)):
            raise FileNotFoundError("ur5_run(resume=True) needs out_dir with a previous data_4dof_vboc_train.npy")
        X_old = np.load(old_path)                      # allow_pickle=False: plain float64 rows
        with open(old_path[:-4] + ".next_id") as f:
            first = int(f.read())
    res, st_train = tt(_shard(np.arange(first, first + num_train)))
    X_save = _gather_rows(ur5_set(res).reshape(-1, 8))
    X_train = np.concatenate((X_old, X_save))
    log(f"training set: {X_save.shape[0]} new rows of {num_train} in {time.time() - t1:.1f} s, "
        f"{X_train.shape[0]} with the previous run's")
    mean, std = position_stats(X_train, 4)
    if not _is_rank0():
        return dict(X_test=X_test, X_train=X_train, fit=None, rmse_train=None, rmse_test=None,
                    stats=(st_test, st_train), mean=mean, std=std)
    F = dir_features(X_train, mean, std, 4)
    F_test = dir_features(X_test, mean, std, 4)
    k = min(minibatch, F.shape[0])
    tr = make_trainer(4, device=device, hidden=hidden, minibatch=k, beta=0.95, stop_val=1e-3, seed=seed)
    B = int(F.shape[0] * 100 / k)
    fit = tr.fit(F, it_max=max(1, B * 20))
    rmse_train, rmse_test = tr.rmse(F), tr.rmse(F_test)
    log(f"fit {fit}  RMSE train {rmse_train:.4g} test {rmse_test:.4g}")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        np.save(os.path.join(out_dir, "data_4dof_vboc_test.npy"), X_test)
        np.save(os.path.join(out_dir, "data_4dof_vboc_train.npy"), X_train)
        with open(os.path.join(out_dir, "data_4dof_vboc_train.next_id"), "w") as f:
            f.write(str(first + num_train))
        torch.save({kk: v.detach().cpu() for kk, v in tr.model.state_dict().items()},
                   os.path.join(out_dir, "model_4dof_vboc"))
        torch.save(mean, os.path.join(out_dir, "mean_4dof_vboc"))
        torch.save(std, os.path.join(out_dir, "std_4dof_vboc"))
    return dict(X_test=X_test, X_train=X_train, fit=fit, rmse_train=rmse_train, rmse_test=rmse_test,
                stats=(st_test, st_train), mean=mean, std=std)


def cartesian_run(backend=None, num_test=1000, num_train=100000, out_dir=None, device="cuda", seed=0,
                  minibatch=4096, hidden=300, log=None):
    """The main block of VBOC/Cartesian constraints/vboc_multiprocessing.py (double pendulum with the end-effector
    keep-out circle), on one GPU or sharded over the ranks of torch.distributed like ur5_run:
      test set      `testing_test` over ids [0, num_test) (:557-562)
      training set  `testing_test` over ids [num_test, + num_train) (:567-585)  -> data_2dof_vboc_10.npy (5 columns,
                    dt included, as the reference saves X_save)
      features      [(q - mean) / std, qdot / |qdot|] -> |qdot| with the scalar position mean / std of the training
                    set (:600-615)
      fit           NeuralNetRegression(4, 300, 1) (same layers as NeuralNetDIR), Adam lr 1e-3, minibatch 4096,
                    EMA beta 0.95, stop at val <= 1e-3 or it_max = 100 * int(n * 100 / 4096) steps (:617-660), on
                    the HIP-graph trainer
      RMSE          on the training and the test data (:662-690); artefacts model_/mean_/std_2dof_vboc_10_300.
    backend: a drivers backend carrying the circle (default: GpuBackend(2, path_constraint=...)).  Returns
    dict(X_test, X_train, fit, rmse_train, rmse_test, stats)."""
    import torch
    from .drivers import GpuBackend, cartesian_testing_batch, cartesian_testing_device
    from .systems import cartesian_constraint
    log = log or (lambda *a: None)
    backend = backend or GpuBackend(2, nmax=200, path_constraint=cartesian_constraint())
    rows = lambda res: np.array([r for t in res if t is not None for r in t], dtype=np.float64).reshape(-1, 5)
    t0 = time.time()
    dev = _device_solver(backend, 112)
    tt = (lambda ids: cartesian_testing_device(ids, dev)) if dev is not None else \
        (lambda ids: cartesian_testing_batch(ids, backend))
    # under torch.distributed: per-rank contiguous shards, rows all-gathered in problem order, rank 0 fits and writes
    res, st_test = tt(_shard(np.arange(num_test)))
    X_test = _gather_rows(rows(res))
    log(f"test set: {X_test.shape[0]} rows of {num_test} in {time.time() - t0:.1f} s")
    t1 = time.time()
    res, st_train = tt(_shard(np.arange(num_test, num_test + num_train)))
    X_train = _gather_rows(rows(res))
    log(f"training set: {X_train.shape[0]} rows of {num_train} in {time.time() - t1:.1f} s")
    mean, std = position_stats(X_train, 2)
    if not _is_rank0():
        return dict(X_test=X_test, X_train=X_train, fit=None, rmse_train=None, rmse_test=None,
                    stats=(st_test, st_train), mean=mean, std=std)
    F = dir_features(X_train, mean, std, 2)
    F_test = dir_features(X_test, mean, std, 2)
    k = min(minibatch, F.shape[0])
    tr = make_trainer(2, device=device, hidden=hidden, minibatch=k, beta=0.95, stop_val=1e-3, seed=seed)
    B = int(F.shape[0] * 100 / k)
    fit = tr.fit(F, it_max=max(1, B * 100))
    rmse_train, rmse_test = tr.rmse(F), tr.rmse(F_test)
    log(f"fit {fit}  RMSE train {rmse_train:.4g} test {rmse_test:.4g}")
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        tag = f"2dof_vboc_10_{hidden}"
        np.save(os.path.join(out_dir, "data_2dof_vboc_10.npy"), X_train)
        torch.save({kk: v.detach().cpu() for kk, v in tr.model.state_dict().items()}, os.path.join(out_dir, "model_" + tag))
        torch.save(mean, os.path.join(out_dir, "mean_" + tag))
        torch.save(std, os.path.join(out_dir, "std_" + tag))
    return dict(X_test=X_test, X_train=X_train, fit=fit, rmse_train=rmse_train, rmse_test=rmse_test,
                stats=(st_test, st_train), mean=mean, std=std)
