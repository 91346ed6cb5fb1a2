"""NN fit / RMSE / artefacts of the VBOC loop (vboc_amd.learn, vboc_amd.pipeline) against plain
PyTorch restatements of the reference (VBOC/triplependulum_vboc.py:407-215, my_nn.py)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn as nn
from numpy.linalg import norm

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _ref_features(X, mean, std, nq):
    """The reference's per-row loop (VBOC/triplependulum_vboc.py:55-65)."""
    out = np.empty((X.shape[0], 2 * nq + 1))
    for i in range(X.shape[0]):
        for j in range(nq):
            out[i][j] = (X[i][j] - mean) / std
        vel_norm = norm([X[i][nq + j] for j in range(nq)])
        if vel_norm != 0:
            for j in range(nq):
                out[i][nq + j] = X[i][nq + j] / vel_norm
        out[i][2 * nq] = vel_norm
    return out


def _data(n, nq, seed=0):
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(3 * np.pi / 4, 5 * np.pi / 4, (n, nq)), rng.uniform(-10, 10, (n, nq))]
    X[3, nq:] = 0.0
    return X


@pytest.mark.parametrize("nq", [3, 2, 1])
def test_features_and_stats_match_reference(nq):
    from vboc_amd.learn import dir_features, position_stats
    X = _data(20000, nq)
    mean, std = position_stats(X, nq)
    t = torch.tensor(X[:, :nq].tolist())
    assert mean == torch.mean(t).item() and std == torch.std(t).item()
    got = dir_features(X, mean, std, nq)
    ref = _ref_features(X, mean, std, nq)
    got[3, nq:2 * nq] = ref[3, nq:2 * nq] = 0.0     # the reference leaves np.empty garbage there
    np.testing.assert_array_equal(torch.Tensor(got), torch.Tensor(ref))   # what the model sees
    np.testing.assert_allclose(got, ref, rtol=1e-15, atol=0)   # last-bit norm rounding


def test_model_layout_is_the_reference_state_dict():
    from vboc_amd.learn import NeuralNetDIR
    sd = NeuralNetDIR(6, 500, 1).state_dict()
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [
        ("linear_relu_stack.0.weight", (500, 6)), ("linear_relu_stack.0.bias", (500,)),
        ("linear_relu_stack.2.weight", (500, 500)), ("linear_relu_stack.2.bias", (500,)),
        ("linear_relu_stack.4.weight", (1, 500)), ("linear_relu_stack.4.bias", (1,))]


def _plain_fit(trainer_seed, F, nq, hidden, k, it_max, n_new=0, init=None):
    """Plain PyTorch restatement of the reference loop (:71-99 / :156-184) with the SAME minibatch
    indices as DirTrainer (same generator draws) and torch.optim.Adam."""
    from vboc_amd.learn import NeuralNetDIR
    torch.manual_seed(trainer_seed)
    model = NeuralNetDIR(2 * nq, hidden, 1)
    if init is not None:
        model.load_state_dict(init)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    crit = nn.MSELoss()
    from vboc_amd.learn import DirTrainer
    gen = torch.Generator().manual_seed(DirTrainer.fit_seed(trainer_seed, 1))   # the trainer's first fit
    Ft = torch.tensor(F, dtype=torch.float32)
    n = F.shape[0]
    it, val = 1, max(F[:, 2 * nq])
    val = float(torch.tensor(val, dtype=torch.float32))
    while val > 1e-3 and it < it_max:
        def samp(lo, hi, kk):
            return torch.topk(torch.rand(hi - lo, generator=gen), kk, sorted=False).indices + lo
        idx = torch.cat([samp(0, n - n_new, k // 2), samp(n - n_new, n, k // 2)]) if n_new else samp(0, n, k)
        out = model(Ft[idx, :2 * nq])
        loss = crit(out, Ft[idx, 2 * nq:])
        loss.backward()
        opt.step()
        opt.zero_grad()
        val = 0.95 * val + (1 - 0.95) * loss.item()
        it += 1
    return model, it


def test_trainer_equals_plain_adam_loop():
    from vboc_amd.learn import DirTrainer, dir_features, position_stats
    nq, hidden, k = 3, 32, 128
    X = _data(3000, nq)
    m, s = position_stats(X, nq)
    F = dir_features(X, m, s, nq)
    tr = DirTrainer(nq, "cpu", hidden=hidden, minibatch=k, seed=5)
    r = tr.fit(F, it_max=40)
    model, it = _plain_fit(5, F, nq, hidden, k, 40)
    assert r["iterations"] == it - 1 == 39
    for a, b in zip(tr.model.parameters(), model.parameters()):
        np.testing.assert_allclose(a.detach().numpy(), b.detach().numpy(), rtol=2e-4, atol=2e-6)
    # refit: half old / half new rows (:156-166); continues from the fitted model and Adam state
    X2 = _data(1000, nq, seed=1)
    F2 = np.concatenate((F, dir_features(X2, m, s, nq)))
    r2 = tr.fit(F2, n_new=1000, it_max=10)
    assert r2["iterations"] == 9


def test_trainer_stop_rule_is_exact():
    """The gated device-side stop test: iterations = the reference loop's count even though the
    host polls the flag only every `poll` steps."""
    from vboc_amd.learn import DirTrainer, dir_features, position_stats
    nq = 2
    X = _data(2000, nq)
    m, s = position_stats(X, nq)
    F = dir_features(X, m, s, nq)
    F[:, 4] = 0.02                       # easy target: the EMA crosses the threshold quickly
    tr = DirTrainer(nq, "cpu", hidden=16, minibatch=64, seed=3, stop_val=5e-3, poll=7)
    r = tr.fit(F, it_max=10**6)
    # the same trainer polling after every step is the reference's per-step loop
    tr1 = DirTrainer(nq, "cpu", hidden=16, minibatch=64, seed=3, stop_val=5e-3, poll=1)
    r1 = tr1.fit(F, it_max=10**6)
    assert r["iterations"] == r1["iterations"] and r["launched"] >= r1["launched"]
    assert r["val"] <= 5e-3
    for a, b in zip(tr.model.parameters(), tr1.model.parameters()):
        np.testing.assert_array_equal(a.detach().numpy(), b.detach().numpy())


def test_rmse_and_predict_batches():
    from vboc_amd.learn import DirTrainer
    tr = DirTrainer(3, "cpu", hidden=16, minibatch=64)
    F = np.random.default_rng(0).uniform(0, 1, (70000, 7))
    out = tr.predict(F[:, :6], batch=1 << 15)
    with torch.no_grad():
        ref = tr.model(torch.Tensor(F[:, :6]))
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-6, atol=1e-7)
    r = tr.rmse(F)
    assert abs(r - float(torch.sqrt(nn.MSELoss()(ref, torch.Tensor(F[:, 6:]))))) < 1e-6


def test_pipeline_round_trip_on_oracle(tmp_path):
    """Two VBOC iterations of the double pendulum on the oracle backend, artefacts written in the
    reference's formats and read back with weights_only loads."""
    from oracle_backend import OracleBackend
    from vboc_amd.drivers import data_generation_batch
    from vboc_amd.pipeline import load_artifacts, make_test_set, samples_array, vboc_run
    nq = 2
    X_test, _ = make_test_set(nq, OracleBackend(nq), num_prob=8, out_dir=str(tmp_path))
    assert np.load(tmp_path / "data2_test.npy").shape == (8, 4)
    out = vboc_run(nq, OracleBackend(nq), X_test, stop_time=1e9, num_prob=6, max_iterations=1,
                   out_dir=str(tmp_path), trainer_kw=dict(hidden=16, minibatch=32))
    res0, _ = data_generation_batch(nq, np.arange(6), OracleBackend(nq))
    res1, _ = data_generation_batch(nq, np.arange(6, 12), OracleBackend(nq))
    np.testing.assert_array_equal(out["X_save"], np.concatenate((samples_array(nq, res0), samples_array(nq, res1))))
    art = load_artifacts(str(tmp_path), nq)
    np.testing.assert_array_equal(art["data"], out["X_save"])
    assert art["mean"] == out["mean"] and art["std"] == out["std"]
    assert len(art["times"]) == len(art["rmse"]) == 2
    for a, b in zip(art["model"].parameters(), out["trainer"].model.parameters()):
        np.testing.assert_array_equal(a.detach().numpy(), b.detach().cpu().numpy())


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from vboc_amd.dist import gather_samples
    rows = torch.arange(rank * 10, rank * 10 + 3 * (rank + 1) * 4, dtype=torch.float64).reshape(-1, 4)  # 3 / 6 rows
    out = gather_samples(rows)
    q.put((rank, out.numpy()))
    dist.destroy_process_group()


def test_gather_samples_ragged_two_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29613
    ps = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    exp = np.concatenate([np.arange(0, 12, dtype=float).reshape(-1, 4), np.arange(10, 34, dtype=float).reshape(-1, 4)])
    for r in range(2):
        np.testing.assert_array_equal(got[r], exp)


def test_chunked_sampler_is_the_single_topk_subset():
    """A range longer than TOPK_CHUNK is sampled as the top-k of per-chunk top-k candidates: the same index set
    as one top-k over all keys, distinct and inside [lo, hi)."""
    from vboc_amd.learn import DirTrainer
    tr = DirTrainer(3, "cpu", graphs=False)
    for chunk, n, k in [(1000, 5500, 64), (1000, 4000, 1000), (4096, 4097, 2048)]:
        tr.TOPK_CHUNK = chunk
        tr.gen.manual_seed(5)
        idx = tr._sample(10, 10 + n, k)
        g = torch.Generator()
        g.manual_seed(5)
        ref = torch.topk(torch.rand(n, generator=g), k).indices + 10
        assert sorted(idx.tolist()) == sorted(ref.tolist())


@pytest.mark.gpu
def test_trainer_graph_replay_equals_eager_on_gpu():
    """HIP-graph replay (poll every 64 steps, gated updates) == eager per-step loop, on cuda:0."""
    from vboc_amd.learn import DirTrainer, dir_features, position_stats
    nq = 3
    X = _data(50000, nq)
    m, s = position_stats(X, nq)
    F = dir_features(X, m, s, nq)
    a = DirTrainer(nq, "cuda", seed=11, graphs=True, poll=64)
    b = DirTrainer(nq, "cuda", seed=11, graphs=False)
    ra, rb = a.fit(F, it_max=300), b.fit(F, it_max=300)
    assert ra["iterations"] == rb["iterations"] == 299
    for p, q in zip(a.model.parameters(), b.model.parameters()):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)
    assert abs(a.rmse(F) - b.rmse(F)) < 1e-4


@pytest.mark.gpu
def test_vboc_loop_on_gpu(tmp_path):
    """Test set + two VBOC iterations of the triple pendulum with the GPU solver and GPU training."""
    from vboc_amd.drivers import GpuBackend
    from vboc_amd.pipeline import load_artifacts, make_test_set, vboc_run
    nq = 3
    be = GpuBackend(nq)
    X_test, st = make_test_set(nq, be, num_prob=256, first_id=10**7, out_dir=str(tmp_path))
    assert X_test.shape == (256, 6)
    out = vboc_run(nq, be, X_test, stop_time=1e9, num_prob=256, max_iterations=1, out_dir=str(tmp_path))
    assert out["X_save"].shape[0] > 4096 and len(out["rmse"]) == 2
    assert all(np.isfinite(out["rmse"]))
    art = load_artifacts(str(tmp_path), nq, device="cuda")
    np.testing.assert_array_equal(art["rmse"], out["rmse"])


@pytest.mark.gpu
def test_large_refit_with_graphs_on_gpu():
    """A refit at configs[2]'s scale (1.5M old + 1.5M new feature rows, HIP-graph replay) runs and samples inside
    each half: the 1.5M-key top-k this replaced faulted the GPU (profiles/r03f_vboc_loop_fault.log)."""
    from vboc_amd.learn import DirTrainer
    nq = 3
    n = 3_000_000
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    F = torch.rand((n, 2 * nq + 1), device="cuda", generator=g)
    tr = DirTrainer(nq, "cuda", seed=2, graphs=True, poll=64)
    tr.it_max = 10**9
    r = tr.fit(F, n_new=n // 2, it_max=256)
    assert r["iterations"] == 255 and np.isfinite(r["val"])
    idx = tr._sample(n // 2, n, 2048)
    assert idx.min().item() >= n // 2 and idx.max().item() < n and torch.unique(idx).numel() == 2048


@pytest.mark.gpu
def test_consecutive_captured_fits_on_gpu():
    """Verdict r03 item 2: consecutive HIP-graph-captured fits in ONE process, at the shapes of the configs[2] loop
    whose third fit faulted in round 3 (profiles/r03f_vboc_loop_fault.log: a first fit, then refits whose halves
    grow past 2^20 rows; the triple's refit quirk makes the new half all of X_save), each a new capture over new
    feature tensors, then the UR5's 8-1000-1 fit (minibatch 2^15) twice on the same trainer class.  Every fit
    runs its steps and keeps the parameters finite."""
    from vboc_amd.learn import DirTrainer
    nq = 3
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    tr = DirTrainer(nq, "cuda", seed=4, graphs=True, poll=64)
    tr.it_max = 10**9
    for n, n_new in ((500_000, 0), (1_010_000, 505_000), (2_520_000, 1_510_000), (4_030_000, 2_520_000)):
        F = torch.rand((n, 2 * nq + 1), device="cuda", generator=g)
        r = tr.fit(F, n_new=n_new, it_max=192)
        assert r["iterations"] == 191 and np.isfinite(r["val"]), (n, r)
        del F
    assert all(torch.isfinite(p).all() for p in tr.model.parameters())
    arm = DirTrainer(4, "cuda", hidden=1000, minibatch=1 << 15, seed=1, graphs=True, poll=64)
    for n, n_new in ((200_000, 0), (400_000, 200_000)):
        F = torch.rand((n, 9), device="cuda", generator=g)
        r = arm.fit(F, n_new=n_new, it_max=128)
        assert r["iterations"] == 127 and np.isfinite(r["val"])
    assert all(torch.isfinite(p).all() for p in arm.model.parameters())


class _FakeSegment:
    """A streamed segment (StreamedRounds' interface) over precomputed rounds: round r of the segment starting at
    `first` returns the host driver's results for iteration first + r (oracle backend), or synthetic rows."""
    made = []

    def __init__(self, first, n, rounds_fn):
        self.first, self.n, self.fn, self.cancelled = first, n, rounds_fn, False
        _FakeSegment.made.append((first, n))

    def round(self, r):
        assert 0 <= r < self.n
        return self.fn(self.first + r)

    def cancel(self):
        self.cancelled = True

    def close(self):
        return dict(seconds=0.0, spec_solves=0, spec_used=0, waited_s=0.0)


def test_streamed_segments_equal_synchronous_rounds_on_oracle():
    """vboc_run's segmented producer (stream_rounds = 2 rounds per launch, 5 iterations -> segments [0, 1], [2, 3],
    [4]) trains on exactly the rows of the synchronous round-by-round loop."""
    from oracle_backend import OracleBackend
    from vboc_amd.pipeline import _generate, vboc_run
    nq, n = 2, 4
    be = OracleBackend(nq)
    X_test = np.tile([np.pi, np.pi, 1.0, 1.0], (4, 1))
    kw = dict(stop_time=1e9, num_prob=n, max_iterations=4, trainer_kw=dict(hidden=8, minibatch=16, stop_val=1e9))
    sync = vboc_run(nq, be, X_test, stream=False, **kw)
    _FakeSegment.made = []
    fn = lambda it: _generate(nq, be, np.arange(it * n, (it + 1) * n), None, 20250124)
    seg = vboc_run(nq, be, X_test, stream_rounds=2, segment_factory=lambda f, k: _FakeSegment(f, k, fn), **kw)
    assert _FakeSegment.made == [(0, 2), (2, 2), (4, 1)]
    assert seg["producer"]["segments"] == 3
    np.testing.assert_array_equal(seg["X_save"], sync["X_save"])


def test_time_budget_is_the_only_stop_rule_of_a_streamed_run():
    """without an iteration limit a streamed run must not stop when its first launch's rounds run out
    (stream_rounds = 2): the next segment starts and the loop runs until the time budget is spent."""
    import time as _t
    from vboc_amd.pipeline import vboc_run
    nq = 3

    def fn(it):
        _t.sleep(0.15)
        rows = [[[3.0 + 0.01 * (it % 7), 3.1, 3.2, 1.0 + 0.1 * b, -1.0, 0.5]] for b in range(8)]
        return rows, dict(solves=8, rk4=0, sqp_iter=8, rounds=1)
    _FakeSegment.made = []
    X_test = np.tile([3.0, 3.1, 3.2, 1.0, -1.0, 0.5], (4, 1))
    out = vboc_run(nq, None, X_test, stop_time=2.0, num_prob=8, stream_rounds=2,
                   segment_factory=lambda f, k: _FakeSegment(f, k, fn),
                   trainer_kw=dict(hidden=8, minibatch=8, stop_val=1e9))
    assert len(out["stats"]) > 4                       # past the first segment's 2 rounds
    assert len(_FakeSegment.made) >= 3 and all(k == 2 for _, k in _FakeSegment.made)
    assert out["producer"]["segments"] == len(_FakeSegment.made)
