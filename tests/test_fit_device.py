"""The VBOC loop's NN fit on the device (vboc_amd/csrc/fit.hip via learn.HipTrainer) against a plain PyTorch fp32
restatement of the reference's loop (VBOC/triplependulum_vboc.py:446-466: random.sample minibatch, MSELoss,
torch.optim.Adam(lr 1e-3), val = beta val + (1 - beta) loss.item()).

The torch reference is fed the device sampler's own minibatch indices (a second trainer with the same seed
replays the sampler's stream), so gradients, Adam moments and parameters are compared step for step.  Tolerances:
exp_avg after one step (= 0.1 g) within 2e-5 of max|g| per tensor (f32 GEMM summation order), parameters after
five steps within 1e-5 absolute (Adam moves each by <= lr = 1e-3 per step).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fit_library_exports_every_declared_symbol():
    import re
    from vboc_amd import fitlib
    hdr = open(os.path.join(HERE, "..", "include", "vboc_fit.h")).read()
    declared = set(re.findall(r"\b(vboc_fit_\w+)\s*\(", hdr))
    assert declared == set(fitlib.EXPORTS)
    lib = ctypes.CDLL(fitlib.LIB_PATH)
    for name in declared:
        getattr(lib, name)


def test_make_trainer_picks_torch_on_cpu_and_for_unsupported_shapes():
    from vboc_amd import fitlib
    from vboc_amd.learn import DirTrainer, make_trainer
    assert type(make_trainer(3, "cpu")) is DirTrainer
    assert type(make_trainer(3, "cpu", native=True)) is DirTrainer
    assert fitlib.supported(6, 500, 4096) and fitlib.supported(4, 300, 4096) and fitlib.supported(2, 100, 64)
    assert not fitlib.supported(8, 1000, 32768) and not fitlib.supported(6, 500, 8192)


def _features(n, nq, seed=0):
    from vboc_amd.learn import dir_features, position_stats
    rng = np.random.default_rng(seed)
    X = np.c_[rng.uniform(3 * np.pi / 4, 5 * np.pi / 4, (n, nq)), rng.uniform(-10, 10, (n, nq))]
    m, s = position_stats(X, nq)
    return dir_features(X, m, s, nq)


def _torch_steps(model, opt, F, nin, idx_steps, val, beta):
    crit = torch.nn.MSELoss()
    for idx in idx_steps:
        ii = torch.as_tensor(idx, dtype=torch.long, device="cuda")
        x = F[ii, :nin]
        y = F[ii, nin:nin + 1]
        loss = crit(model(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        val = beta * val + (1 - beta) * loss.item()
    return val


@pytest.mark.gpu
@pytest.mark.parametrize("nq,refit", [(3, False), (3, True), (2, False), (1, False)])
def test_device_fit_matches_torch_adam_loop(nq, refit):
    import copy
    from vboc_amd.learn import HipTrainer
    Fn = _features(30000 if nq > 1 else 3000, nq, seed=nq)
    nin = 2 * nq
    n_new = Fn.shape[0] // 3 if refit else 0
    F = torch.as_tensor(Fn, dtype=torch.float32, device="cuda")
    a = HipTrainer(nq, "cuda", seed=5)
    twin = HipTrainer(nq, "cuda", seed=5)
    idx = twin.sample(Fn.shape[0], n_new, steps=5).cpu().numpy()
    ref = copy.deepcopy(a.model)
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    val0 = float(Fn[:, nin].max())
    # one step: Adam's exp_avg = (1 - 0.9) g exposes the gradient
    r1 = a.fit(Fn, n_new=n_new, it_max=2)
    assert r1["iterations"] == 1
    v_ref = _torch_steps(ref, opt, F, nin, idx[:1], val0, a.beta)
    m_dev, v_dev = a.moments()
    for p, md, vd in zip(ref.parameters(), m_dev, v_dev):
        mr = opt.state[p]["exp_avg"]
        scale = float(mr.abs().max()) + 1e-30
        assert float((md - mr).abs().max()) <= 2e-5 * scale, (p.shape, float((md - mr).abs().max()), scale)
        vr = opt.state[p]["exp_avg_sq"]
        assert float((vd - vr).abs().max()) <= 5e-5 * float(vr.abs().max()) + 1e-30
    assert abs(r1["val"] - v_ref) <= 1e-5 * abs(v_ref)
    for p, q in zip(a.model.parameters(), ref.parameters()):
        assert float((p - q).abs().max()) <= 1e-5
    # four more steps (a refit call continues the same optimizer and sampler stream)
    r2 = a.fit(Fn, n_new=n_new, it_max=5)
    assert r2["iterations"] == 4
    v_ref = _torch_steps(ref, opt, F, nin, idx[1:5], float(Fn[:, nin].max()), a.beta)
    assert abs(r2["val"] - v_ref) <= 1e-5 * abs(v_ref)
    for p, q in zip(a.model.parameters(), ref.parameters()):
        assert float((p - q).abs().max()) <= 2e-5


@pytest.mark.gpu
def test_device_fit_graph_replay_equals_eager_and_stops_exactly():
    """poll-64 graph replays == step-by-step launches, bit for bit, on a run that stops on val (not it_max)."""
    from vboc_amd.learn import HipTrainer
    Fn = _features(20000, 3, seed=3)
    Fn[:, 6] = 0.0                                       # targets 0 but one: val starts at 1, the EMA decays
    Fn[0, 6] = 1.0                                       # below the stop within a few hundred steps
    a = HipTrainer(3, "cuda", seed=9, graphs=True, poll=64)
    b = HipTrainer(3, "cuda", seed=9, graphs=False, poll=1)
    ra, rb = a.fit(Fn, it_max=5000), b.fit(Fn, it_max=5000)
    assert ra["iterations"] == rb["iterations"] < 4999, (ra, rb)
    assert ra["val"] == rb["val"] and ra["val"] <= 1e-3
    assert rb["launched"] == rb["iterations"] + 1 and ra["launched"] % 64 == 0
    for p, q in zip(a.model.parameters(), b.model.parameters()):
        assert torch.equal(p, q)


@pytest.mark.gpu
def test_sampler_is_a_uniform_subset_of_each_range():
    from vboc_amd.learn import HipTrainer
    tr = HipTrainer(1, "cuda", seed=1, minibatch=32)
    # direct path (2k <= n) and the complement path (2k > n): every row equally likely, no repeats
    for n, n_new, steps in [(100, 0, 3000), (40, 0, 3000), (100, 40, 3000), (80, 30, 3000)]:
        idx = tr.sample(n, n_new, steps=steps).cpu().numpy()
        assert idx.min() >= 0 and idx.max() < n
        assert all(len(np.unique(r)) == 32 for r in idx)
        parts = [(0, n, 32)] if not n_new else [(0, n - n_new, 16), (n - n_new, n, 16)]
        for c, (lo, hi, kk) in enumerate(parts):
            sub = idx[:, c * kk:(c + 1) * kk] if n_new else idx
            assert sub.min() >= lo and sub.max() < hi
            cnt = np.bincount(sub.ravel() - lo, minlength=hi - lo)
            e = steps * kk / (hi - lo)
            chi2 = float(((cnt - e) ** 2 / e).sum())
            dof = hi - lo - 1
            assert chi2 < dof + 6 * np.sqrt(2 * dof), (n, n_new, chi2, dof)
    # a long range (the configs[2] refit size): distinct and inside each half
    tr3 = HipTrainer(3, "cuda", seed=2)
    idx = tr3.sample(3_000_000, 1_500_000, steps=4).cpu().numpy()
    for r in idx:
        assert len(np.unique(r)) == 4096
        assert r[:2048].max() < 1_500_000 <= r[2048:].min() and r.max() < 3_000_000


@pytest.mark.gpu
def test_device_fit_learns_like_the_torch_trainer():
    """2 000 steps of the triple's fit: the device trainer's RMSE on held-out rows within 15 % of DirTrainer's."""
    from vboc_amd.learn import DirTrainer, HipTrainer
    F = _features(60000, 3, seed=11)
    Ft = _features(5000, 3, seed=12)
    h = HipTrainer(3, "cuda", seed=4)
    d = DirTrainer(3, "cuda", seed=4, graphs=False)
    h.fit(F, it_max=2001)
    d.fit(F, it_max=2001)
    rh, rd = h.rmse(Ft), d.rmse(Ft)
    assert abs(rh - rd) <= 0.15 * rd, (rh, rd)


@pytest.mark.gpu
def test_make_trainer_defaults_to_pytorch_on_gpu():
    """north_star keeps the NN fit on PyTorch-ROCm: the loop's trainer is DirTrainer unless the native one is asked
    for (native=True, the device trainer of csrc/fit.hip)."""
    from vboc_amd.learn import DirTrainer, HipTrainer, make_trainer
    assert type(make_trainer(3, "cuda")) is DirTrainer
    assert type(make_trainer(3, "cuda", native=True)) is HipTrainer
