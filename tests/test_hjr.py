"""HJR one-step OCP (compute_problem of HJR/<sys>_hjr_class.py): the oracle restatement (oracle/vboc_oracle_hjr.c)
pinned independently, and the GPU solver (vboc_amd.hjr, csrc/hjr.h) against it.

The network is a NeuralNetCLS(2nq, 100, 2) with seeded torch initialisation (the reference trains it on its own
labels; any weights define a valid instance of the OCP).  Pins of the oracle (CPU):
  * KKT at the final iterate, recomputed here from the oracle's multipliers with the golden-pinned RK4
    sensitivities and an independent numpy evaluation of the network and its gradient;
  * scipy SLSQP on min_u NN_0(RK4(x0, u)) over the torque box, started at the oracle's u: no lower cost.
Problems whose SQP stops at max_iter are kinks of the ReLU network (stationarity cannot reach 1e-6 there); the
reference labels them 0 (compute_problem returns 0 for any status != 0), and so does this port.
"""
import numpy as np
import pytest
from scipy.optimize import minimize

import oracle

NQ_BOX = {1: 3.0, 2: 10.0, 3: 10.0}


def make_net(nq, seed=0):
    import torch
    torch.manual_seed(seed)
    net = torch.nn.Sequential(torch.nn.Linear(2 * nq, 100), torch.nn.ReLU(), torch.nn.Linear(100, 100),
                              torch.nn.ReLU(), torch.nn.Linear(100, 2))
    return [p.detach().numpy().astype(np.float64) for p in net.parameters()], net


def states(nq, B, seed=1):
    rng = np.random.default_rng(seed)
    return np.c_[rng.uniform(3 * np.pi / 4, 5 * np.pi / 4, (B, nq)), rng.uniform(-10, 10, (B, nq))]


MEAN, STD = 1.5, 4.5


def nn_np(W, x):
    """Logit 0 and its gradient in numpy (independent of the oracle's C)."""
    z0 = (x - MEAN) / STD
    a1 = W[0] @ z0 + W[1]
    h1 = np.maximum(a1, 0.0)
    a2 = W[2] @ h1 + W[3]
    h2 = np.maximum(a2, 0.0)
    out = W[4][0] @ h2 + W[5][0]
    g = W[0].T @ ((W[2].T @ (W[4][0] * (a2 > 0))) * (a1 > 0)) / STD
    return out, g


def shoot(nq, x0, u):
    if nq > 1:
        x1, _, B = oracle.rk4_sens(nq, 1e-2, x0, u)
        return x1, B
    # the undamped pendulum of HJR/pendulum_hjr_class.py (finite differences are enough for the checks)
    def f(x, uu):
        return np.array([x[1], (0.5 * 9.81 * 0.3 * np.sin(x[0]) + uu[0]) / (0.3 * 0.3 * 0.5)])
    def rk(uu):
        h = 1e-2
        k1 = f(x0, uu); k2 = f(x0 + h / 2 * k1, uu); k3 = f(x0 + h / 2 * k2, uu); k4 = f(x0 + h * k3, uu)
        return x0 + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
    x1 = rk(u)
    B = ((rk(u + 1e-6) - rk(u - 1e-6)) / 2e-6)[:, None]
    return x1, B


@pytest.mark.parametrize("nq", [3, 2, 1])
def test_hjr_oracle_kkt_and_no_descent(nq):
    W, _ = make_net(nq)
    X0 = states(nq, 24)
    r = oracle.hjr_solve_batch(nq, X0, W, MEAN, STD)
    ok = np.flatnonzero(r["status"] == 0)
    assert ok.size >= 12, r["status"]
    umax = NQ_BOX[nq]
    for i in ok:
        x1, B = shoot(nq, X0[i], r["u"][i])
        c, g = nn_np(W, r["x1"][i])
        assert abs(c - r["cost"][i]) < 1e-12
        assert np.abs(x1 - r["x1"][i]).max() < 1e-6                              # dynamics
        pi, ll, lu = r["pi"][i], r["lam_l"][i], r["lam_u"][i]
        stat = max(np.abs(g - pi).max(), np.abs(B.T @ pi - ll + lu).max())
        assert stat < (1e-6 if nq > 1 else 1e-5), (i, stat)                     # stationarity
        u = r["u"][i]
        assert np.all(np.abs(u) <= umax + 1e-6) and ll.min() >= 0 and lu.min() >= 0
        assert max(np.abs(ll * (u + umax)).max(), np.abs(lu * (umax - u)).max()) < 1e-6   # complementarity
        # no lower cost near the oracle's u (SLSQP on the reduced NLP, box only)
        fun = lambda uu: nn_np(W, shoot(nq, X0[i], uu)[0])[0]
        s = minimize(fun, u, method="SLSQP", bounds=[(-umax, umax)] * nq, options=dict(maxiter=200, ftol=1e-12))
        assert s.fun > r["cost"][i] - 1e-6, (i, s.fun, r["cost"][i])


def test_hjr_labelling_driver_matches_reference_semantics():
    """vboc_amd.hjr.hjr_labels (HJR/triplependulum_hjr.py:21-40) with the oracle as the OCP: candidates outside
    the box or predicted 0 get [1, 0] without a solve; solved ones [0, 1] iff cost < 0; unsolved (None, None)."""
    from vboc_amd.hjr import hjr_labels
    W, _ = make_net(3)

    class OracleHjr:
        def compute_problems(self, X):
            r = oracle.hjr_solve_batch(3, X, W, MEAN, STD)
            return (r["status"] == 0).astype(np.int64), r

    X = states(3, 40)
    X[:4, 3] = 12.0                      # outside the velocity box
    pred = np.array([1, 0] * 20)
    out = hjr_labels(OracleHjr(), X, pred)
    r = oracle.hjr_solve_batch(3, X, W, MEAN, STD)
    for i, (state, lab) in enumerate(out):
        if i < 4 or pred[i] == 0:
            assert lab == [1, 0] and np.array_equal(state, X[i])
        elif r["status"][i] == 0:
            assert lab == ([0, 1] if r["cost"][i] < 0 else [1, 0])
        else:
            assert state is None and lab is None


@pytest.mark.gpu
@pytest.mark.parametrize("nq", [3, 2, 1])
def test_hjr_gpu_matches_oracle(nq):
    """GPU (one problem per lane) vs the oracle on 256 states: the same status on >= 95 %, and on problems both
    solve the same cost (1e-9) and controls (1e-6)."""
    from vboc_amd.hjr import OCPdoublependulum, OCPpendulum, OCPtriplependulum
    W, net = make_net(nq)
    X0 = states(nq, 256, seed=7)
    ocp = {3: OCPtriplependulum, 2: OCPdoublependulum, 1: OCPpendulum}[nq](MEAN, STD, net.parameters())
    lab, g = ocp.compute_problems(X0)
    r = oracle.hjr_solve_batch(nq, X0, W, MEAN, STD)
    same = np.mean(g["status"] == r["status"])
    assert same >= 0.95, same
    both = (g["status"] == 0) & (r["status"] == 0)
    assert both.sum() >= 0.4 * len(X0)
    assert np.abs(g["cost"][both] - r["cost"][both]).max() < 1e-9
    assert np.abs(g["u"][both] - r["u"][both]).max() < 1e-6
    assert np.array_equal(lab, (g["status"] == 0).astype(np.int64))
    # the drop-in single-problem call
    x = X0[int(np.flatnonzero(both)[0])]
    res = ocp.compute_problem(x) if nq > 1 else ocp.compute_problem(x[0], x[1])
    assert res == 1 and abs(ocp.ocp_solver.get_cost() - r["cost"][int(np.flatnonzero(both)[0])]) < 1e-9


def _fixture():
    import json
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    g = json.load(open(os.path.join(here, "golden", "hjr_3.json")))
    z = np.load(os.path.join(here, "golden", "hjr_net_3.npz"))
    return g, [z[f"arr_{i}"] for i in range(6)]


def _same(a, b):
    (sa, la), (sb, lb) = a, b
    return la == lb and ((sa is None and sb is None) or (sa is not None and sb is not None and np.array_equal(sa, sb)))


def test_hjr_labels_reproduce_reference_function():
    """tests/golden/hjr_3.json: the reference's own data_generation (HJR/triplependulum_hjr.py:21-40, AST-extracted,
    tests/golden/make_driver_golden.py hjr) over 96 candidates on the oracle; hjr_labels on the same oracle
    returns the same (state, output) pairs."""
    from vboc_amd.hjr import hjr_labels
    g, W = _fixture()

    class OracleHjr:
        def compute_problems(self, X):
            r = oracle.hjr_solve_batch(3, X, W, g["mean"], g["std"])
            return (r["status"] == 0).astype(np.int64), r

    out = hjr_labels(OracleHjr(), np.array(g["X"]), np.array(g["y_pred"]))
    ref = [(None if s is None else np.array(s), o) for s, o in g["results"]]
    bad = [i for i, (a, b) in enumerate(zip(out, ref)) if not _same(a, b)]
    assert not bad, bad


@pytest.mark.gpu
def test_hjr_labels_on_gpu_match_reference_function():
    """The same fixture with the GPU drop-in class (vboc_amd.hjr.OCPtriplependulum): >= 95 % of the candidates get
    the reference function's (state, output)."""
    from vboc_amd.hjr import OCPtriplependulum, hjr_labels
    g, W = _fixture()
    ocp = OCPtriplependulum(g["mean"], g["std"], W)
    out = hjr_labels(ocp, np.array(g["X"]), np.array(g["y_pred"]))
    ref = [(None if s is None else np.array(s), o) for s, o in g["results"]]
    same = sum(_same(a, b) for a, b in zip(out, ref))
    assert same >= 0.95 * len(ref), same
