"""Active learning's labelling OCP (AL/triplependulum_class_al.py:148-169, compute_problem of OCPtriplependulumINIT)
and its driver testing(s0) (AL/triplependulum_al.py:24-42): the oracle restatement (oracle/vboc_oracle_ft.c
vboc_oracle_al_solve_batch) pinned independently, the batched driver against the reference's own function, and the
GPU solver (vboc_al_solve_batch, csrc/ft.h) against the oracle.

Pins of the oracle (CPU):
  * every label equals the feasibility of the linearised QP, decided by scipy's LP solver (tests/al_reference.py) -
    no part of the solver under test involved;
  * a label-1 step satisfies the linearised QP's constraints (dynamics, boxes, terminal rest) to 1e-8;
  * a QP the interior-point solver has not finished after qp_solver_iter_max (50) iterations is a failure by this
    restatement's definition (HPIPM's own status there is unpinned): such problems are counted - a feasible QP at the
    cap would be labelled 0 against the LP - and capped at 2 % of the sample (measured: 0).
The driver: tests/golden/al_testing_3.json is the reference's testing(s0), AST-extracted and run on the oracle
(tests/golden/make_driver_golden.py al); vboc_amd.al.testing_batch on the same oracle reproduces it exactly."""
import json
import os

import numpy as np
import pytest

import oracle
from al_reference import lp_feasible, step_violation
from vboc_amd.al import AlSpec, nn_guess, out_of_bounds, unlabeled_states
from vboc_amd.al import testing_batch as al_testing_batch

HERE = os.path.dirname(os.path.abspath(__file__))
CAP_SHARE = 0.02


def in_bounds_states(spec, n, seed):
    S = unlabeled_states(spec, 2 * n, np.random.default_rng(seed))
    return np.array([s for s in S if not out_of_bounds(spec, s)][:n])


def oracle_label_fn(spec):
    def fn(X):
        r = oracle.al_solve_batch(spec, X)
        return r["label"], r["x"]
    return fn


def test_oracle_labels_are_the_linearised_qps_feasibility():
    spec = AlSpec()
    S = in_bounds_states(spec, 96, seed=11)
    r = oracle.al_solve_batch(spec, S)
    feas = np.array([lp_feasible(spec, s) for s in S])
    assert set(np.unique(r["status"])) <= {0, 4}
    capped_feasible = int(((r["qp_iter"] >= spec.qp_iter_max) & feas).sum())
    assert capped_feasible <= CAP_SHARE * len(S), capped_feasible
    wrong = np.flatnonzero((r["label"] == 1) != feas)
    # a disagreement is allowed only as a feasible QP stopped at the iteration cap (counted above)
    assert all(feas[i] and r["qp_iter"][i] >= spec.qp_iter_max for i in wrong), [(int(i), bool(feas[i]),
                                                                               int(r["qp_iter"][i])) for i in wrong]
    # both classes present: the sample exercises feasibility and infeasibility
    assert 0 < feas.sum() < len(S)
    for i in np.flatnonzero(r["label"] == 1):
        assert step_violation(spec, S[i], r["x"][i], r["u"][i]) < 1e-8, i


def test_oracle_terminal_rest_and_fixed_x0():
    spec = AlSpec()
    S = in_bounds_states(spec, 24, seed=12)
    r = oracle.al_solve_batch(spec, S)
    ok = r["label"] == 1
    assert ok.any()
    assert np.abs(r["x"][:, 0] - S).max() == 0.0                     # x_0 pinned by lbx = ubx (:154-155)
    assert np.abs(r["x"][ok, -1, 3:]).max() < 1e-9                   # zero final velocity (:210-216)


def test_testing_batch_reproduces_reference_driver_on_oracle():
    g = json.load(open(os.path.join(HERE, "golden", "al_testing_3.json")))
    spec = AlSpec()
    X = np.array(g["X"])
    got = al_testing_batch(spec, X, oracle_label_fn(spec))
    assert len(got) == len(g["results"])
    for b, (a, ref) in enumerate(zip(got, g["results"])):
        if ref is None:
            assert a is None, b
            continue
        assert a[0] == ref[0], b
        assert (a[1] is None) == (ref[1] is None), b
        if ref[1] is not None:
            assert np.array_equal(np.asarray(a[1]), np.asarray(ref[1])), b
    n_out = sum(out_of_bounds(spec, s) for s in X)
    n_feas = sum(r is not None and r[0][-1] == 1 for r in g["results"])
    assert n_out > 0 and n_feas > 0 and n_feas < len(X) - n_out


def guess_network(g, spec):
    """The fixture's guess network (seeded NeuralNetCLS(6, 500, 6 N)) and the scalar statistics of its states."""
    import torch
    from vboc_amd.learn import NeuralNetCLS
    torch.manual_seed(g["guess_seed"])
    model = NeuralNetCLS(6, 500, 6 * spec.N)
    Xt = torch.Tensor(np.array(g["X"]))
    return model, torch.mean(Xt), torch.std(Xt)


def oracle_guess_label_fn(spec, model, mean, std):
    def fn(X):
        xg = np.stack([nn_guess(spec.N, s[:3], s[3:], model, mean, std) for s in X])
        r = oracle.al_solve_batch(spec, X, x_guess=xg)
        return r["label"], r["x"]
    return fn


def _same_driver_results(got, ref, tol=0.0):
    assert len(got) == len(ref)
    for b, (a, r) in enumerate(zip(got, ref)):
        if r is None:
            assert a is None, b
            continue
        assert a[0] == r[0], b
        assert (a[1] is None) == (r[1] is None), b
        if r[1] is not None:
            assert np.abs(np.asarray(a[1]) - np.asarray(r[1])).max() <= tol, b


def test_testing_guess_reproduces_reference_driver_on_oracle():
    """testing_guess (AL/triplependulum_al.py:44-62) with compute_problem_nnguess: the fixture's guess network's
    trajectories as the stage guesses; every label also equals the LP feasibility of the QP linearised there."""
    g = json.load(open(os.path.join(HERE, "golden", "al_testing_3.json")))
    spec = AlSpec()
    X = np.array(g["X"])
    model, mean, std = guess_network(g, spec)
    got = al_testing_batch(spec, X, oracle_guess_label_fn(spec, model, mean, std))
    _same_driver_results(got, g["results_guess"])
    S = np.array([s for s in X if not out_of_bounds(spec, s)])
    xg = np.stack([nn_guess(spec.N, s[:3], s[3:], model, mean, std) for s in S])
    r = oracle.al_solve_batch(spec, S, x_guess=xg)
    feas = np.array([lp_feasible(spec, s, x) for s, x in zip(S, xg)])
    assert 0 < feas.sum() < len(S)
    # label 1 only on a feasible QP; a feasible QP labelled 0 is one the interior point has not finished at the
    # 50-iteration cap - with this untrained network's guesses (linearisation points far from feasibility) most of the
    # feasible ones (33 of 40, measured); the count is printed, the reference's HPIPM status there is unpinned
    capped = (r["label"] == 0) & feas
    assert all(r["qp_iter"][i] >= spec.qp_iter_max for i in np.flatnonzero(capped))
    assert not ((r["label"] == 1) & ~feas).any()
    print(f"testing_guess: {feas.sum()} LP-feasible of {len(S)}, labelled 1: {(r['label'] == 1).sum()}, feasible at the "
          f"QP cap: {capped.sum()}")
    for i in np.flatnonzero(r["label"] == 1):
        assert step_violation(spec, S[i], r["x"][i], r["u"][i], xg[i]) < 1e-8, i


# --------------------------------------------------------------------------------------------------------------
# GPU
# --------------------------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_labels_match_oracle():
    from vboc_amd.al import OCPtriplependulumINIT
    ocp = OCPtriplependulumINIT()
    spec = ocp.spec
    S = in_bounds_states(spec, 512, seed=13)
    g = ocp.compute_problem_batch(S)
    r = oracle.al_solve_batch(spec, S)
    diff = np.flatnonzero(g["label"] != r["label"])
    # a label may differ only where one side stops at the QP iteration cap (a rounding-level difference in the last
    # iterations), capped at 1 % and counted
    assert all(max(g["qp_iter"][i], r["qp_iter"][i]) >= spec.qp_iter_max for i in diff), diff
    assert len(diff) <= 0.01 * len(S), len(diff)
    ok = (g["label"] == 1) & (r["label"] == 1)
    assert ok.sum() > 0.2 * len(S)
    assert np.abs(g["x"][ok] - r["x"][ok]).max() < 1e-7
    assert np.abs(g["u"][ok] - r["u"][ok]).max() < 1e-6
    same_iter = (g["qp_iter"] == r["qp_iter"]).mean()
    assert same_iter >= 0.95, same_iter


@pytest.mark.gpu
def test_gpu_testing_driver_reproduces_fixture():
    from vboc_amd.al import OCPtriplependulumINIT
    g = json.load(open(os.path.join(HERE, "golden", "al_testing_3.json")))
    ocp = OCPtriplependulumINIT()
    got = al_testing_batch(ocp.spec, np.array(g["X"]), ocp.labels)
    for b, (a, ref) in enumerate(zip(got, g["results"])):
        if ref is None:
            assert a is None, b
            continue
        assert a[0] == ref[0], b
        if ref[1] is not None:
            assert np.abs(np.asarray(a[1]) - np.asarray(ref[1])).max() < 1e-7, b


@pytest.mark.gpu
def test_gpu_testing_guess_driver_reproduces_fixture():
    """testing_guess on the GPU against the reference's function on the oracle, both fed the same network guesses
    (evaluated once, on this host): every state as the oracle's, except a state whose label parts because one side's
    QP stopped at the 50-iteration cap (with the untrained network's guesses most feasible QPs end near the cap,
    DESIGN.md section 20); those are counted and capped at 10 %.  The fixture itself was made with the guesses of the
    container's CPU; the FP32 network rounds differently on another host's CPU, which moves near-cap QPs across the cap
    (state 6 on the round-6 box) and moves every RTI point by the network's FP32 rounding, so against the fixture the
    labels are held to 90 % agreement and the trajectories of agreeing label-1 states to 1e-5 (6.2e-7 seen on the
    round-6 box; 0 where the host's guesses equal the container's)."""
    from vboc_amd.al import OCPtriplependulumINIT
    g = json.load(open(os.path.join(HERE, "golden", "al_testing_3.json")))
    ocp = OCPtriplependulumINIT()
    spec = ocp.spec
    model, mean, std = guess_network(g, spec)
    X = np.array(g["X"])
    S = np.array([s for s in X if not out_of_bounds(spec, s)])
    xg = np.stack([nn_guess(spec.N, s[:3], s[3:], model, mean, std) for s in S])
    import torch
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda")
    out = ocp.solver.al_solve_device(spec, T(S), x_guess=T(xg))
    torch.cuda.synchronize()
    lg, xgpu, ig = (out[k].cpu().numpy() for k in ("label", "x", "qp_iter"))
    rr = oracle.al_solve_batch(spec, S, x_guess=xg)
    cap = np.maximum(ig, rr["qp_iter"]) >= spec.qp_iter_max
    diff = np.flatnonzero(lg != rr["label"])
    assert all(cap[i] for i in diff), diff
    print(f"network guesses: sum {xg.sum():.17g}")
    print(f"testing_guess on the GPU: {len(diff)} of {len(S)} states part from the oracle at the QP cap: {diff}")
    assert len(diff) <= 0.1 * len(S), diff
    ok = (lg == 1) & (rr["label"] == 1)
    assert np.abs(xgpu[ok] - rr["x"][ok]).max() < 1e-7
    got = al_testing_batch(spec, X, ocp.labels_nnguess(model, mean, std))
    ref = g["results_guess"]
    agree = 0
    for b, (a, r) in enumerate(zip(got, ref)):
        if (a is None) != (r is None) or (a is not None and a[0] != r[0]):
            continue
        agree += 1
        if r is not None and r[1] is not None:
            assert np.abs(np.asarray(a[1]) - np.asarray(r[1])).max() < 1e-5, b
    print(f"testing_guess on the GPU against the fixture: {agree} of {len(X)} states agree")
    assert agree >= 0.9 * len(X), agree
    S = np.array(g["X"])[:8]
    for s in S:
        if out_of_bounds(ocp.spec, s):
            continue
        assert ocp.compute_problem_nnguess(s[:3], s[3:], model, mean, std) in (0, 1)


@pytest.mark.gpu
def test_gpu_dropin_compute_problem():
    from vboc_amd.al import OCPtriplependulumINIT
    ocp = OCPtriplependulumINIT()
    spec = ocp.spec
    S = in_bounds_states(spec, 8, seed=14)
    r = oracle.al_solve_batch(spec, S)
    for i, s in enumerate(S):
        res = ocp.compute_problem(s[:3], s[3:])
        assert res == r["label"][i]
        if res == 1:
            assert np.abs(np.array([ocp.ocp_solver.get(k, "x") for k in range(ocp.N + 1)]) - r["x"][i]).max() < 1e-7


@pytest.mark.gpu
def test_gpu_al_error_codes_and_empty_batch():
    """The C ABI's argument checks: an nq != 3 handle is refused (VBOC_ERR_UNSUPPORTED), a horizon past nmax is an
    argument error, an empty batch is a no-op."""
    import ctypes
    import torch
    from vboc_amd import lib
    spec = AlSpec()
    s2 = lib.Solver(2, 100)
    x0 = torch.zeros((4, 6), dtype=torch.float64, device="cuda:0")
    with pytest.raises(lib.VbocError, match="nq = 3"):
        s2.al_solve_device(spec, x0)
    s3 = lib.Solver(3, 50)
    with pytest.raises(lib.VbocError, match="nmax"):
        s3.al_solve_device(spec, x0)
    s = lib.Solver(3, 100)
    out = s.al_solve_device(spec, torch.zeros((0, 6), dtype=torch.float64, device="cuda:0"))
    torch.cuda.synchronize()
    assert out["label"].numel() == 0
