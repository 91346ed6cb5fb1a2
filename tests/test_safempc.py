"""Safe MPC with the VBOC network as terminal constraint (VBOC/Safe MPC/
triplependulum_class_vboc.py:91-240, OCPtriplependulumHardTerm) on the batched solver.

Oracle pin (CPU): the C restatement (oracle/vboc_oracle_ft.c vboc_oracle_mpc_solve) lands on the optimum of an
independently written NLP (tests/nlp_reference.py slsqp_mpc: single-step RK4 defects, the LINEAR_LS cost, boxes,
the terminal row h(x_N) >= 0 with a finite-difference gradient): SLSQP started at the oracle's point does not
move, and started cold from the reference's constant guess it reaches the same cost.  The terminal row is active
at these optima (h(x_N) = 0 to rounding), so its IPM treatment is exercised.  ACADOS-level parity is unpinned (no
ACADOS here); the network is a seeded NeuralNetDIR(6, 500, 1) - the reference's trained
model_3dof_vboc is not in the repository - with its output bias raised so the row is active for some states.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import oracle  # noqa: E402

MEAN, STD = np.pi, 0.5


def _net():
    import torch
    from vboc_amd.learn import NeuralNetDIR
    from vboc_amd.safempc import nn_params
    torch.manual_seed(0)
    net = NeuralNetDIR(6, 500, 1)
    with torch.no_grad():
        net.linear_relu_stack[4].bias.fill_(4.0)
    return nn_params(net)


def _states(B, seed=1):
    from vboc_amd.safempc import MpcSpec
    sp = MpcSpec()
    rng = np.random.default_rng(seed)
    x0 = np.zeros((B, 6))
    x0[:, :3] = rng.uniform(sp.thetamin, sp.thetamax, (B, 3))
    x0[:, 3:] = rng.uniform(-2, 2, (B, 3))
    xg = np.repeat(x0[:, None, :], sp.N + 1, 1)
    ug = np.zeros((B, sp.N, 3))
    return sp, x0, xg, ug


def _capped(sp):
    """The oracle's options with the SQP stopped at 150 iterations instead of the class's 1000: the tests below compare
    the converged problems only, whose iterates do not depend on the cap (the problems still iterating at 150 spend
    most of the CPU suite's time otherwise)."""
    return oracle.default_opts(lm=sp.lm, tol_stat=1e-6, qp_tol_stat=1e-8, max_iter=150)


def test_spec_is_the_reference_ocp():
    from vboc_amd.safempc import MpcSpec
    sp = MpcSpec(4e-3, 0.148)
    assert sp.N == int(0.148 / 4e-3)                      # :105
    assert sp.W.tolist() == [1e-4, 1e4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4]
    assert sp.yref[1] == np.pi / 4 + np.pi - 0.05 and sp.yref[0] == sp.yref[2] == np.pi
    assert sp.cost_scale == 4e-3 and sp.lm == 1e-2


def test_nn_row_gradient_in_the_oracle_matches_finite_differences():
    """The oracle's h(x_N) equals vboc_amd.safempc.nn_row (the reference's nn_decisionfunction restated in numpy)
    at the solutions it returns."""
    from vboc_amd.safempc import nn_row
    P = _net()
    sp, x0, xg, ug = _states(8)
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, rti=True)
    for i in range(8):
        assert abs(h[i] - nn_row(P, MEAN, STD, x[i, -1])) < 1e-12


@pytest.mark.parametrize("with_row", [False, True])
def test_oracle_optimum_is_the_slsqp_optimum(with_row):
    from nlp_reference import slsqp_mpc
    P = _net() if with_row else None
    sp, x0, xg, ug = _states(16)
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, opts=_capped(sp))
    ok = np.flatnonzero(r["status"] == 0)
    assert ok.size >= 6
    if with_row:
        assert (h[ok] >= -1e-9).all() and (np.abs(h[ok]) < 1e-9).sum() >= 3   # the row is active at the optimum
    for i in ok[:2]:
        X, U, c, _ = slsqp_mpc(sp, x0[i], (x[i], u[i]), P, MEAN, STD)
        assert np.abs(X - x[i]).max() < 1e-6 and c > r["cost"][i] - 1e-7 * abs(r["cost"][i])
        X2, U2, c2, _ = slsqp_mpc(sp, x0[i], (xg[i], ug[i]), P, MEAN, STD, maxiter=1000)
        assert abs(c2 - r["cost"][i]) < 1e-7 * abs(r["cost"][i]), (c2, r["cost"][i])
        assert np.abs(X2 - x[i]).max() < 1e-3


def test_rti_is_one_qp_with_the_full_step():
    """SQP_RTI (the Safe-MPC drivers' option): one QP and its full step, status 0; the same as the first iteration
    of the SQP when that iteration's line search accepts alpha = 1."""
    P = _net()
    sp, x0, xg, ug = _states(8)
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, rti=True)
    assert (r["status"] == 0).all() and (r["sqp_iter"] == 1).all() and (r["qp_iter"] > 0).all()
    assert (x[:, 0] == x0).all()


def _oracle_solve(sp, P, rti):
    def solve(x0, xg, ug):
        x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, rti=rti)
        return dict(status=r["status"], x=x, u=u)
    return solve


def _oracle_rk4(sp):
    return lambda X, U: np.stack([oracle.rk4(3, sp.time_step, X[i], U[i]) for i in range(X.shape[0])])


def test_closed_loop_driver_on_the_oracle():
    """vboc_amd.safempc.simulate_batch (the reference's simulate(p), hard_terminal_constraints/3dof_sym.py:15-72)
    over a batch: the same per-problem result as running each problem alone, and the plant follows the applied
    controls."""
    from vboc_amd.safempc import simulate_batch
    P = _net()
    sp, x0, xg, ug = _states(4, seed=3)
    x0[:, 3:] = 0.0                                   # the drivers start at rest (x0[:nu] = data[p])
    xg = np.repeat(x0[:, None, :], sp.N + 1, 1)
    res, simX, solves = simulate_batch(_oracle_solve(sp, P, True), _oracle_rk4(sp), sp, x0, xg, ug, tot_steps=12)
    assert solves >= 4 and (res >= 0).all() and (res <= 11).all()
    for b in range(2):
        r1, X1, _ = simulate_batch(_oracle_solve(sp, P, True), _oracle_rk4(sp), sp, x0[b:b + 1], xg[b:b + 1],
                                   ug[b:b + 1], tot_steps=12)
        assert r1[0] == res[b]
        np.testing.assert_array_equal(X1[0], simX[b])


# ------------------------------------------------------------------------------------------------
# GPU: vboc_mpc_solve_batch (ft.h with the tracking cost and the terminal row) against the oracle
# ------------------------------------------------------------------------------------------------
def _gpu(sp, P, x0, xg, ug, rti, max_iter=None):
    import torch
    from vboc_amd import lib
    s = lib.Solver(3, sp.N)
    s.set_option("levenberg_marquardt", sp.lm)
    s.set_option("nlp_solver_tol_stat", 1e-6)
    s.set_option("qp_solver_tol_stat", 1e-8)
    if max_iter:
        s.set_option("nlp_solver_max_iter", max_iter)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda:0")
    prm = [T(p) for p in P] if P is not None else None
    out = s.mpc_solve_device(sp, T(x0), T(xg), T(ug), prm, MEAN, STD, rti=rti)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}


@pytest.mark.gpu
@pytest.mark.parametrize("with_row", [False, True])
def test_gpu_rti_matches_oracle(with_row):
    """SQP_RTI (the Safe-MPC drivers' mode) on 128 states: status, the QP's iteration count and the step agree with
    the oracle.  A QP stopped at qp_solver_iter_max (100) returns an unconverged interior-point iterate, which
    rounding moves freely (one problem of these 128: measured max |du| 2.9 there, 1e-8 elsewhere): the step
    bars apply to the QPs that converged."""
    P = _net() if with_row else None
    sp, x0, xg, ug = _states(128, seed=5)
    g = _gpu(sp, P, x0, xg, ug, rti=True)
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, rti=True)
    assert (g["status"] == r["status"]).mean() >= 0.98
    assert (g["qp_iter"] == r["qp_iter"]).mean() >= 0.95
    ok = (g["status"] == 0) & (r["status"] == 0) & (g["qp_iter"] < 100) & (r["qp_iter"] < 100)
    assert ok.mean() >= 0.9
    assert np.abs(g["u"][ok] - u[ok]).max() < 1e-6 and np.median(np.abs(g["x"][ok] - x[ok]).max(axis=(1, 2))) < 1e-9
    if with_row:
        assert np.abs(g["h"][ok] - h[ok]).max() < 1e-8


@pytest.mark.gpu
@pytest.mark.parametrize("with_row", [False, True])
def test_gpu_sqp_matches_oracle(with_row):
    """Full SQP (nlp_solver_max_iter 1000, the class's own setting, :153-161) on 96 states at the section-3 bars:
    status >= 98 %, SQP iterations >= 95 % or as close as the oracle is to itself under a 1e-15 perturbation (below),
    cost and x_N of problems converged on both: median <= 1e-9, max <= 2e-3 (relative to the cost).  From these random states (any position in the box, |dtheta| <= 2) the SQP to
    tol_stat 1e-6 stalls for about half of them: they reach 1000 iterations on both sides (status 2, the same
    problems), so the cost / x_N bars also apply to those - the two runs' 1000th iterates.  (At a cap of 200, 2 of
    96 problems that converge just before / after the 200th iteration on one side made the status bar 97.9 %.)"""
    P = _net() if with_row else None
    sp, x0, xg, ug = _states(96, seed=7)
    g = _gpu(sp, P, x0, xg, ug, rti=False, max_iter=1000)
    o = oracle.default_opts(lm=sp.lm, tol_stat=1e-6, qp_tol_stat=1e-8, max_iter=1000)
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, opts=o)
    assert (g["status"] == r["status"]).mean() >= 0.98, (g["status"], r["status"])
    # SQP iterations per problem, classified instead of an agreement bar: on this OCP the converged iteration count
    # moves with rounding (the oracle against itself with the guess perturbed by 1e-15 agrees on only 95 % / 74 % of
    # the problems, round 4).  A problem whose iteration counts differ must have reached the same optimum: both
    # converged (tol_stat 1e-6) with the cost to 1e-6 relative and x_N to 1e-3 - two KKT points to tol_stat 1e-6 of a
    # problem whose QP Hessian is >= levenberg_marquardt 1e-2 differ by at most ~1e-4 - or both stopped at the cap.
    moved = np.flatnonzero((g["sqp_iter"] != r["sqp_iter"]) & (g["status"] == r["status"]))
    dcm = np.abs(g["cost"] - r["cost"])[moved] / np.abs(r["cost"][moved])
    dxm = np.abs(g["x"][moved, -1] - x[moved, -1]).max(axis=1)
    print(f"{moved.size} problems with moved SQP-iteration counts, statuses {np.unique(g['status'][moved])}, "
          f"max rel dcost {dcm.max() if moved.size else 0:.2e}, max |dx_N| {dxm.max() if moved.size else 0:.2e}")
    assert set(np.unique(g["status"][moved]).tolist()) <= {0, 2}
    conv = g["status"][moved] == 0
    assert (dcm[conv] <= 1e-6).all() and (dxm[conv] <= 1e-3).all(), (moved, dcm, dxm)
    for st_, least in ((0, 30), (2, 40)):
        both = (g["status"] == st_) & (r["status"] == st_)
        assert both.sum() >= least, (st_, both.sum())
        dc = np.abs(g["cost"] - r["cost"])[both] / np.abs(r["cost"][both])
        dx = np.abs(g["x"][:, -1] - x[:, -1]).max(axis=1)[both]
        assert np.median(dc) <= 1e-9 and dc.max() <= 2e-3, (st_, np.median(dc), dc.max())
        assert np.median(dx) <= 1e-9 and dx.max() <= 2e-3, (st_, np.median(dx), dx.max())


# Per-step lockstep of a closed loop (the drivers' simulate): the loop runs on the GPU, and every MPC step's OCP is
# also solved by the oracle from the SAME inputs (state, shifted guesses, weights).  Each step pair is classified:
#   same    - equal status; for status 0 the applied u_0 and the predicted states agree to STEP_TOL;
#   cap     - a QP stopped at qp_solver_iter_max (100) - an unconverged interior-point iterate, which rounding moves
#             freely - while the other solver's QP also needed >= 50 iterations (a QP hard for both);
#   status  - the solvers returned different statuses for the same request;
#   value   - anything else: a defect.
# STEP_TOL: an RTI QP converged to qp_tol_stat 1e-8 on a Hessian >= levenberg_marquardt 1e-2 is within ~1e-6 of its
# solution; two such solves agree to 2e-6.
STEP_TOL = 2e-6


def _lockstep_solve(gpu_solve, ora_solve, pairs):
    def solve(x0, xg, ug, w=None):
        a = gpu_solve(x0, xg, ug, w) if w is not None else gpu_solve(x0, xg, ug)
        b = ora_solve(x0, xg, ug, w) if w is not None else ora_solve(x0, xg, ug)
        for j in range(x0.shape[0]):
            if a["status"][j] != b["status"][j]:
                k = "status"
            elif a["status"][j] != 0:
                k = "same"
            elif max(a["qp_iter"][j], b["qp_iter"][j]) >= 100:
                k = "cap" if min(a["qp_iter"][j], b["qp_iter"][j]) >= 50 else "value"
            else:
                d = max(np.abs(a["u"][j] - b["u"][j]).max(), np.abs(a["x"][j] - b["x"][j]).max())
                k = "same" if d <= STEP_TOL else "value"
            pairs.append(k)
        return a
    return solve


def _classify_closed_loop(pairs):
    counts = {k: pairs.count(k) for k in ("same", "cap", "status", "value")}
    print("closed-loop step pairs:", counts)
    assert counts["value"] == 0, counts
    assert counts["status"] <= max(2, len(pairs) // 100), counts   # reported and capped at 1 %
    return counts


def _gpu_hard_solve(ocp):
    def solve(x0, xg, ug):
        return ocp.solve_batch(x0, xg, ug)
    return solve


def _oracle_solve_q(sp, P, rti):
    def solve(x0, xg, ug):
        x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD, rti=rti)
        return dict(status=r["status"], x=x, u=u, qp_iter=r["qp_iter"])
    return solve


@pytest.mark.gpu
def test_gpu_closed_loop_matches_oracle():
    """The Safe-MPC closed loop (simulate_batch, SQP_RTI, 60 steps) of 48 initial states at rest on the GPU drop-in
    class, every step's OCP also solved by the oracle from the same inputs: every step pair classified (above), no
    'value'; QP-cap pairs reported (measured: 31 of 2 880), status pairs capped at 1 %.  (The trajectories themselves are not compared at a
    fixed tolerance: a closed loop feeds each step's QP tolerance into the next state.)"""
    from vboc_amd.safempc import OCPtriplependulumHardTerm, simulate_batch
    from vboc_amd import lib
    P = _net()
    sp, x0, xg, ug = _states(48, seed=9)
    x0[:, 3:] = 0.0
    xg = np.repeat(x0[:, None, :], sp.N + 1, 1)
    ocp = OCPtriplependulumHardTerm("SQP_RTI", sp.time_step, sp.tot_time, P, MEAN, STD)
    rk4 = lambda X, U: lib.rk4_host(3, sp.time_step, X, U)
    pairs = []
    simulate_batch(_lockstep_solve(_gpu_hard_solve(ocp), _oracle_solve_q(sp, P, True), pairs), rk4, sp, x0, xg, ug,
                   tot_steps=60)
    _classify_closed_loop(pairs)
    # the drop-in batch-of-one call gives the batched call's result
    st = ocp.OCP_solve(x0[0], xg[0], ug[0])
    r = ocp.solve_batch(x0[:1], xg[:1], ug[:1])
    assert st == r["status"][0] and np.array_equal(ocp.ocp_solver.get(3, "x"), r["x"][0, 3])


# ------------------------------------------------------------------------------------------------
# OCPtriplependulumSoftTraj (:242-304): the margin-scaled row on every stage, soft lower sides
# ------------------------------------------------------------------------------------------------
MARGIN = 2.0


def _soft_weights(N, kind):
    if kind == "soft_traj":                       # soft_traj_constraints/3dof_sym.py:102-105
        Zl = np.zeros(N + 1)
        Zl[N] = 1e6
        return Zl
    return np.full(N + 1, 1e2)                    # every stage penalised (the receding driver's kind of weights)


def test_soft_row_is_the_margin_scaled_network():
    """The oracle's row (vboc_oracle_mpc_row) equals vboc_amd.safempc.nn_row with the safety margin:
    nn_decisionfunction_conservative (:284-304), out * (100 - margin) / 100 - vn; margin < 0 the HardTerm row."""
    from vboc_amd.safempc import nn_row
    P = _net()
    sp, x0, xg, ug = _states(16, seed=11)
    h = oracle.mpc_row(x0, P, MEAN, STD, MARGIN)
    h0 = oracle.mpc_row(x0, P, MEAN, STD, -1.0)
    for i in range(16):
        assert abs(h[i] - nn_row(P, MEAN, STD, x0[i], safety_margin=MARGIN)) < 1e-12
        assert abs(h0[i] - nn_row(P, MEAN, STD, x0[i])) < 1e-12


def test_soft_oracle_optimum_is_the_slsqp_optimum():
    """The oracle's SoftTraj SQP optimum is the optimum of an independently written NLP with the slacks explicit
    (tests/nlp_reference.py slsqp_mpc_soft): SLSQP started at the oracle's point (slacks at the rows' violations)
    does not move and has the oracle's cost (slack penalties included), and started cold from the constant guess it
    reaches the same cost.  The soft rows are violated at these optima (slacks > 0 on the path, where Zl = 0)."""
    from nlp_reference import slsqp_mpc_soft
    from vboc_amd.safempc import nn_row
    P = _net()
    sp, x0, xg, ug = _states(16)
    Zl = _soft_weights(sp.N, "soft_traj")
    x, u, r, h = oracle.mpc_soft_solve_batch(sp, x0, xg, ug, P, MEAN, STD, MARGIN, Zl, rti=False, opts=_capped(sp))
    ok = np.flatnonzero(r["status"] == 0)
    assert ok.size >= 6
    for n, i in enumerate(ok[:2]):
        X, U, S, c, _ = slsqp_mpc_soft(sp, x0[i], (x[i], u[i]), P, MEAN, STD, MARGIN, Zl)
        assert np.abs(X - x[i]).max() < 1e-6 and abs(c - r["cost"][i]) < 1e-8 * abs(r["cost"][i]), (c, r["cost"][i])
        hk = np.array([nn_row(P, MEAN, STD, x[i, k], safety_margin=MARGIN) for k in range(sp.N + 1)])
        assert hk.min() < -1e-3 and S.max() > 1e-3 and -1e-2 < hk[-1] < 0.0   # path rows violated, the terminal one only
        # slightly: Zl = 1e6 there trades the cost against an L2 penalty (a slack of ~1e-4 costs ~1e-2)
        if n == 0:
            X2, U2, S2, c2, _ = slsqp_mpc_soft(sp, x0[i], (xg[i], ug[i]), P, MEAN, STD, MARGIN, Zl, maxiter=1000)
            assert abs(c2 - r["cost"][i]) < 1e-7 * abs(r["cost"][i]), (c2, r["cost"][i])
            assert np.abs(X2 - x[i]).max() < 1e-4


def test_soft_rows_with_zero_weights_are_free():
    """With zl = Zl = 0 on every stage the soft rows cost nothing: the SoftTraj optimum is the unconstrained
    (OCPtriplependulumSTD) optimum, up to the solvers' tolerances."""
    P = _net()
    sp, x0, xg, ug = _states(16)
    x, u, r, h = oracle.mpc_soft_solve_batch(sp, x0, xg, ug, P, MEAN, STD, MARGIN, np.zeros(sp.N + 1), rti=False,
                                             opts=_capped(sp))
    xs, us, rs, hs = oracle.mpc_solve_batch(sp, x0, xg, ug, None, rti=False, opts=_capped(sp))
    both = (r["status"] == 0) & (rs["status"] == 0)
    assert both.sum() >= 6
    assert np.abs(x[both] - xs[both]).max() < 1e-4 and np.abs(r["cost"][both] - rs["cost"][both]).max() < 1e-6


def test_soft_rti_is_one_qp():
    P = _net()
    sp, x0, xg, ug = _states(8)
    for kind in ("soft_traj", "all"):
        x, u, r, h = oracle.mpc_soft_solve_batch(sp, x0, xg, ug, P, MEAN, STD, MARGIN, _soft_weights(sp.N, kind))
        assert (r["status"] == 0).all() and (r["sqp_iter"] == 1).all() and (r["qp_iter"] > 0).all()
        assert (x[:, 0] == x0).all()


def _fixture():
    g = np.load(os.path.join(HERE, "golden", "mpc_drivers.npz"))
    from vboc_amd.safempc import MpcSpec, halton_states
    sp = MpcSpec(4e-3, 0.148)
    x0 = halton_states(sp, int(g["test_num"]))
    return g, sp, x0, np.repeat(x0[:, None, :], sp.N + 1, 1), np.zeros((x0.shape[0], sp.N, 3))


def _oracle_soft_solve(sp, P, Zl_default):
    def solve(x0, xg, ug, w=None):
        w = w or {}
        Zl = w.get("Zl", np.tile(Zl_default, (x0.shape[0], 1)))
        x, u, r, h = oracle.mpc_soft_solve_batch(sp, x0, xg, ug, P, MEAN, STD, MARGIN, Zl, W=w.get("W"),
                                                 We=w.get("We"), rti=True)
        return dict(status=r["status"], x=x, u=u, qp_iter=r["qp_iter"])
    return solve


@pytest.mark.parametrize("kind", ["hard", "soft", "receding"])
def test_mpc_drivers_reproduce_the_reference_simulate(kind):
    """tests/golden/mpc_drivers.npz: the reference's own simulate(p) of hard_terminal_constraints/,
    soft_traj_constraints/ and receiding_hard_constraints/3dof_sym.py (AST-extracted, run on the oracle,
    tests/golden/make_mpc_golden.py).  vboc_amd.safempc.simulate_batch on the same oracle - all initial states at once
    - reproduces every problem's stop step and every control applied to the plant, bit for bit."""
    from vboc_amd.safempc import receding_weights, simulate_batch, soft_traj_weights
    g, sp, x0, xg, ug = _fixture()
    P = _net()
    if kind == "hard":
        solve, weights = _oracle_solve(sp, P, True), None
    else:
        solve = _oracle_soft_solve(sp, P, soft_traj_weights(sp.N) if kind == "soft" else np.zeros(sp.N + 1))
        weights = receding_weights(P, MEAN, STD, MARGIN, sp.N) if kind == "receding" else None
    log = {}
    res, simX, _ = simulate_batch(solve, _oracle_rk4(sp), sp, x0, xg, ug, tot_steps=int(g["tot_steps"]),
                                  weights=weights, log=log)
    np.testing.assert_array_equal(res, g[f"{kind}_res"])
    A = g[f"{kind}_applied"]
    np.testing.assert_array_equal(simX[:, :A.shape[1]], np.where(np.isnan(A[..., :6]), simX[:, :A.shape[1]], A[..., :6]))
    np.testing.assert_array_equal(log["u"], A[..., 6:])


# ------------------------------------------------------------------------------------------------
# GPU: vboc_mpc_soft_solve_batch (ft.h, SoftTraj) against the oracle
# ------------------------------------------------------------------------------------------------
def _gpu_soft(sp, P, x0, xg, ug, Zl, W=None, We=None, rti=True):
    import torch
    from vboc_amd import lib
    s = lib.Solver(3, sp.N)
    s.set_option("levenberg_marquardt", sp.lm)
    s.set_option("nlp_solver_tol_stat", 1e-6)
    s.set_option("qp_solver_tol_stat", 1e-8)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device="cuda:0")
    B = x0.shape[0]
    soft = dict(margin=MARGIN, Zl=T(np.broadcast_to(Zl, (B, sp.N + 1))),
                W=T(W) if W is not None else None, We=T(We) if We is not None else None)
    out = s.mpc_solve_device(sp, T(x0), T(xg), T(ug), [T(p) for p in P], MEAN, STD, rti=rti, soft=soft)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["soft_traj", "weighted"])
def test_gpu_soft_rti_matches_oracle(kind):
    """OCPtriplependulumSoftTraj's SQP_RTI solve on 128 states: with the soft_traj driver's weights (Zl = 1e6 at N),
    and with every stage penalised and per-problem stage weights (the receding driver's kind of call).  Every problem
    classified as the closed-loop step pairs: equal status, u_0 / x to STEP_TOL when both QPs converged, QP-cap pairs
    reported; the margin-scaled row at the results' x_N as the oracle's."""
    P = _net()
    sp, x0, xg, ug = _states(128, seed=5)
    W = We = None
    Zl = _soft_weights(sp.N, "soft_traj" if kind == "soft_traj" else "all")
    if kind == "weighted":
        rng = np.random.default_rng(3)
        q0 = 1e-2 + 10 ** rng.uniform(0, 2, 128)
        W = np.tile(np.r_[1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4, 1e-4], (128, 1))
        W[:, 0] = q0
        We = W[:, :6].copy()
    g = _gpu_soft(sp, P, x0, xg, ug, Zl, W, We)
    x, u, r, h = oracle.mpc_soft_solve_batch(sp, x0, xg, ug, P, MEAN, STD, MARGIN, Zl, W=W, We=We, rti=True)
    pairs = []
    _lockstep_solve(lambda *a: dict(g), lambda *a: dict(status=r["status"], x=x, u=u, qp_iter=r["qp_iter"]),
                    pairs)(x0, xg, ug)
    _classify_closed_loop(pairs)
    ok = (g["status"] == 0) & (r["status"] == 0) & (g["qp_iter"] < 100) & (r["qp_iter"] < 100)
    assert ok.mean() >= 0.9 and np.abs(g["h"][ok] - h[ok]).max() < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["hard", "soft", "receding"])
def test_gpu_mpc_drivers_lockstep(kind):
    """The three Safe-MPC drivers' closed loops (tests/golden/mpc_drivers.npz initial states, 100 steps) on the GPU
    drop-in classes, every step's OCP also solved by the oracle from the same inputs and classified (no 'value');
    the problems whose every step pair is 'same' and whose GPU loop ended at the fixture's step are counted and
    printed beside the fixture comparison of their applied controls."""
    from vboc_amd import lib
    from vboc_amd.safempc import (OCPtriplependulumHardTerm, OCPtriplependulumSoftTraj, receding_weights,
                                  simulate_batch, soft_traj_weights)
    g, sp, x0, xg, ug = _fixture()
    P = _net()
    rk4 = lambda X, U: lib.rk4_host(3, sp.time_step, X, U)
    if kind == "hard":
        ocp = OCPtriplependulumHardTerm("SQP_RTI", sp.time_step, sp.tot_time, P, MEAN, STD)
        gs, os_, weights = _gpu_hard_solve(ocp), _oracle_solve_q(sp, P, True), None
    else:
        ocp = OCPtriplependulumSoftTraj("SQP_RTI", sp.time_step, sp.tot_time, P, MEAN, STD, MARGIN)
        if kind == "soft":   # the soft_traj driver's main block (:102-105)
            for i in range(1, sp.N):
                ocp.ocp_solver.cost_set(i, "Zl", 0 * np.ones((1,)))
            ocp.ocp_solver.cost_set(sp.N, "Zl", 1e6 * np.ones((1,)))
        gs = lambda x0_, xg_, ug_, w=None: ocp.solve_batch(x0_, xg_, ug_, w)
        os_ = _oracle_soft_solve(sp, P, soft_traj_weights(sp.N) if kind == "soft" else np.zeros(sp.N + 1))
        weights = receding_weights(P, MEAN, STD, MARGIN, sp.N) if kind == "receding" else None
    pairs, log = [], {}
    res, _, _ = simulate_batch(_lockstep_solve(gs, os_, pairs), rk4, sp, x0, xg, ug, tot_steps=int(g["tot_steps"]),
                               weights=weights, log=log)
    _classify_closed_loop(pairs)
    dev = np.nanmax(np.abs(log["u"] - g[f"{kind}_applied"][..., 6:]), axis=(1, 2))
    print(f"{kind}: stop steps as the fixture {(res == g[kind + '_res']).sum()}/{res.size}; applied controls vs the "
          f"fixture: median max |du| {np.median(dev):.2e}, {(dev < 1e-6).sum()} problems within 1e-6")
