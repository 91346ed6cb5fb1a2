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
    x, u, r, h = oracle.mpc_solve_batch(sp, x0, xg, ug, P, mean=MEAN, std=STD)
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
