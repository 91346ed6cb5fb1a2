"""Free-time OCP path (OCPpendulum.OCP_solve, VBOC/pendulum_class_vboc.py:107-130; the pendulum's VBOC
data generation VBOC/pendulum_vboc.py:52-205) on CPU: the oracle's free-time restatement
(oracle/vboc_oracle_ft.c) pinned to the reference's expressions and to an independent NLP solve, the
batched pendulum driver pinned to the reference's own loop, and the drop-in class's mapping."""
import json
import os
import sys

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from nlp_reference import slsqp_free_time  # noqa: E402
from oracle_backend import OracleBackend, OracleOcpBackend, _oracle_solve  # noqa: E402


@pytest.mark.parametrize("nq", [1, 2, 3])
def test_shooting_map_and_jacobian_match_golden(nq):
    """Phi(x, u) with dt a state and its full Jacobian (incl. d/d(dt)) against RK4 (h = 1) of the
    reference's f_expl and the forward sensitivities of its symbolic Jacobian (tests/golden/)."""
    g = np.load(os.path.join(HERE, "golden", f"dynamics_{nq}.npz"))
    nx = 2 * nq + 1
    for i in range(g["x"].shape[0]):
        x1, A, B = oracle.ft_rk4_sens(nq, g["x"][i], g["u"][i])
        np.testing.assert_allclose(x1, g["shoot_x1"][i], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(A, g["shoot_jac"][i][:, :nx], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(B, g["shoot_jac"][i][:, nx:], rtol=1e-10, atol=1e-12)


def _batch(ids, N_range=(20, 60)):
    from vboc_amd.ics import pendulum_free_time_ics
    return pendulum_free_time_ics(np.asarray(ids), N_range)


def test_oracle_free_time_solves_converge():
    b = _batch(np.arange(64))
    xo, uo, r = oracle.solve_batch(1, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], free_time=True)
    assert np.mean(r["status"] == 0) >= 0.95
    for i in np.where(r["status"] == 0)[0]:
        N = b["N"][i]
        x = xo[i, :N + 1]
        # the solution is a feasible free-time trajectory: one dt, dynamics, fixed ends, boxes
        assert np.ptp(x[:, 2]) < 1e-9 and 0.0 <= x[0, 2] <= 1e-2 + 1e-9
        for k in range(N):
            np.testing.assert_allclose(oracle.ft_rk4_sens(1, x[k], uo[i, k])[0], x[k + 1], atol=1e-6)
        assert abs(x[0, 0] - b["lbx0"][i, 0]) < 1e-12
        assert abs(x[N, 0] - b["lbxe"][i, 0]) < 1e-6 and abs(x[N, 1]) < 1e-6
        cost = b["p"][i, 0] * x[0, 1] + b["p"][i, 1] * x[:N, 2].sum()
        assert abs(cost - r["cost"][i]) < 1e-9


@pytest.mark.parametrize("idx", [0, 1, 2, 3])
def test_oracle_free_time_optimum_matches_slsqp(idx):
    b = _batch(np.arange(idx * 7, idx * 7 + 1), N_range=(15, 25))
    xo, uo, r = oracle.solve_batch(1, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], free_time=True)
    assert r["status"][0] == 0
    # SLSQP started AT the oracle's solution (it finds no feasible point from the straight-line guess
    # of these minimum-time problems, nor reliably from perturbed starts) must find no descent: the
    # oracle's point is a KKT point of the independently stated NLP, not an artefact of its own QP
    N = int(b["N"][0])
    xs, us = xo[0, :N + 1], uo[0, :N]
    fun, ok, viol, x0 = slsqp_free_time(b, 0, start=(xs, us))
    assert viol < 1e-7
    # SLSQP finds no better point (beyond 1e-5) and stays within the SQP tolerance (tol_stat 1e-3)
    assert fun > r["cost"][0] - 1e-5 and abs(fun - r["cost"][0]) < 1e-3, (fun, r["cost"][0])
    np.testing.assert_allclose(xo[0, 0], x0, atol=1e-3)


def test_pendulum_data_generation_matches_reference_loop():
    """The batched driver on the oracle reproduces X_save of the reference's own loop
    (VBOC/pendulum_vboc.py:52-205, AST-extracted, run on the drop-in OCPpendulum) bit for bit."""
    from vboc_amd.drivers import pendulum_data_generation
    fx = json.load(open(os.path.join(HERE, "golden", "driver_1.json")))
    X, stats = pendulum_data_generation(OracleBackend(1), fx["N_start"], fx["eps"])
    np.testing.assert_array_equal(X, np.array(fx["X_save"]))
    assert stats["solves"] >= 2


def test_dropin_pendulum_ocp_solve_is_the_free_time_problem():
    from vboc_amd import ocp as dropin
    b = _batch(np.arange(4), N_range=(50, 50))
    ref = _oracle_solve(1, b, free_time=True)
    dropin.use_backend(OracleOcpBackend())
    try:
        o = dropin.OCPpendulum()
        for i in range(4):
            q_init, q_fin = b["lbx0"][i, 0], b["lbxe"][i, 0]
            st = o.OCP_solve(b["x_guess"][i], b["u_guess"][i], b["p"][i, 0], b["lbx"][i], b["ubx"][i], q_init, q_fin)
            assert st == ref["status"][i]
            assert o.ocp_solver.get_cost() == ref["cost"][i]
            np.testing.assert_array_equal(o.ocp_solver.get(0, "x"), ref["x"][i, 0])
            np.testing.assert_array_equal(o.ocp_solver.get(o.N, "x"), ref["x"][i, o.N])
    finally:
        dropin.use_backend(None)


def test_pendulum_vboc_run_on_cpu(tmp_path):
    """The pendulum main block end to end on the oracle backend (CPU): data, fit, RMSE, artefacts."""
    import torch
    from vboc_amd.pipeline import pendulum_vboc_run
    r = pendulum_vboc_run(str(tmp_path), device="cpu", backend=OracleBackend(1), it_max=300)
    fx = json.load(open(os.path.join(HERE, "golden", "driver_1.json")))
    np.testing.assert_array_equal(r["X"], np.array(fx["X_save"]))
    assert r["fit"]["iterations"] <= 300 and np.isfinite(r["rmse"])
    np.testing.assert_array_equal(np.load(tmp_path / "data_1dof_vboc_10.npy"), r["X"])
    sd = torch.load(tmp_path / "model_1dof_vboc_10", weights_only=True)
    assert sd["linear_relu_stack.0.weight"].shape == (100, 2)
    assert torch.load(tmp_path / "mean_1dof_vboc_10", weights_only=True) == r["mean"]
