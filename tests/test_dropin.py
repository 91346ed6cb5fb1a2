"""The drop-in OCP classes (vboc_amd.ocp) on CPU: with the oracle injected as their solver
(vboc_amd.ocp.use_backend, test-only), OCP_solve / the ocp_solver API must hand the solver exactly the
problem the reference's ACADOS calls describe (VBOC/triplependulum_class_vboc.py:155-191), and reject
structures the boundary solver does not implement loudly."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from oracle_backend import OracleOcpBackend, _oracle_solve  # noqa: E402


@pytest.fixture
def oracle_dropin():
    from vboc_amd import ocp
    ocp.use_backend(OracleOcpBackend())
    yield ocp
    ocp.use_backend(None)


@pytest.mark.parametrize("nq,cls", [(3, "OCPtriplependulumINIT"), (2, "OCPdoublependulumINIT")])
def test_ocp_solve_is_the_batched_problem(oracle_dropin, nq, cls):
    from vboc_amd.ics import data_generation_ics
    b = data_generation_ics(nq, np.arange(4))
    ref = _oracle_solve(nq, b)
    ocp = getattr(oracle_dropin, cls)()
    N = ocp.N
    for i in range(4):
        st = ocp.OCP_solve(b["x_guess"][i, :N], b["u_guess"][i, :N], b["p"][i], b["lbx"][i], b["ubx"][i],
                           b["lbu"][i], b["ubu"][i], b["lbx0"][i], b["ubx0"][i], b["lbxe"][i], b["ubxe"][i])
        assert st == ref["status"][i]
        assert ocp.ocp_solver.get_cost() == ref["cost"][i]
        np.testing.assert_array_equal(ocp.ocp_solver.get(0, "x"), ref["x"][i, 0])
        np.testing.assert_array_equal(ocp.ocp_solver.get(N - 1, "u"), ref["u"][i, N - 1])
        assert ocp.ocp_solver.get_stats("sqp_iter") == ref["sqp_iter"][i]


def test_pendulum_solver_api(oracle_dropin):
    """pendulum_testdata.py:29-47: x guesses and p only (u from reset, u bounds the class defaults)."""
    from vboc_amd.ics import heldout_ics
    b = heldout_ics(1, np.arange(3))
    ref = _oracle_solve(1, b)
    ocp = oracle_dropin.OCPpendulum()
    N, S = ocp.N, ocp.ocp_solver
    for i in range(3):
        S.reset()
        for k in range(N):
            S.set(k, "x", b["x_guess"][i, k])
            S.set(k, "p", b["p"][i])
            S.constraints_set(k, "lbx", b["lbx"][i])
            S.constraints_set(k, "ubx", b["ubx"][i])
        S.constraints_set(0, "lbx", b["lbx0"][i])
        S.constraints_set(0, "ubx", b["ubx0"][i])
        S.constraints_set(N, "lbx", b["lbxe"][i])
        S.constraints_set(N, "ubx", b["ubxe"][i])
        S.set(N, "x", b["x_guess"][i, N])
        S.set(N, "p", b["p"][i])
        assert S.solve() == ref["status"][i]
        np.testing.assert_array_equal(S.get(0, "x"), ref["x"][i, 0])


def test_unsupported_structures_raise(oracle_dropin):
    from vboc_amd.ics import data_generation_ics
    ocp = oracle_dropin.OCPtriplependulumINIT()
    b = data_generation_ics(3, np.arange(1))
    N, S = ocp.N, ocp.ocp_solver
    args = (b["x_guess"][0, :N], b["u_guess"][0, :N], b["p"][0], b["lbx"][0], b["ubx"][0], b["lbu"][0],
            b["ubu"][0], b["lbx0"][0], b["ubx0"][0], b["lbxe"][0], b["ubxe"][0])
    assert ocp.OCP_solve(*args) in (0, 1, 2, 3, 4)
    S.set(5, "p", b["p"][0] * 0.5)                        # stage-varying parameters
    with pytest.raises(NotImplementedError):
        S.solve()
    lb = b["lbx"][0].copy()
    lb[6] = 0.0                                           # free time step
    ocp.OCP_solve(*args)
    S.constraints_set(3, "lbx", lb)
    with pytest.raises(NotImplementedError):
        S.solve()
    with pytest.raises(NotImplementedError):
        S.set_new_time_steps(np.full(N, 0.5))
    S.set_new_time_steps(np.full(N, 1.0))
    ocp.OCP_solve(*args)
    for k in range(1, N):
        S.constraints_set(k, "lbx", lb)
    with pytest.raises(NotImplementedError):              # free time + general constraint C
        S.solve()
