"""Oracle dynamics vs golden vectors computed from the reference's own f_expl expressions
(tests/golden/make_golden.py; VBOC/*_class_vboc.py f_expl)."""
import numpy as np
import pytest

import oracle

SYSTEMS = (1, 2, 3)


@pytest.fixture(scope="module", params=SYSTEMS)
def golden(request):
    nq = request.param
    return nq, np.load(f"{oracle.HERE}/../tests/golden/dynamics_{nq}.npz")


def test_rhs_and_jacobian(golden):
    nq, g = golden
    for i in range(g["x"].shape[0]):
        x, u = g["x"][i], g["u"][i]
        dt = x[2 * nq]
        acc, Jth, Jom, Ju = oracle.model(nq, x[:nq], x[nq:2 * nq], u)
        f = g["f"][i]
        # f_expl = dt * [dtheta; acc; 0]
        np.testing.assert_allclose(dt * acc, f[nq:2 * nq], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(dt * x[nq:2 * nq], f[:nq], rtol=1e-14)
        assert f[2 * nq] == 0.0
        J = g["jac"][i]
        np.testing.assert_allclose(dt * Jth, J[nq:2 * nq, :nq], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(dt * Jom, J[nq:2 * nq, nq:2 * nq], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(dt * Ju, J[nq:2 * nq, 2 * nq + 1:], rtol=1e-10, atol=1e-12)


def test_twin_rk4_step(golden):
    """SYM<sys>INIT integrator: ERK4, 4 stages, T = 1e-2 (triplependulum_class_vboc.py:235-239)."""
    nq, g = golden
    for i in range(g["x"].shape[0]):
        x1 = oracle.rk4(nq, float(g["rk4_T"]), g["x"][i, :2 * nq], g["u"][i])
        np.testing.assert_allclose(x1, g["rk4_x1"][i], rtol=1e-13, atol=1e-13)


def test_shooting_interval_equals_dt_scaled_rk4(golden):
    """One OCP shooting interval (RK4, h = 1 on dt*f with the dt state, tf/N = 1) equals RK4 with
    h = dt on the physics rhs - the exact dt elimination used by the solver."""
    nq, g = golden
    for i in range(g["x"].shape[0]):
        x = g["x"][i]
        x1 = oracle.rk4(nq, x[2 * nq], x[:2 * nq], g["u"][i])
        np.testing.assert_allclose(x1, g["shoot_x1"][i, :2 * nq], rtol=1e-13, atol=1e-13)
        assert g["shoot_x1"][i, 2 * nq] == x[2 * nq]


def test_rk4_sensitivities_match_finite_differences(golden):
    nq, g = golden
    x, u = g["x"][0, :2 * nq], g["u"][0]
    x1, A, B = oracle.rk4_sens(nq, 1e-2, x, u)
    np.testing.assert_allclose(x1, oracle.rk4(nq, 1e-2, x, u), rtol=0, atol=1e-15)
    eps = 1e-6
    for j in range(2 * nq):
        dx = np.zeros(2 * nq)
        dx[j] = eps
        fd = (oracle.rk4(nq, 1e-2, x + dx, u) - oracle.rk4(nq, 1e-2, x - dx, u)) / (2 * eps)
        np.testing.assert_allclose(A[:, j], fd, rtol=1e-6, atol=1e-8)
    for j in range(nq):
        du = np.zeros(nq)
        du[j] = eps
        fd = (oracle.rk4(nq, 1e-2, x, u + du) - oracle.rk4(nq, 1e-2, x, u - du)) / (2 * eps)
        np.testing.assert_allclose(B[:, j], fd, rtol=1e-6, atol=1e-8)
