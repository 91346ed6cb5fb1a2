"""Independent NLP check (test helper): the same discretised OCP solved by scipy SLSQP.

Decision vector (s, u_0..u_{N-1}, x_1..x_N); equality constraints x_{k+1} = RK4(x_k, u_k) and
v_N = v_fin; boxes as in OCP_solve (VBOC/triplependulum_class_vboc.py:155-191).  Used to show that
the oracle's SQP lands on a KKT point of the reference problem, independently of its own QP.
"""
import numpy as np
from scipy.optimize import minimize

import oracle


def slsqp(nq, b, i, maxiter=500):
    N = int(b["N"][i])
    h = b["lbx"][i, 2 * nq]
    p = b["p"][i]
    d = p[:nq] / np.linalg.norm(p[:nq]) if nq > 1 else np.ones(1)
    cs = float(p[:nq] @ d)
    q0 = b["lbx0"][i, :nq]
    nx = 2 * nq
    lo_s, hi_s = -np.inf, np.inf
    for j in range(nq):
        lo, hi = b["lbx0"][i, nq + j], b["ubx0"][i, nq + j]
        if d[j] > 0:
            lo_s, hi_s = max(lo_s, lo / d[j]), min(hi_s, hi / d[j])
        elif d[j] < 0:
            lo_s, hi_s = max(lo_s, hi / d[j]), min(hi_s, lo / d[j])
    nv = 1 + N * nq + N * nx

    def unpack(z):
        U = z[1:1 + N * nq].reshape(N, nq)
        X = z[1 + N * nq:].reshape(N, nx)
        return U, np.vstack([np.r_[q0, z[0] * d], X])

    def eq(z):
        U, X = unpack(z)
        r = [X[k + 1] - oracle.rk4(nq, h, X[k], U[k]) for k in range(N)]
        r.append(X[N, nq:] - b["lbxe"][i, nq:2 * nq])
        return np.concatenate(r)

    def eqjac(z):
        U, X = unpack(z)
        J = np.zeros((N * nx + nq, nv))
        for k in range(N):
            _, A, B = oracle.rk4_sens(nq, h, X[k], U[k])
            r = slice(k * nx, (k + 1) * nx)
            J[r, 1 + k * nq:1 + (k + 1) * nq] = -B
            if k == 0:
                J[r, 0] = -(A[:, nq:] @ d)
            else:
                J[r, 1 + N * nq + (k - 1) * nx:1 + N * nq + k * nx] = -A
            J[r, 1 + N * nq + k * nx:1 + N * nq + (k + 1) * nx] += np.eye(nx)
        J[N * nx:, 1 + N * nq + (N - 1) * nx + nq:1 + N * nq + N * nx] = np.eye(nq)
        return J

    bounds = [(lo_s, hi_s)] + [(b["lbu"][i, a], b["ubu"][i, a]) for _ in range(N) for a in range(nq)]
    for k in range(1, N + 1):
        for j in range(nx):
            if k < N:
                bounds.append((b["lbx"][i, j], b["ubx"][i, j]))
            else:
                bounds.append((b["lbxe"][i, j], b["ubxe"][i, j]) if j < nq else (None, None))
    xg, ug = b["x_guess"][i], b["u_guess"][i]
    z0 = np.r_[d @ xg[0, nq:2 * nq], ug[:N].ravel(), xg[1:N + 1, :nx].ravel()]
    lo = [bb[0] if bb[0] is not None else -1e9 for bb in bounds]
    hi = [bb[1] if bb[1] is not None else 1e9 for bb in bounds]
    z0 = np.clip(z0, lo, hi)
    r = minimize(lambda z: cs * z[0], z0, jac=lambda z: np.r_[cs, np.zeros(nv - 1)], bounds=bounds,
                 constraints=[dict(type="eq", fun=eq, jac=eqjac)], method="SLSQP",
                 options=dict(maxiter=maxiter, ftol=1e-10))
    return r.fun, bool(r.success), float(np.abs(eq(r.x)).max())
