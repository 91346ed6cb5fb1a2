"""Independent NLP check (test helper): the same discretised OCP solved by scipy SLSQP.

Decision vector (s, u_0..u_{N-1}, x_1..x_N); equality constraints x_{k+1} = RK4(x_k, u_k) and
v_N = v_fin; boxes as in OCP_solve (VBOC/triplependulum_class_vboc.py:155-191).  Used to show that
the oracle's SQP lands on a KKT point of the reference problem, independently of its own QP.
"""
import numpy as np
from scipy.optimize import minimize

import oracle


def slsqp(nq, b, i, maxiter=500, hc=None, start=None):
    """start: optional (x [N+1, >= 2nq], u [N, nq]) initial point instead of the batch's guess.  hc: optional (x_c, y_c, lh, uh) - the Cartesian keep-out circle lh <= |tip(x_k) - c|^2 <= uh on
    stages 1..N-1 (VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160), written here
    independently of the oracle as SLSQP inequality constraints with their own Jacobian."""
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
    xg, ug = (b["x_guess"][i], b["u_guess"][i]) if start is None else start
    z0 = np.r_[d @ xg[0, nq:2 * nq], ug[:N].ravel(), xg[1:N + 1, :nx].ravel()]
    lo = [bb[0] if bb[0] is not None else -1e9 for bb in bounds]
    hi = [bb[1] if bb[1] is not None else 1e9 for bb in bounds]
    z0 = np.clip(z0, lo, hi)
    cons = [dict(type="eq", fun=eq, jac=eqjac)]
    if hc is not None:
        xc, yc, lh, uh = hc
        L = np.full(nq, 0.8)

        def tip(X):
            return (np.sin(X[1:N, :nq]) @ L - xc, np.cos(X[1:N, :nq]) @ L - yc)

        def ineq(z):
            _, X = unpack(z)
            dx, dy = tip(X)
            hv = dx * dx + dy * dy
            return np.r_[hv - lh, uh - hv]

        def ineqjac(z):
            _, X = unpack(z)
            dx, dy = tip(X)
            J = np.zeros((2 * (N - 1), nv))
            for k in range(1, N):
                g = 2 * dx[k - 1] * L * np.cos(X[k, :nq]) - 2 * dy[k - 1] * L * np.sin(X[k, :nq])
                c0 = 1 + N * nq + (k - 1) * nx
                J[k - 1, c0:c0 + nq] = g
                J[N - 1 + k - 1, c0:c0 + nq] = -g
            return J
        cons.append(dict(type="ineq", fun=ineq, jac=ineqjac))
    r = minimize(lambda z: cs * z[0], z0, jac=lambda z: np.r_[cs, np.zeros(nv - 1)], bounds=bounds,
                 constraints=cons, method="SLSQP", options=dict(maxiter=maxiter, ftol=1e-10))
    if hc is not None:
        _, X = unpack(r.x)
        return r.fun, bool(r.success), float(np.abs(eq(r.x)).max()), float(ineq(r.x)[:N - 1].min())
    return r.fun, bool(r.success), float(np.abs(eq(r.x)).max())


def slsqp_free_time(b, i, maxiter=500, start=None):
    """The free-time pendulum OCP (OCPpendulum.OCP_solve, VBOC/pendulum_class_vboc.py:107-130) as one
    NLP for scipy SLSQP: z = (x_0..x_N, u_0..u_{N-1}) with x = [theta, dtheta, dt]; equalities
    x_{k+1} = Phi(x_k, u_k) (RK4 with h = dt, oracle.ft_rk4_sens), stage-0 and terminal components with
    lb == ub; boxes; cost p[0] dtheta_0 + p[1] sum_{k<N} dt_k.  Returns (cost, success, max eq viol,
    x_0).  start: optional (x [N+1, 3], u [N, 1]) initial point (default: the batch's guess; SLSQP does
    not find a feasible point from the straight-line guess of these minimum-time problems)."""
    N, nx, nu = int(b["N"][i]), 3, 1
    nv = (N + 1) * nx + N * nu
    p = b["p"][i]
    c = np.zeros(nv)
    c[1] = p[0]
    for k in range(N):
        c[k * nx + 2] += p[1]
    fix0 = [j for j in range(nx) if b["lbx0"][i, j] == b["ubx0"][i, j]]
    fixN = [j for j in range(nx) if b["lbxe"][i, j] == b["ubxe"][i, j]]
    X = lambda z: z[:(N + 1) * nx].reshape(N + 1, nx)
    U = lambda z: z[(N + 1) * nx:].reshape(N, nu)

    def eq(z):
        x, u = X(z), U(z)
        r = [x[k + 1] - oracle.ft_rk4_sens(1, x[k], u[k])[0] for k in range(N)]
        r.append(np.array([x[0, j] - b["lbx0"][i, j] for j in fix0] + [x[N, j] - b["lbxe"][i, j] for j in fixN]))
        return np.concatenate(r)

    def eqjac(z):
        x, u = X(z), U(z)
        J = np.zeros((N * nx + len(fix0) + len(fixN), nv))
        for k in range(N):
            _, A, B = oracle.ft_rk4_sens(1, x[k], u[k])
            r = slice(k * nx, (k + 1) * nx)
            J[r, k * nx:(k + 1) * nx] = -A
            J[r, (k + 1) * nx:(k + 2) * nx] += np.eye(nx)
            J[r, (N + 1) * nx + k * nu:(N + 1) * nx + (k + 1) * nu] = -B
        row = N * nx
        for j in fix0:
            J[row, j] = 1.0
            row += 1
        for j in fixN:
            J[row, N * nx + j] = 1.0
            row += 1
        return J

    bounds = []
    for k in range(N + 1):
        lo, hi = (b["lbx0"][i], b["ubx0"][i]) if k == 0 else ((b["lbxe"][i], b["ubxe"][i]) if k == N else
                                                                (b["lbx"][i], b["ubx"][i]))
        bounds += [(lo[j], hi[j]) for j in range(nx)]
    bounds += [(b["lbu"][i, 0], b["ubu"][i, 0])] * N
    xs, us = start if start is not None else (b["x_guess"][i, :N + 1], b["u_guess"][i, :N])
    z0 = np.r_[np.ravel(xs), np.ravel(us)]
    z0 = np.clip(z0, [bb[0] for bb in bounds], [bb[1] for bb in bounds])
    r = minimize(lambda z: c @ z, z0, jac=lambda z: c, bounds=bounds, constraints=[dict(type="eq", fun=eq, jac=eqjac)],
                 method="SLSQP", options=dict(maxiter=maxiter, ftol=1e-12))
    return r.fun, bool(r.success), float(np.abs(eq(r.x)).max()), X(r.x)[0]


def slsqp_mpc(spec, x0, start, params=None, mean=0.0, std=1.0, maxiter=300):
    """The Safe-MPC OCP (VBOC/Safe MPC/triplependulum_class_vboc.py:91-240, vboc_amd.safempc.MpcSpec) as an
    independent NLP for scipy SLSQP: decision vector (u_0..u_{N-1}, x_1..x_N), x_0 fixed, equality constraints
    x_{k+1} = RK4(x_k, u_k; time_step) of the 6-state model (golden-pinned oracle.rk4 / rk4_sens), boxes, and
    with params the terminal row h(x_N) = NN(x_N) - max(|x_N[2:]|, 1e-3) >= 0 (vboc_amd.safempc.nn_row, its
    gradient by central differences).  Objective: the LINEAR_LS cost with stage costs scaled by spec.cost_scale.
    start = (x [N+1, 6], u [N, 3]).  Returns (x, u, cost, scipy result)."""
    from vboc_amd.safempc import nn_row
    N, h, nx, nu = spec.N, spec.time_step, 6, 3
    x0 = np.asarray(x0, dtype=np.float64)
    W, We, yr, yre, cs = spec.W, spec.W_e, spec.yref, spec.yref_e, spec.cost_scale
    nv = N * nu + N * nx

    def unpack(z):
        return z[:N * nu].reshape(N, nu), np.vstack([x0, z[N * nu:].reshape(N, nx)])

    def cost(z):
        U, X = unpack(z)
        c = 0.0
        for k in range(N):
            d = np.r_[X[k], U[k]] - yr
            c += cs * 0.5 * float(d @ (W * d))
        d = X[N] - yre
        return c + 0.5 * float(d @ (We * d))

    def grad(z):
        U, X = unpack(z)
        g = np.zeros(nv)
        for k in range(N):
            d = np.r_[X[k], U[k]] - yr
            g[k * nu:(k + 1) * nu] = cs * W[nx:] * d[nx:]
            if k > 0:
                g[N * nu + (k - 1) * nx:N * nu + k * nx] += cs * W[:nx] * d[:nx]
        g[N * nu + (N - 1) * nx:] += We * (X[N] - yre)
        return g

    def eq(z):
        U, X = unpack(z)
        return np.concatenate([X[k + 1] - oracle.rk4(3, h, X[k], U[k]) for k in range(N)])

    def eqjac(z):
        U, X = unpack(z)
        J = np.zeros((N * nx, nv))
        for k in range(N):
            _, A, B = oracle.rk4_sens(3, h, X[k], U[k])
            r = slice(k * nx, (k + 1) * nx)
            J[r, k * nu:(k + 1) * nu] = -B
            if k > 0:
                J[r, N * nu + (k - 1) * nx:N * nu + k * nx] = -A
            J[r, N * nu + k * nx:N * nu + (k + 1) * nx] += np.eye(nx)
        return J

    cons = [dict(type="eq", fun=eq, jac=eqjac)]
    if params is not None:
        def row(z):
            return np.array([nn_row(params, mean, std, unpack(z)[1][N])])

        def rowjac(z):
            xN = unpack(z)[1][N]
            J = np.zeros((1, nv))
            for j in range(nx):
                e = np.zeros(nx)
                e[j] = 1e-6
                J[0, N * nu + (N - 1) * nx + j] = (nn_row(params, mean, std, xN + e) -
                                                   nn_row(params, mean, std, xN - e)) / 2e-6
            return J
        cons.append(dict(type="ineq", fun=row, jac=rowjac))
    bounds = [(spec.umin[a], spec.umax[a]) for _ in range(N) for a in range(nu)]
    bounds += [(spec.xmin[j], spec.xmax[j]) for _ in range(N) for j in range(nx)]
    xs, us = start
    z0 = np.r_[np.asarray(us, dtype=np.float64).ravel(), np.asarray(xs, dtype=np.float64)[1:].ravel()]
    r = minimize(cost, z0, jac=grad, bounds=bounds, constraints=cons, method="SLSQP",
                 options=dict(maxiter=maxiter, ftol=1e-14))
    U, X = unpack(r.x)
    return X, U, cost(r.x), r


def slsqp_mpc_soft(spec, x0, start, params, mean, std, margin, Zl, zl=None, W=None, We=None, maxiter=500):
    """OCPtriplependulumSoftTraj (VBOC/Safe MPC/triplependulum_class_vboc.py:242-304) as an independent NLP for scipy
    SLSQP: decision vector (u_0..u_{N-1}, x_1..x_N, s_0..s_N) with the slacks explicit, RK4 defects, boxes, the
    margin-scaled row h(x_k) = NN(x_k) (100 - margin) / 100 - vn(x_k) on every stage softened as h(x_k) + s_k >= 0,
    s_k >= 0, and the slack cost sum_k zl_k s_k + Zl_k s_k^2 / 2 (zu = Zu = 0: the upper side h <= 1e6 is never active
    and left out).  start = (x [N+1, 6], u [N, 3], s [N+1] or None).  Returns (x, u, s, cost, scipy result)."""
    from vboc_amd.safempc import nn_row
    N, h, nx, nu = spec.N, spec.time_step, 6, 3
    x0 = np.asarray(x0, dtype=np.float64)
    W = spec.W if W is None else np.asarray(W, float)
    We = spec.W_e if We is None else np.asarray(We, float)
    Zl = np.broadcast_to(np.asarray(Zl, float), (N + 1,))
    zl = np.zeros(N + 1) if zl is None else np.broadcast_to(np.asarray(zl, float), (N + 1,))
    yr, yre, cs = spec.yref, spec.yref_e, spec.cost_scale
    nq = N * nu + N * nx
    nv = nq + N + 1
    row = lambda x: nn_row(params, mean, std, x, safety_margin=margin)

    def unpack(z):
        return z[:N * nu].reshape(N, nu), np.vstack([x0, z[N * nu:nq].reshape(N, nx)]), z[nq:]

    def cost(z):
        U, X, S = unpack(z)
        c = 0.0
        for k in range(N):
            d = np.r_[X[k], U[k]] - yr
            c += cs * 0.5 * float(d @ (W * d))
        d = X[N] - yre
        return c + 0.5 * float(d @ (We * d)) + float(zl @ S) + 0.5 * float(S @ (Zl * S))

    def grad(z):
        U, X, S = unpack(z)
        g = np.zeros(nv)
        for k in range(N):
            d = np.r_[X[k], U[k]] - yr
            g[k * nu:(k + 1) * nu] = cs * W[nx:] * d[nx:]
            if k > 0:
                g[N * nu + (k - 1) * nx:N * nu + k * nx] += cs * W[:nx] * d[:nx]
        g[N * nu + (N - 1) * nx:nq] += We * (X[N] - yre)
        g[nq:] = zl + Zl * S
        return g

    def eq(z):
        U, X, _ = unpack(z)
        return np.concatenate([X[k + 1] - oracle.rk4(3, h, X[k], U[k]) for k in range(N)])

    def eqjac(z):
        U, X, _ = unpack(z)
        J = np.zeros((N * nx, nv))
        for k in range(N):
            _, A, B = oracle.rk4_sens(3, h, X[k], U[k])
            r = slice(k * nx, (k + 1) * nx)
            J[r, k * nu:(k + 1) * nu] = -B
            if k > 0:
                J[r, N * nu + (k - 1) * nx:N * nu + k * nx] = -A
            J[r, N * nu + k * nx:N * nu + (k + 1) * nx] += np.eye(nx)
        return J

    def ineq(z):
        _, X, S = unpack(z)
        return np.array([row(X[k]) + S[k] for k in range(N + 1)])

    def ineqjac(z):
        _, X, _ = unpack(z)
        J = np.zeros((N + 1, nv))
        for k in range(N + 1):
            J[k, nq + k] = 1.0
            if k == 0:
                continue                      # x_0 fixed
            for j in range(nx):
                e = np.zeros(nx)
                e[j] = 1e-6
                J[k, N * nu + (k - 1) * nx + j] = (row(X[k] + e) - row(X[k] - e)) / 2e-6
        return J

    bounds = [(spec.umin[a], spec.umax[a]) for _ in range(N) for a in range(nu)]
    bounds += [(spec.xmin[j], spec.xmax[j]) for _ in range(N) for j in range(nx)]
    bounds += [(0.0, None)] * (N + 1)
    xs, us = start[0], start[1]
    s0 = start[2] if len(start) > 2 and start[2] is not None else np.array(
        [max(0.0, -row(np.asarray(xs, float)[k])) for k in range(N + 1)])
    z0 = np.r_[np.asarray(us, float).ravel(), np.asarray(xs, float)[1:].ravel(), np.asarray(s0, float)]
    r = minimize(cost, z0, jac=grad, bounds=bounds,
                 constraints=[dict(type="eq", fun=eq, jac=eqjac), dict(type="ineq", fun=ineq, jac=ineqjac)],
                 method="SLSQP", options=dict(maxiter=maxiter, ftol=1e-14))
    U, X, S = unpack(r.x)
    return X, U, S, cost(r.x), r
