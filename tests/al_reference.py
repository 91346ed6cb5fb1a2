"""Independent pin of AL's labels (test helper, never imported by the product path).

The label of AL's compute_problem (AL/triplependulum_class_al.py:148-169) is the status of ONE SQP_RTI iteration:
the QP linearised at the reset point (x_0 = (q0, v0) fixed, every other stage's x = (q0, 0), u = 0) either has a
solution (status 0 -> 1) or not (status 4 -> 0).  The QP is convex (a positive semi-definite Gauss-Newton Hessian),
so it has a solution exactly when its constraints are feasible - a linear program that does not involve the solver
under test at all: scipy's HiGHS decides it here from the linearisation rebuilt with the golden-pinned RK4
sensitivities (oracle.rk4_sens, tests/test_golden_dynamics.py)."""
import numpy as np
import scipy.sparse as sp
from scipy.optimize import linprog


def guesses(spec, x0, x_guess=None):
    """The stage guesses of the RTI point [N+1, 6]: compute_problem's (q0, 0) (x0 at stage 0, which is fixed), or
    compute_problem_nnguess's network trajectory x_guess."""
    xg = np.tile(np.r_[x0[:3], np.zeros(3)], (spec.N + 1, 1)) if x_guess is None else np.array(x_guess, dtype=float)
    xg[0] = x0
    return xg


def linearisation(spec, x0, x_guess=None):
    """(A_k, B_k, b_k) of the SQP_RTI point: stage k at (x_k, 0) with the stage guesses x_k (`guesses`);
    b_k = RK4(x_k, u_k) - x_{k+1}."""
    import oracle
    xg = guesses(spec, x0, x_guess)
    out = []
    for k in range(spec.N):
        x1, A, B = oracle.rk4_sens(3, spec.time_step, xg[k], np.zeros(3))
        out.append((A, B, x1 - xg[k + 1]))
    return out


def lp_feasible(spec, x0, x_guess=None):
    """True if the linearised QP of compute_problem(x0) (or compute_problem_nnguess with the stage guesses x_guess) has
    a feasible point (HiGHS on the zero-objective LP over du_0..du_{N-1}, dx_1..dx_N: the linearised dynamics, the path
    boxes, the terminal box with its fixed velocities)."""
    N = spec.N
    xgs = guesses(spec, x0, x_guess)
    nvar = 3 * N + 6 * N
    iu = lambda k: 3 * k
    ix = lambda k: 3 * N + 6 * (k - 1)
    rows, cols, vals, beq = [], [], [], []
    r = 0
    for k, (A, B, b) in enumerate(linearisation(spec, x0, x_guess)):
        for i in range(6):       # dx_{k+1} - A_k dx_k - B_k du_k = b_k  (dx_0 = 0: x_0 is fixed)
            rows.append(r); cols.append(ix(k + 1) + i); vals.append(1.0)
            if k > 0:
                for q in range(6):
                    rows.append(r); cols.append(ix(k) + q); vals.append(-A[i, q])
            for a in range(3):
                rows.append(r); cols.append(iu(k) + a); vals.append(-B[i, a])
            beq.append(b[i])
            r += 1
    Aeq = sp.csr_matrix((vals, (rows, cols)), shape=(r, nvar))
    lo, hi = np.empty(nvar), np.empty(nvar)
    for k in range(N):
        lo[iu(k):iu(k) + 3], hi[iu(k):iu(k) + 3] = spec.umin, spec.umax
    for k in range(1, N + 1):
        xl, xh = (spec.xmin_e, spec.xmax_e) if k == N else (spec.xmin, spec.xmax)
        lo[ix(k):ix(k) + 6], hi[ix(k):ix(k) + 6] = xl - xgs[k], xh - xgs[k]
    res = linprog(np.zeros(nvar), A_eq=Aeq, b_eq=np.array(beq), bounds=list(zip(lo, hi)), method="highs")
    assert res.status in (0, 2), res.message
    return res.status == 0


def step_violation(spec, x0, x, u, x_guess=None):
    """Largest violation, by the returned step (x [N+1, 6], u [N, 3]), of the linearised QP's constraints: the
    linearised dynamics, x_0, the boxes, the terminal velocities."""
    xg = guesses(spec, x0, x_guess)
    v = float(np.abs(x[0] - x0).max())
    for k, (A, B, b) in enumerate(linearisation(spec, x0, x_guess)):
        v = max(v, float(np.abs(x[k + 1] - xg[k + 1] - (A @ (x[k] - xg[k]) + B @ u[k] + b)).max()))
    v = max(v, float(np.max(np.r_[spec.xmin - x[1:-1].min(0), x[1:-1].max(0) - spec.xmax])))
    v = max(v, float(np.max(np.r_[spec.umin - u.min(0), u.max(0) - spec.umax])))
    v = max(v, float(np.max(np.r_[spec.xmin_e - x[-1], x[-1] - spec.xmax_e])))
    return v
