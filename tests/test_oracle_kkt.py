"""Independent optimality pins of the oracle's optimum for the headline triple pendulum and the UR5 arm.

SURVEY.md section 7 step 1 asks for the CPU restatement to be validated "against an independent NLP solve
... against a solved OCP's KKT residuals".  Two checks, both outside the oracle's own code:

* KKT recomputed here: at the oracle's final iterate, with the multipliers it returns
  (oracle.solve_mult), the Lagrangian gradient of the reference NLP (VBOC/triplependulum_class_vboc.py:155-191:
  cost p'v_0 with v_0 = s d, dynamics x_{k+1} = RK4(x_k, u_k), boxes, terminal rest) is rebuilt stage by
  stage from the golden-pinned RK4 sensitivities, together with primal feasibility, dual feasibility and
  complementarity.  Its stationarity must be below the reference's tol_stat = 1e-3 (:137).
* scipy SLSQP on the same discretised NLP (tests/nlp_reference.py): started at the oracle's point it finds
  no lower cost (a local minimum, not only a KKT point), and started from the same guess as the oracle it
  lands on the same optimum on >= 5 triple and 5 UR5 problems (on two more triple ICs it converges to a
  different local minimum of this non-convex NLP; those keep the no-descent pin).  Problems: data-generation first solves, a verification-type problem (horizon N - f
  from x_sol[f], cost direction -v_f / |v_f|, VBOC/triplependulum_vboc.py:232-262) and a long-tail id of the
  GPU parity suite; horizons are the smallest at which SLSQP converges in seconds.

Two UR5 first solves (ids 1 and 3 at N 15) stop at a KKT point within tol_stat = 1e-3 (the reference's own
option, :137 of the class files) from which SLSQP, started there, still descends to a lower cost: a flat
valley where a 1e-3 gradient leaves room for a 0.08 cost change.  Those are pinned as KKT points (the
stopping rule ACADOS applies too), not as optima; DESIGN.md section 3 records it.
"""
from concurrent.futures import ProcessPoolExecutor

import numpy as np
import pytest

import oracle
from nlp_reference import slsqp
from vboc_amd.ics import data_generation_ics, ur5_ics

LONG_TAIL_ID = 988   # tests/test_gpu.py LONG_TAIL: a first solve that runs hundreds of SQP iterations at N = 100


def _sub(b, i):
    return {k: v[i:i + 1] for k, v in b.items()}


def _cat(parts):
    return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}


def verification_problem(nq, b, i, r, f):
    """The verification OCP of data_generation from x_sol[f] of solution r of problem i (:245-290):
    horizon N - f, positions fixed at x_sol[f], velocity box, cost direction -v_f / |v_f|, guess x_sol[f:]."""
    N = int(b["N"][i])
    Nt = N - f
    nx = 2 * nq
    x = r["x"]
    v = x[f, nq:nx]
    out = {k: np.array(b[k][i:i + 1]) for k in ("p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")}
    out["p"][0, :nq] = -v / np.linalg.norm(v)
    out["lbx0"][0, :nq] = x[f, :nq]
    out["ubx0"][0, :nq] = x[f, :nq]
    xg = np.zeros((1,) + b["x_guess"].shape[1:])
    ug = np.zeros((1,) + b["u_guess"].shape[1:])
    xg[0, :Nt + 1, :nx] = x[f:N + 1]
    xg[0, :Nt + 1, nx] = b["lbx"][i, nx]
    ug[0, :Nt] = r["u"][f:N]
    out.update(N=np.array([Nt], np.int32), x_guess=xg, u_guess=ug)
    return out


def kkt_residuals(nq, b, i, r):
    """(stationarity, primal infeasibility, min dual, complementarity) of the reference NLP at the oracle's
    final iterate r (oracle.solve_mult), recomputed from oracle.rk4_sens (pinned to the reference-expression
    goldens, tests/test_golden_dynamics.py)."""
    N = int(b["N"][i])
    nx, nu = 2 * nq, nq
    h = float(b["lbx"][i, nx])
    p = b["p"][i, :nq]
    d = p / np.linalg.norm(p) if nq > 1 else np.ones(1)
    cs = float(p @ d)
    X, U, pi, ll, lu = r["x"], r["u"], r["pi"], r["lam_l"], r["lam_u"]
    A, B, defect = [], [], 0.0
    for k in range(N):
        x1, Ak, Bk = oracle.rk4_sens(nq, h, X[k], U[k])
        A.append(Ak)
        B.append(Bk)
        defect = max(defect, float(np.abs(x1 - X[k + 1]).max()))
    g = [np.r_[cs - ll[0, 0] + lu[0, 0] + (A[0][:, nq:] @ d) @ pi[0],
               -ll[0, 1:1 + nu] + lu[0, 1:1 + nu] + B[0].T @ pi[0]]]
    for k in range(1, N):
        g.append(np.r_[-ll[k, :nx] + lu[k, :nx] + A[k].T @ pi[k] - pi[k - 1],
                       -ll[k, nx:] + lu[k, nx:] + B[k].T @ pi[k]])
    g.append(-ll[N, :nx] + lu[N, :nx] - pi[N - 1] + np.r_[np.zeros(nq), r["nu"]])
    stat = max(float(np.abs(v).max()) for v in g)
    # boxes of z_k (stage layout) and their values
    s_lo, s_hi = -np.inf, np.inf
    for j in range(nq):
        lo, hi = b["lbx0"][i, nq + j], b["ubx0"][i, nq + j]
        if d[j] > 0:
            s_lo, s_hi = max(s_lo, lo / d[j]), min(s_hi, hi / d[j])
        elif d[j] < 0:
            s_lo, s_hi = max(s_lo, hi / d[j]), min(s_hi, lo / d[j])
    infeas = max(defect, float(np.abs(X[N, nq:] - b["lbxe"][i, nq:nx]).max()),
                 float(np.abs(X[0, :nq] - b["lbx0"][i, :nq]).max()), float(np.abs(X[0, nq:] - r["s"] * d).max()))
    comp, dual = 0.0, 0.0
    for k in range(N + 1):
        if k == 0:
            z, lb, ub = np.r_[r["s"], U[0]], np.r_[s_lo, b["lbu"][i]], np.r_[s_hi, b["ubu"][i]]
        elif k < N:
            z, lb, ub = np.r_[X[k], U[k]], np.r_[b["lbx"][i, :nx], b["lbu"][i]], np.r_[b["ubx"][i, :nx], b["ubu"][i]]
        else:
            z, lb, ub = X[N, :nq], b["lbxe"][i, :nq], b["ubxe"][i, :nq]
        n = z.shape[0]
        infeas = max(infeas, float(np.max(np.r_[lb - z, z - ub])))
        comp = max(comp, float(np.max(np.abs(np.r_[ll[k, :n] * (z - lb), lu[k, :n] * (ub - z)]))))
        dual = min(dual, float(min(ll[k, :n].min(), lu[k, :n].min())))
    return stat, infeas, dual, comp


def _slsqp(args):
    nq, b, i, start = args
    return slsqp(nq, b, i, maxiter=3000, start=start)


def _problems():
    """(name, nq, batch, same_from_guess) of the pinned problems; every batch holds one problem.
    same_from_guess: SLSQP from the batch's own guess reaches the oracle's optimum; on the others it
    converges to a different local minimum (the NLP is non-convex), and only the no-descent check pins them."""
    out = []
    b3 = data_generation_ics(3, np.arange(8), N=20)
    for i in (0, 1, 3, 6):
        out.append((f"triple dg first solve id {i}, N 20", 3, _sub(b3, i), True))
    for i in (4, 5):
        out.append((f"triple dg first solve id {i}, N 20", 3, _sub(b3, i), False))
    r0 = oracle.solve_mult(3, b3, 0)
    out.append(("triple verification-type (x_sol[4] of id 0), N 16", 3, verification_problem(3, b3, 0, r0, 4), True))
    out.append((f"triple long-tail id {LONG_TAIL_ID}, N 20", 3, data_generation_ics(3, np.array([LONG_TAIL_ID]), N=20),
                True))
    b4 = ur5_ics(np.arange(10), N=15)
    for i in (0, 2, 4, 5, 6):
        out.append((f"UR5 testing_test first solve id {i}, N 15", 4, _sub(b4, i), True))
    return out


PROBLEMS = _problems()
UR5_EARLY_STOP = [("UR5 id 1, N 15", _sub(ur5_ics(np.arange(10), N=15), 1)),
                  ("UR5 id 3, N 15", _sub(ur5_ics(np.arange(10), N=15), 3))]


@pytest.mark.parametrize("name,nq,b", [p[:3] for p in PROBLEMS] + [(n, 4, b) for n, b in UR5_EARLY_STOP],
                         ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_final_iterate_is_a_kkt_point(name, nq, b):
    r = oracle.solve_mult(nq, b, 0)
    assert r["status"] == 0, (name, r["status"])
    stat, infeas, dual, comp = kkt_residuals(nq, b, 0, r)
    # the oracle's own residual and the one recomputed here agree, and both are within the reference's tolerances
    assert stat < 1e-3 and abs(stat - r["res_stat"]) < 1e-9, (name, stat, r["res_stat"])
    assert infeas < 1e-6, (name, infeas)
    assert dual >= 0.0, (name, dual)
    assert comp < 1e-6, (name, comp)


def test_oracle_optimum_matches_slsqp_triple_and_ur5():
    """SLSQP started at the oracle's point finds no lower cost (a local minimum, not only a KKT point), and
    SLSQP from the same guess as the oracle reaches the same optimum (|dcost| < 1e-4) on >= 5 triple and 5 UR5
    problems."""
    sols = [oracle.solve_mult(nq, b, 0) for _, nq, b, _ in PROBLEMS]
    jobs = [(nq, b, 0, None) for _, nq, b, _ in PROBLEMS] + \
           [(nq, b, 0, (r["x"], r["u"])) for (_, nq, b, _), r in zip(PROBLEMS, sols)]
    with ProcessPoolExecutor(max_workers=4) as ex:
        ref = list(ex.map(_slsqp, jobs))
    cold, warm = ref[:len(PROBLEMS)], ref[len(PROBLEMS):]
    bad = []
    for (name, nq, _, same), r, (f, ok, viol), (fw, okw, violw) in zip(PROBLEMS, sols, cold, warm):
        if not (r["status"] == 0 and okw and violw < 1e-8 and fw > r["cost"] - 1e-5):
            bad.append(("descent from the oracle's point", name, r["cost"], fw, okw, violw))
        if same and not (ok and viol < 1e-8 and abs(r["cost"] - f) < 1e-4):
            bad.append(("other optimum from the same guess", name, r["cost"], f, ok, viol))
    assert not bad, bad
    assert sum(p[1] == 3 and p[3] for p in PROBLEMS) >= 5 and sum(p[1] == 4 and p[3] for p in PROBLEMS) >= 5


def test_ur5_early_stops_are_kkt_points_but_not_minima():
    """The two UR5 problems where the oracle stops within tol_stat short of a minimum: SLSQP started at the
    oracle's point descends (the loose tol_stat of the reference's option set, not a solver defect - the
    KKT test above pins the point itself)."""
    sols = [oracle.solve_mult(4, b, 0) for _, b in UR5_EARLY_STOP]
    with ProcessPoolExecutor(max_workers=2) as ex:
        ref = list(ex.map(_slsqp, [(4, b, 0, (r["x"], r["u"])) for (_, b), r in zip(UR5_EARLY_STOP, sols)]))
    for (name, _), r, (f, ok, viol) in zip(UR5_EARLY_STOP, sols, ref):
        assert ok and viol < 1e-8
        assert f < r["cost"] - 1e-2, (name, r["cost"], f)
        assert 1e-5 < r["res_stat"] < 1e-3
