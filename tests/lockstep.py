"""Lockstep comparison of a batched driver on two solver backends (test helper, never imported by the
product path).

Each problem's generator (vboc_amd.drivers: data_generation_problem / testing_problem / ...) runs twice, once
per backend, in lockstep: every round, each copy's pending request goes to its own backend (batched), and the
two answers are compared.  While both copies issue the same kind of request (same horizon for a solve) and get
answers that agree to rounding, the copies are on the same path.  When they part, the first differing answer
pair says why:
  'decision' - every answer so far agreed to rounding (same status; |d cost| <= 1e-6 (1 + |cost|), |d x_0| <=
               1e-6, 1e-5 for a solve past 300 SQP iterations; twin steps from the same inputs to 1e-9): a tolerance decision of the state machine (the horizon-extension
               test, the at-limit tests, the stop rule) flipped on a rounding-level difference;
  'status'   - the two solvers returned different statuses for the same request (a rounding-level difference
               that changed the SQP path enough to hit max_iter or a QP failure on one side only);
  'optimum'  - same status 0, results differ beyond the comparison tolerance, and each side's result is confirmed as
               a valid stop of the request by an independent check (`verify`, tests/kkt_check.py: the point passes
               the solver's own stopping test - tol_stat 1e-3, eq / ineq / comp 1e-6 - with the best multipliers for
               it): two points that both satisfy the stopping tolerances - after a long SQP path (hundreds of
               iterations), or on a build whose arithmetic is re-associated, the two solvers stop at different such
               points;
  'value'    - same status, results differ beyond rounding and not both confirmed (a genuine solver disagreement).
Problems that end on the same path with the same result are 'same'."""
import numpy as np

from vboc_amd.drivers import Rk4, Solve, _pack


# x_0 agreement of two solves of the same request: 1e-6, and 1e-5 only for a long solve (either side at >= LONG_SQP
# SQP iterations): a solve that stops at tol_stat 1e-3 after hundreds of SQP iterations (the widened fixture's
# long-tail problem 1464: 531 / 664 iterations) ends 1.2e-6 from the other solver's stop with the same cost to 2e-7
X0_TOL, X0_TOL_LONG, LONG_SQP = 1e-6, 1e-5, 300


def _close_solve(a, b, sqp=(0, 0)):
    if a.status != b.status:
        return "status"
    if a.status != 0:
        return "ok"       # failed solves: the iterate is not a result
    tol = X0_TOL_LONG if max(sqp) >= LONG_SQP else X0_TOL
    if abs(a.cost - b.cost) > 1e-6 * (1 + abs(b.cost)) or np.abs(a.x[0] - b.x[0]).max() > tol:
        return "value"
    return "ok"


def _equal_result(a, b, tol=1e-5):
    if a is None or b is None:
        return (a is None) == (b is None)
    if isinstance(a, tuple):
        return all(_equal_result(x, y, tol) for x, y in zip(a, b))
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and (a.size == 0 or np.abs(a - b).max() < tol)


def _answers(nq, backend, reqs, nmax, sqp=None):
    """Answers of one backend to a round's requests; sqp (dict, optional) receives each solve's SQP iterations."""
    from vboc_amd.drivers import Solution
    out = {}
    rk = [i for i, r in reqs.items() if isinstance(r, Rk4)]
    sv = [i for i, r in reqs.items() if isinstance(r, Solve)]
    if rk:
        x1 = backend.rk4(np.stack([reqs[i].x for i in rk]), np.stack([reqs[i].u for i in rk]), reqs[rk[0]].T)
        for k, i in enumerate(rk):
            out[i] = x1[k]
    if sv:
        rs = [reqs[i] for i in sv]
        r = backend.solve(_pack(nq, rs, nmax))
        for k, i in enumerate(sv):
            n = rs[k].N
            out[i] = Solution(int(r["status"][k]), r["x"][k, :n + 1], r["u"][k, :n], float(r["cost"][k]))
            if sqp is not None:
                sqp[i] = int(r["sqp_iter"][k]) if "sqp_iter" in r else 0
    return out


def lockstep(nq, make_gen, ids, backend_a, backend_b, nmax=200, verify=None, trace=None):
    """make_gen(pid) -> a fresh generator.  Returns {pid: (kind, detail)} with kind in same / decision /
    status / optimum / value (see the module doc).  verify(request, solution) -> bool confirms a solution.
    trace (dict, optional) receives, per problem that does not end 'same', its solve pairs (side a, side b: horizon,
    status, SQP iterations, cost, x_0) - the evidence of the classification."""
    pairs = {p: [] for p in ids}
    ga = {p: make_gen(p) for p in ids}
    gb = {p: make_gen(p) for p in ids}
    ra, rb, kind = {}, {}, {}
    pa, pb = {}, {}
    for p in ids:
        pa[p], pb[p] = next(ga[p]), next(gb[p])
    last = {p: "ok" for p in ids}
    while pa:
        for p in list(pa):
            x, y = pa[p], pb[p]
            if type(x) is not type(y) or (isinstance(x, Solve) and x.N != y.N):
                kind[p] = ("decision" if last[p] == "ok" else last[p], "parted")
                del pa[p], pb[p]
        if not pa:
            break
        # twin steps first, as run_problems does (solves only once no twin step is outstanding)
        rk = {p: r for p, r in pa.items() if isinstance(r, Rk4)}
        sel = rk if rk else dict(pa)
        sa, sb = {}, {}
        aa = _answers(nq, backend_a, {p: pa[p] for p in sel}, nmax, sa)
        ab = _answers(nq, backend_b, {p: pb[p] for p in sel}, nmax, sb)
        for p in sel:
            if isinstance(pa[p], Rk4):
                # a twin step is a pure function of its inputs: only a step taken from the SAME (x, u) on both sides
                # says anything about the integrators; a step from states that already differ (two solves that
                # agree to the solver's tolerance, not to the bit) differs by what it inherited
                same_in = (np.abs(np.asarray(pa[p].x) - np.asarray(pb[p].x)).max() <= 1e-12
                           and np.abs(np.asarray(pa[p].u) - np.asarray(pb[p].u)).max() <= 1e-12)
                if same_in and np.abs(aa[p] - ab[p]).max() > 1e-9:
                    last[p] = "value"
            else:
                c = _close_solve(aa[p], ab[p], (sa.get(p, 0), sb.get(p, 0)))
                pairs[p].append({side: dict(N=int(pa[p].N), status=int(r.status), sqp=n, cost=float(r.cost),
                                            x0=[float(v) for v in np.asarray(r.x[0])])
                                 for side, r, n in (("a", aa[p], sa.get(p, 0)), ("b", ab[p], sb.get(p, 0)))})
                pairs[p][-1]["class"] = c
                if c == "value" and verify is not None and verify(pa[p], aa[p]) and verify(pb[p], ab[p]):
                    c = "optimum"
                if c != "ok" and last[p] != "value":
                    last[p] = c
            done_a = done_b = False
            try:
                pa[p] = ga[p].send(aa[p])
            except StopIteration as e:
                ra[p], done_a = e.value, True
            try:
                pb[p] = gb[p].send(ab[p])
            except StopIteration as e:
                rb[p], done_b = e.value, True
            if done_a or done_b:
                if done_a and done_b and _equal_result(ra[p], rb[p]):
                    kind[p] = ("same", "end")
                else:
                    kind[p] = ("decision" if last[p] == "ok" else last[p], "end")
                del pa[p], pb[p]
    if trace is not None:
        trace.update({p: dict(kind=list(kind[p]), solves=pairs[p]) for p in ids if kind[p][0] != "same"})
    return kind


def explain_mismatches(nq, make_gen, ids, gpu, oracle, verify, nmax=200, allowed=("decision", "optimum", "status")):
    """The fixture tests' rule, instead of an agreement bar: every problem whose GPU result differs from the
    reference fixture must be one on which the GPU-backed and the oracle-backed drivers part in lockstep for a reason
    in `allowed`.  Returns ({pid: kind}, trace)."""
    trace = {}
    kinds = lockstep(nq, make_gen, [int(p) for p in ids], gpu, oracle, nmax=nmax, verify=verify, trace=trace)
    return {p: k[0] for p, k in kinds.items()}, trace
