"""Shared parity rules of the GPU driver tests (test helper, never imported by the product path).

The fixture tests compare a GPU run of a driver (`data_generation`, `testing`) with the reference's own function
run on the CPU oracle (tests/golden/).  Instead of an agreement bar, every problem whose GPU result differs from the
fixture must be explained: the GPU-backed and the oracle-backed drivers run in lockstep (tests/lockstep.py) and
part for an allowed reason - a tolerance decision flipped on a rounding-level difference ('decision'), a different
status for the same request ('status'), or two points that both pass the solver's own stopping test ('optimum':
tests/kkt_check.py, the ACADOS tolerances tol_stat 1e-3 / eq / ineq / comp 1e-6 with the best multipliers for each
point).  A same-status disagreement neither point of which passes ('value') or a mismatch the lockstep run does not
reproduce fails the test.  'optimum' partings are capped at 1 % of a fixture set and 'decision' partings at 3 % (at
least 2), so a build that adds many rounding-level flips fails too; the counts are returned and printed."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ALLOWED = ("decision", "optimum", "status")
DECISION_CAP, OPTIMUM_CAP = 0.03, 0.01


def caps(n):
    """(decision, optimum) partings allowed in a fixture set of n problems."""
    return max(2, int(DECISION_CAP * n)), max(1, int(OPTIMUM_CAP * n))


def golden(name):
    return json.load(open(os.path.join(HERE, "golden", name)))


class FailingGpu:
    """The product backend with the fixtures' deterministic failure injection applied on top."""

    def __init__(self, nq, fail_mod, nmax=None):
        from vboc_amd.drivers import GpuBackend
        from oracle_backend import forced_failure
        self.gpu = GpuBackend(nq) if nmax is None else GpuBackend(nq, nmax=nmax)
        self.fail_mod, self.ff = fail_mod, forced_failure
        self.nmax = self.gpu.nmax

    def solve(self, b, free_time=False):
        r = self.gpu.solve(b)
        st = np.array(r["status"], copy=True)
        for i in range(st.shape[0]):
            if self.ff(b["lbx0"][i, 0], self.fail_mod):
                st[i] = 4
        return dict(r, status=st)

    def rk4(self, x, u, T):
        return self.gpu.rk4(x, u, T)


def gens(nq, law, g):
    """pid -> a fresh generator of the driver's per-problem state machine for the fixture's law ('dg' / 'test')."""
    from vboc_amd.drivers import ProblemRNG, TEST_STREAM, data_generation_problem, testing_problem
    from vboc_amd.ics import uniforms
    ids = np.array(g["ids"] + g.get("fail_ids", []))
    U = uniforms(ids, 3 * nq + 1, g.get("seed", 20250124), stream=0 if law == "dg" else 1)
    row = {int(p): k for k, p in enumerate(ids)}
    if law == "dg":
        return lambda p: data_generation_problem(nq, p, U[row[p]], ProblemRNG(p), g["N_start"])
    return lambda p: testing_problem(nq, p, U[row[p]], ProblemRNG(p, stream=TEST_STREAM), g["N_start"])


def same_result(law, nq, a, b, tol=1e-5):
    """One problem's driver result against the fixture's: rows or None; the double's data_generation returns the
    3-tuple (rows, store_ic, store_ic) of VBOC/doublependulum_vboc.py:239,345."""
    if law == "dg" and nq == 2:
        return all(same_result("test", 1, x, y, tol) for x, y in zip(a, b))
    if a is None or b is None:
        return (a is None) == (b is None)
    a, b = np.asarray(a, float), np.asarray(b, float)
    return a.shape == b.shape and (a.size == 0 or np.abs(a - b).max() <= tol)


def explain(nq, law, g, ids, got, ref, fail_mod, gpu_result_of=None, tol=1e-5):
    """Every id whose GPU result `got` differs from the fixture's `ref` must part in lockstep (GPU vs oracle) for an
    ALLOWED reason.  gpu_result_of(pid) (device-loop tests, double pendulum only): the host driver's result on the
    GPU, for an id the lockstep run finds 'same' - allowed only when the device loop itself differs from the host
    driver there (the double's gravity-compensation guess takes the device's sin, the host driver glibc's).
    Returns (n_mismatch, {pid: kind}, trace); raises AssertionError with the evidence otherwise."""
    from kkt_check import kkt_verify
    from lockstep import explain_mismatches
    from oracle_backend import OracleBackend
    bad = [int(p) for p, a, b in zip(ids, got, ref) if not same_result(law, nq, a, b, tol)]
    if not bad:
        return 0, {}, {}
    kinds, trace = explain_mismatches(nq, gens(nq, law, g), bad, FailingGpu(nq, fail_mod),
                                      OracleBackend(nq, fail_mod), kkt_verify(nq))
    for p in bad:
        k = kinds[p]
        if k == "same" and gpu_result_of is not None and nq == 2:
            dev = got[list(map(int, ids)).index(p)]
            assert not same_result(law, nq, dev, gpu_result_of(p), 0.0), (p, "device loop equals the host driver, "
                                                                           "which equals the oracle, yet differs")
            continue
        assert k in ALLOWED, (p, k, trace.get(p))
    cap_dec, cap_opt = caps(len(ids))
    n_dec = sum(kinds[p] == "decision" for p in bad)
    n_opt = sum(kinds[p] == "optimum" for p in bad)
    assert n_dec <= cap_dec, (f"{n_dec} 'decision' partings of {len(ids)} (cap {cap_dec})", kinds)
    assert n_opt <= cap_opt, (f"{n_opt} 'optimum' partings of {len(ids)} (cap {cap_opt})", kinds)
    return len(bad), kinds, trace


def dump(name, payload):
    """Write a parity record to $VBOC_PARITY_OUT/<name> (GPU runs: the evidence copied to profiles/)."""
    d = os.environ.get("VBOC_PARITY_OUT")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, name), "w") as f:
        json.dump(payload, f, indent=1, default=lambda o: o.tolist() if hasattr(o, "tolist") else str(o))
