"""Golden outputs of the reference's data_generation state machine (run HERE only, needs /root/reference).

`data_generation` is taken from the reference driver files by AST (the function alone, parsed from the
text of VBOC/triplependulum_vboc.py and VBOC/doublependulum_vboc.py) and executed with injected globals:
  * `random`: serves the problem's Philox draws (vboc_amd.ics.uniforms stream 0 for the IC sampling,
    vboc_amd.drivers.ProblemRNG stream 2 afterwards) in the order the function asks for them;
  * `ocp`: an object with the OCP<sys>INIT surface the driver uses (N, OCP_solve, ocp_solver.get /
    get_cost / set_new_time_steps / update_qp_solver_cond_N, and the double's g, l1, l2, m1, m2)
    whose OCP_solve follows VBOC/triplependulum_class_vboc.py:155-191 (stages i < N from the guess
    rows, stage N from the last row) and solves with the CPU oracle (oracle/, test infrastructure);
  * `sim`: the twin integrator (set x/u/T, solve, get) as one oracle RK4 step.
The fixture records each problem's return value.  tests/test_drivers.py runs vboc_amd.drivers with the
same oracle backend and must reproduce it exactly: the pair pins the batched driver's restatement to
the reference's own state machine (given identical solver results).

The held-out driver `testing` (triplependulum_testdata.py:9-125, doublependulum_testdata.py:9-121,
pendulum_testdata.py:7-53) drives `ocp.ocp_solver` directly (reset / set / constraints_set / solve /
get / get_cost / set_new_time_steps).  It is extracted the same way and run against the product's
drop-in classes (vboc_amd.ocp.OCP<sys>INIT / OCPpendulum) with the oracle injected as their solver
(vboc_amd.ocp.use_backend): the fixture then pins the batched `testing_batch` to the reference's state
machine AND the drop-in classes' mapping of the ACADOS calls onto the solver.  `random` serves the
problem's stream-1 block (ics.heldout_ics) and then the restart stream (drivers.TEST_STREAM).

The pendulum's data generation (VBOC/pendulum_vboc.py:52-205) lives in the script's main block, not in a
function: its `for v_sel in [v_min, v_max]:` loop is taken by AST and run against the drop-in
OCPpendulum (free-time OCP_solve) with the oracle's free-time solver injected; the fixture is X_save.

The UR5's `testing_test` (VBOC/UR5/vboc_multiprocessing_ur5.py:369-466, what that script's main block fans
out for its test and training sets) is extracted the same way and run against the drop-in OCPUR5INIT
(vboc_amd.ur5) with the oracle injected; `random` serves the problem's ics.UR5_STREAM block.

The Cartesian double pendulum's `testing_test` (VBOC/Cartesian constraints/vboc_multiprocessing.py:19-129) is
run the same way on the drop-in vboc_amd.cartesian.OCPdoublependulumINIT (keep-out circle on the oracle).

The HJR labelling function data_generation(v) (HJR/triplependulum_hjr.py:21-40) is run the same way on a fake
`ocp` whose compute_problem solves the HJR one-step OCP on the oracle (vboc_oracle_hjr.c).

The active-learning drivers testing(s0) and testing_guess(s0) (AL/triplependulum_al.py:24-62) are run the same way on a
fake `ocp` whose compute_problem / compute_problem_nnguess solve AL's labelling OCP on the oracle
(vboc_oracle_al_solve_batch), the latter with a seeded guess network.

Usage: python tests/golden/make_driver_golden.py [dg|test|pend|ur5|cart|hjr|al]
  ->  tests/golden/driver_{2,3}.json, tests/golden/testing_{1,2,3}.json, tests/golden/driver_1.json,
      tests/golden/testing_ur5.json, tests/golden/testing_cartesian.json, tests/golden/hjr_3.json (+ hjr_net_3.npz),
      tests/golden/al_testing_3.json
"""
import ast
import json
import math
import os
import sys

import numpy as np
from numpy.linalg import norm

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
REF = "/root/reference/VBOC"

from vboc_amd.drivers import IC_DRAWS, TEST_DRAWS, TEST_STREAM, ProblemRNG  # noqa: E402
from vboc_amd.ics import SEED, uniforms  # noqa: E402
from vboc_amd.systems import system  # noqa: E402

# data_generation fixtures: 256 problems each, the triple's long-tail ids (first solves that run hundreds of SQP
# iterations, tests/test_gpu.py LONG_TAIL), and a failure-injected set (FAIL_MOD: restart branches, None returns)
LONG_TAIL = (988, 358, 832, 1464, 703, 125, 73)
IDS = {3: sorted(set(range(0, 256)) | set(LONG_TAIL)), 2: list(range(100, 356))}
FAIL_IDS = {3: list(range(2000, 2064)), 2: list(range(3000, 3064))}
TEST_IDS = {3: list(range(0, 64)), 2: list(range(0, 64)), 1: list(range(0, 128))}
FAIL_MOD = 3   # oracle_backend.forced_failure: about a third of the solves fail -> restarts exercised
N_START = 100


def extract(path, name="data_generation"):
    tree = ast.parse(open(path).read())
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name][0]
    return compile(ast.Module(body=[fn], type_ignores=[]), path, "exec")


class FakeRandom:
    def __init__(self, first, rng):
        self.first, self.rng = [float(v) for v in first], rng

    def random(self):
        return self.first.pop(0) if self.first else self.rng.random()

    def choice(self, seq):
        u = self.random()
        return seq[min(int(u * len(seq)), len(seq) - 1)]


def oracle_solve(nq, N, x_sol_guess, u_sol_guess, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb,
                 q_fin_ub):
    import oracle
    nx = 2 * nq + 1
    xg = np.zeros((1, N + 1, nx))
    ug = np.zeros((1, N, nq))
    for i in range(N):
        xg[0, i] = x_sol_guess[i]
        ug[0, i] = u_sol_guess[i]
    xg[0, N] = x_sol_guess[-1]
    a = lambda v: np.asarray(v, dtype=np.float64)[None]
    xo, uo, r = oracle.solve_batch(nq, np.array([N], np.int32), xg, ug, a(p), a(q_lb), a(q_ub), a(u_lb), a(u_ub),
                                   a(q_init_lb), a(q_init_ub), a(q_fin_lb), a(q_fin_ub), nthreads=1)
    return int(r["status"][0]), xo[0], uo[0], float(r["cost"][0])


class FakeSolver:
    def __init__(self):
        self.x = self.u = None
        self.cost = None

    def set_new_time_steps(self, steps):
        pass

    def update_qp_solver_cond_N(self, N):
        pass

    def get(self, i, field):
        return np.copy(self.x[i] if field == "x" else self.u[i])

    def get_cost(self):
        return self.cost


class FakeOCP:
    def __init__(self, nq, fail_mod=0):
        s = system(nq)
        self.nq, self.N, self.fail_mod = nq, N_START, fail_mod
        self.ocp_solver = FakeSolver()
        self.g, self.l1, self.m1 = s.g, s.l[0], s.m[0]
        if nq == 2:
            self.l2, self.m2 = s.l[1], s.m[1]

    def OCP_solve(self, *args):
        from oracle_backend import forced_failure
        st, x, u, c = oracle_solve(self.nq, self.N, *args)
        if forced_failure(args[7][0], self.fail_mod):   # q_init_lb[0]: tests/oracle_backend.py's injection rule
            st = 4
        self.ocp_solver.x, self.ocp_solver.u, self.ocp_solver.cost = x, u, c
        return st


class FakeIntegrator:
    def __init__(self, nq):
        self.nq, self.T, self.xv, self.uv, self.out = nq, 1e-2, None, None, None

    def set(self, field, v):
        setattr(self, {"x": "xv", "u": "uv", "T": "T"}[field], np.array(v, dtype=np.float64))

    def solve(self):
        import oracle
        self.out = oracle.rk4(self.nq, float(self.T), self.xv, self.uv)
        return 0

    def get(self, field):
        return np.copy(self.out)


class FakeSim:
    def __init__(self, nq):
        self.acados_integrator = FakeIntegrator(nq)


def tolist(v):
    if v is None:
        return None
    if isinstance(v, tuple):
        return [tolist(e) for e in v]
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, list):
        return [tolist(e) for e in v]
    return float(v) if isinstance(v, (float, np.floating)) else v


def _dg_chunk(args):
    """The reference's data_generation for a chunk of problem ids (one worker process)."""
    nq, fname, ids, fail_mod = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    code = extract(os.path.join(REF, fname))
    s = system(nq)
    ocp = FakeOCP(nq, fail_mod)
    g = dict(np=np, norm=norm, math=math, ocp=ocp, sim=FakeSim(nq), q_min=s.q_min, q_max=s.q_max,
             v_min=-s.v_max, v_max=s.v_max, tau_max=s.u_max, dt_sym=s.dt, tol=s.tol, eps=s.eps)
    exec(code, g)
    U = uniforms(np.array(ids), 3 * nq + 1, SEED)
    out = []
    for b, pid in enumerate(ids):
        g["random"] = FakeRandom(U[b, :IC_DRAWS[nq]], ProblemRNG(pid, SEED))
        ocp.N = N_START                       # N_start per problem
        out.append(tolist(g["data_generation"](pid)))
        print(nq, fail_mod, pid, "None" if out[-1] is None or out[-1][0] is None else
              len(out[-1] if nq == 3 else out[-1][0]), flush=True)
    return out


def _dg_run(nq, fname, ids, fail_mod, workers=8):
    from multiprocessing import Pool
    chunks = [list(c) for c in np.array_split(np.array(ids), workers) if len(c)]
    with Pool(len(chunks)) as pool:
        parts = pool.map(_dg_chunk, [(nq, fname, [int(i) for i in c], fail_mod) for c in chunks])
    return [r for part in parts for r in part]


def main():
    for nq, fname in ((3, "triplependulum_vboc.py"), (2, "doublependulum_vboc.py")):
        out = _dg_run(nq, fname, IDS[nq], 0)
        fout = _dg_run(nq, fname, FAIL_IDS[nq], FAIL_MOD)
        with open(os.path.join(HERE, f"driver_{nq}.json"), "w") as f:
            json.dump({"nq": nq, "ids": IDS[nq], "N_start": N_START, "seed": SEED, "results": out,
                       "fail_mod": FAIL_MOD, "fail_ids": FAIL_IDS[nq], "fail_results": fout,
                       "long_tail": [i for i in LONG_TAIL if nq == 3]}, f)


def main_testing():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_backend import OracleOcpBackend
    from vboc_amd import ocp as dropin
    dropin.use_backend(OracleOcpBackend(FAIL_MOD))
    for nq, fname, cls in ((3, "triplependulum_testdata.py", "OCPtriplependulumINIT"),
                           (2, "doublependulum_testdata.py", "OCPdoublependulumINIT"),
                           (1, "pendulum_testdata.py", "OCPpendulum")):
        code = extract(os.path.join(os.path.dirname(REF), fname), "testing")
        ocp = getattr(dropin, cls)()
        s = system(nq)
        g = dict(np=np, norm=norm, math=math, ocp=ocp, v_max=ocp.dthetamax, v_min=-ocp.dthetamax,
                 q_max=ocp.thetamax, q_min=ocp.thetamin, tau_max=s.u_max)
        exec(code, g)
        ids = TEST_IDS[nq]
        U = uniforms(np.array(ids), 3 * nq + 1, SEED, stream=1)
        out = []
        for b, pid in enumerate(ids):
            g["random"] = FakeRandom(U[b, :TEST_DRAWS[nq]], ProblemRNG(pid, SEED, stream=TEST_STREAM))
            out.append(tolist(g["testing"](pid)))
            print(nq, pid, out[-1], flush=True)
        with open(os.path.join(HERE, f"testing_{nq}.json"), "w") as f:
            json.dump({"nq": nq, "ids": ids, "N_start": ocp.N, "seed": SEED, "fail_mod": FAIL_MOD,
                       "results": out}, f)


def extract_pendulum_sweep(path):
    """The data-generation loop `for v_sel in [v_min, v_max]:` of VBOC/pendulum_vboc.py's main block
    (:52-205), taken by AST from the file's text."""
    tree = ast.parse(open(path).read())
    main_if = [n for n in tree.body if isinstance(n, ast.If)][-1]
    loop = [n for n in main_if.body if isinstance(n, ast.For) and isinstance(n.target, ast.Name)
            and n.target.id == "v_sel"][0]
    return compile(ast.Module(body=[loop], type_ignores=[]), path, "exec")


def main_pendulum():
    """Pendulum VBOC data generation (free-time OCPs): the reference's own loop on the drop-in
    OCPpendulum (free-time OCP_solve) with the oracle's free-time solver injected."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_backend import OracleOcpBackend
    from vboc_amd import ocp as dropin
    from vboc_amd.drivers import PEND_EPS, PEND_N_START
    dropin.use_backend(OracleOcpBackend())
    code = extract_pendulum_sweep(os.path.join(REF, "pendulum_vboc.py"))
    ocp = dropin.OCPpendulum()
    g = dict(np=np, ocp=ocp, N_start=PEND_N_START, v_max=ocp.dthetamax, v_min=-ocp.dthetamax,
             q_max=ocp.thetamax, q_min=ocp.thetamin, eps=PEND_EPS, X_save=np.empty((0, 2)))
    exec(code, g)
    X = g["X_save"]
    print("pendulum X_save", X.shape, flush=True)
    with open(os.path.join(HERE, "driver_1.json"), "w") as f:
        json.dump({"nq": 1, "N_start": PEND_N_START, "eps": PEND_EPS, "X_save": X.tolist()}, f)


UR5_IDS = list(range(0, 40))
UR5_FAIL_MOD = 7   # a few forced failures exercise the None branch


def main_ur5():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_backend import OracleOcpBackend
    from vboc_amd import ocp as dropin
    from vboc_amd.ics import UR5_DRAWS, UR5_STREAM
    from vboc_amd.ur5 import OCPUR5INIT
    dropin.use_backend(OracleOcpBackend(UR5_FAIL_MOD))
    code = extract(os.path.join(REF, "UR5", "vboc_multiprocessing_ur5.py"), "testing_test")
    ocp = OCPUR5INIT()
    g = dict(np=np, norm=norm, ocp=ocp, x_min=ocp.xmin, x_max=ocp.xmax, N_start=100, dt_sym=1e-2,
             tol=ocp.ocp.solver_options.nlp_solver_tol_stat)
    exec(code, g)
    U = uniforms(np.array(UR5_IDS), UR5_DRAWS, SEED, stream=UR5_STREAM)
    out = []
    for b, pid in enumerate(UR5_IDS):
        # testing_test draws exactly UR5_DRAWS numbers; a further draw would come from stream 6 and break parity
        g["random"] = FakeRandom(U[b], ProblemRNG(pid, SEED, stream=UR5_STREAM + 1))
        out.append(tolist(g["testing_test"](pid)))
        print("ur5", pid, out[-1], flush=True)
    with open(os.path.join(HERE, "testing_ur5.json"), "w") as f:
        json.dump({"nq": 4, "ids": UR5_IDS, "N_start": 100, "seed": SEED, "fail_mod": UR5_FAIL_MOD,
                   "results": out}, f)


CART_IDS = list(range(0, 48))
CART_FAIL_MOD = 11   # a few forced failures on top of the infeasible initial positions


def main_cartesian():
    """The Cartesian double pendulum's `testing_test` (VBOC/Cartesian constraints/vboc_multiprocessing.py:19-129)
    on the drop-in vboc_amd.cartesian.OCPdoublependulumINIT (keep-out circle) with the oracle injected."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_backend import OracleOcpBackend
    from vboc_amd import ocp as dropin
    from vboc_amd.cartesian import OCPdoublependulumINIT
    from vboc_amd.ics import CART_DRAWS, CART_STREAM
    dropin.use_backend(OracleOcpBackend(CART_FAIL_MOD))
    code = extract(os.path.join(REF, "Cartesian constraints", "vboc_multiprocessing.py"), "testing_test")
    ocp = OCPdoublependulumINIT()
    g = dict(np=np, norm=norm, ocp=ocp, system_sel=2, v_max=ocp.dthetamax, v_min=-ocp.dthetamax,
             q_max=ocp.thetamax, q_min=ocp.thetamin, tau_max=ocp.Cmax, dt_sym=1e-2, N_start=100,
             tol=ocp.ocp.solver_options.nlp_solver_tol_stat)
    exec(code, g)
    U = uniforms(np.array(CART_IDS), CART_DRAWS, SEED, stream=CART_STREAM)
    out = []
    for b, pid in enumerate(CART_IDS):
        g["random"] = FakeRandom(U[b], ProblemRNG(pid, SEED, stream=CART_STREAM + 1))
        out.append(tolist(g["testing_test"](pid)))
        print("cartesian", pid, out[-1], flush=True)
    with open(os.path.join(HERE, "testing_cartesian.json"), "w") as f:
        json.dump({"nq": 2, "ids": CART_IDS, "N_start": 100, "seed": SEED, "fail_mod": CART_FAIL_MOD,
                   "results": out}, f)


def main_hjr():
    """The HJR labelling function data_generation(v) of HJR/triplependulum_hjr.py:21-40, AST-extracted and run
    over 96 candidate states with injected globals: Xu_iter / y_pred (candidates and a classifier prediction),
    the state box, and `ocp` = an object with compute_problem(x0) / ocp_solver.get_cost() solving the HJR one-step
    OCP on the oracle (vboc_oracle_hjr.c).  The network: NeuralNetCLS(6, 100, 2) with seeded torch initialisation,
    stored beside the fixture (tests/golden/hjr_net_3.npz; mean 1.5, std 4.5)."""
    import oracle
    import torch
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(6, 100), torch.nn.ReLU(), torch.nn.Linear(100, 100), torch.nn.ReLU(),
                              torch.nn.Linear(100, 2))
    W = [p.detach().numpy().astype(np.float64) for p in net.parameters()]
    np.savez(os.path.join(HERE, "hjr_net_3.npz"), *W)
    mean, std = 1.5, 4.5
    rng = np.random.default_rng(3)
    X = np.c_[rng.uniform(3 * np.pi / 4 - 0.1, 5 * np.pi / 4 + 0.1, (96, 3)), rng.uniform(-11, 11, (96, 3))]
    pred = (rng.random(96) < 0.7).astype(np.int64)

    class Solver:
        cost = None

        def get_cost(self):
            return self.cost

    class HjrOcp:
        ocp_solver = Solver()

        def compute_problem(self, x0):
            r = oracle.hjr_solve_batch(3, np.asarray(x0)[None], W, mean, std, nthreads=1)
            self.ocp_solver.cost = float(r["cost"][0])
            return 1 if r["status"][0] == 0 else 0

    code = extract(os.path.join(os.path.dirname(REF), "HJR", "triplependulum_hjr.py"))
    g = dict(np=np, ocp=HjrOcp(), Xu_iter=X, y_pred=pred, q_max=np.pi / 4 + np.pi, q_min=-np.pi / 4 + np.pi,
             v_max=10.0, v_min=-10.0)
    exec(code, g)
    out = [g["data_generation"](v) for v in range(X.shape[0])]
    json.dump({"nq": 3, "mean": mean, "std": std, "X": X.tolist(), "y_pred": pred.tolist(),
               "results": [[None if s is None else np.asarray(s).tolist(), o] for s, o in out]},
              open(os.path.join(HERE, "hjr_3.json"), "w"))
    print("hjr_3.json", sum(o is not None and o[0] == 0 for _, o in out), "labelled viable of", len(out))


GUESS_SEED = 0


def main_al():
    """The active-learning labelling driver testing(s0) of AL/triplependulum_al.py:24-42 (fanned out at :133 / :284),
    AST-extracted and run over 96 states of the driver's unlabeled box (:115-123, seeded numpy draws; the widened
    velocity range puts some states out of bounds) with injected globals: the state box (:77-80), ocp_dim, and
    `ocp` = an object with the AL OCPtriplependulumINIT surface (compute_problem(q0, v0) -> 1 / 0 / 2, N,
    ocp_solver.get(i, "x")) solving the labelling OCP on the oracle (vboc_oracle_ft.c vboc_oracle_al_solve_batch)."""
    import oracle
    from vboc_amd.al import AlSpec, unlabeled_states
    spec = AlSpec()
    X = unlabeled_states(spec, 96, np.random.default_rng(4))

    class Solver:
        x = None

        def get(self, i, field):
            assert field == "x"
            return np.copy(self.x[i])

    class AlOcp:
        N, nx = spec.N, spec.nx
        ocp_solver = Solver()

        def compute_problem(self, q0, v0):
            r = oracle.al_solve_batch(spec, np.r_[q0, v0][None], nthreads=1)
            self.ocp_solver.x = r["x"][0]
            return int(r["label"][0])

    # testing_guess (:44-62) calls compute_problem_nnguess(q0, v0, model_guess, mean, std) (class :171-201): the guess
    # network NeuralNetCLS(6, 500, 6 N) seeded with torch.manual_seed(GUESS_SEED) (untrained: the reference trains it on
    # X_traj, :210-240), mean / std the scalar torch statistics of the candidate states as the driver's (:125-126)
    import torch
    from vboc_amd.al import nn_guess
    from vboc_amd.learn import NeuralNetCLS
    torch.manual_seed(GUESS_SEED)
    model_guess = NeuralNetCLS(6, 500, 6 * spec.N)
    Xt = torch.Tensor(X)
    mean, std = torch.mean(Xt), torch.std(Xt)

    class AlOcpGuess(AlOcp):
        def compute_problem_nnguess(self, q0, v0, model, mean_, std_):
            xg = nn_guess(spec.N, q0, v0, model, mean_, std_)
            r = oracle.al_solve_batch(spec, np.r_[q0, v0][None], x_guess=xg[None], nthreads=1)
            self.ocp_solver.x = r["x"][0]
            return int(r["label"][0])

    code = extract(os.path.join(os.path.dirname(REF), "AL", "triplependulum_al.py"), "testing")
    code_g = extract(os.path.join(os.path.dirname(REF), "AL", "triplependulum_al.py"), "testing_guess")
    g = dict(np=np, ocp=AlOcpGuess(), ocp_dim=6, q_max=spec.thetamax, q_min=spec.thetamin, v_max=spec.dthetamax,
             v_min=-spec.dthetamax, model_guess=model_guess, mean=mean, std=std)
    exec(code, g)
    exec(code_g, g)
    out = [g["testing"](list(map(float, s))) for s in X]
    out_g = [g["testing_guess"](list(map(float, s))) for s in X]
    enc = lambda res: [None if o is None else [o[0], o[1]] for o in res]
    json.dump({"nq": 3, "X": X.tolist(), "results": enc(out), "guess_seed": GUESS_SEED, "results_guess": enc(out_g)},
              open(os.path.join(HERE, "al_testing_3.json"), "w"))
    print("al_testing_3.json", sum(o is not None and o[0][-1] == 1 for o in out), "feasible of", len(out), "; with "
          "the guess network", sum(o is not None and o[0][-1] == 1 for o in out_g))


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("al", "all"):
        main_al()
    if what in ("hjr", "all"):
        main_hjr()
    if what in ("dg", "all"):
        main()
    if what in ("test", "all"):
        main_testing()
    if what in ("pend", "all"):
        main_pendulum()
    if what in ("ur5", "all"):
        main_ur5()
    if what in ("cart", "all"):
        main_cartesian()
