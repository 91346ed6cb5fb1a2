"""Batched VBOC drivers: data generation and the held-out test set
(row a10, `testing_batch`).

The reference runs `data_generation(v)` once per problem in a process pool
(VBOC/triplependulum_vboc.py:19-370 with the fan-out at :399-405; VBOC/doublependulum_vboc.py:19-403).
Each call is a state machine that issues OCP solves and twin-integrator steps one at a time:
  1. IC sampling (:32-83), Philox-keyed by problem id;
  2. horizon extension: solve, and while the cost still drops by more than tol, re-solve with N+1
     from the previous solution (<= 10 solves); on a failed solve perturb the cost direction and the
     free initial positions by <= 0.01 and restart (:105-174);
  3. the sweep f = 1..N-1 along the optimal trajectory (:205-365): while a state is on dV the
     "unviable twin" is advanced with one RK4 step (:341-360); when the trajectory leaves dX a
     verification OCP from x_sol[f] decides between V and dV (<= 5 solves, :232-339);
  4. the save filter (:362-365).
Here every problem's state machine is a Python generator that yields its next request - `Solve`
(one OCP_solve) or `Rk4` (one twin step) - and a scheduler gathers the requests of ALL problems into
one batched solve on the GPU (`vboc_solve_batch`) and one batched twin step (`vboc_rk4_batch`) per
round.  The per-problem logic is a restatement of the reference's; quirk A.3 (the duplicated
x_sol[f] sample on the unresolved branch, :333-337) is reproduced, quirk A.1 (a horizon inherited
from the previous problem of the same worker, :23) is fixed to N_start per problem
(VBOC/vboc.py:28 does the same).

Randomness: the IC sampling draws from the problem's Philox block (ics.uniforms stream 0, the
block `ics.data_generation_ics` uses), the perturbations of step 2 from a second per-problem stream
(stream 2), both in the reference's call order (`random.random()` before `random.choice`).  Parity:
tests/test_drivers.py runs the reference's own `data_generation` (AST-extracted, oracle-backed) on the
same draws and requires identical results.
"""
from dataclasses import dataclass

import numpy as np
from numpy.linalg import norm

from .ics import SEED, uniforms
from .systems import system


@dataclass
class Solve:
    """One OCP_solve: guesses have N rows (stage-N guess = last row) or N+1 rows."""
    N: int
    x_guess: np.ndarray
    u_guess: np.ndarray
    p: np.ndarray
    q_lb: np.ndarray
    q_ub: np.ndarray
    u_lb: np.ndarray
    u_ub: np.ndarray
    q_init_lb: np.ndarray
    q_init_ub: np.ndarray
    q_fin_lb: np.ndarray
    q_fin_ub: np.ndarray
    free_time: bool = False    # OCPpendulum.OCP_solve (free-time box OCP, vboc_solve_batch_ft)


@dataclass
class Rk4:
    """One step of the twin integrator (SYM<sys>INIT.acados_integrator, T = dt)."""
    x: np.ndarray
    u: np.ndarray
    T: float


@dataclass
class Solution:
    status: int
    x: np.ndarray      # [N+1, nx]
    u: np.ndarray      # [N, nu]
    cost: float


class ProblemRNG:
    """`random.random()` / `random.choice(seq)` drawn from one problem's Philox stream."""

    def __init__(self, pid, seed=SEED, stream=2, block=32):
        self.pid, self.seed, self.stream, self.block = int(pid), seed, stream, block
        self.buf, self.pos, self.blocks = np.empty(0), 0, 0

    def random(self):
        if self.pos >= self.buf.shape[0]:
            n = self.block * (self.blocks + 1)
            self.buf = uniforms(np.array([self.pid]), n, self.seed, self.stream)[0, self.block * self.blocks:]
            self.blocks += 1
            self.pos = 0
        u = float(self.buf[self.pos])
        self.pos += 1
        return u

    def choice(self, seq):
        u = self.random()
        return seq[min(int(u * len(seq)), len(seq) - 1)]


# ------------------------------------------------------------------------------------------------
# per-problem state machine (a restatement of the reference's data_generation)
# ------------------------------------------------------------------------------------------------
def _gravity_u(sysd, q):
    """Double-pendulum guess: gravity compensation (VBOC/doublependulum_vboc.py:84)."""
    import math
    return np.array([sysd.g * sysd.l[0] * (sysd.m[0] + sysd.m[1]) * math.sin(q[0]),
                     sysd.g * sysd.l[1] * sysd.m[1] * math.sin(q[1])])


# draws of the reference's IC sampling from the problem's first uniform block (stream 0):
# triple :33-73 (choice, choice, random, choice, random, choice, random, random x3) -> 10,
# double VBOC/doublependulum_vboc.py:35-60 (choice, choice, random, choice, random, random) -> 6
IC_DRAWS = {3: 10, 2: 6}


def data_generation_problem(nq, pid, U, rng, N_start):
    """Generator for one problem.  U: the problem's first uniform block (ics.uniforms stream 0), drawn
    in the reference's order; rng: its perturbation stream.  Yields Solve / Rk4 requests, receives
    Solution / next state.  Returns the saved samples (list of rows) or None (triple); for the
    double pendulum a 3-tuple (samples | None, ic | None, ic | None) like
    VBOC/doublependulum_vboc.py:399,402."""
    sysd = system(nq)
    NX = 2 * nq
    q_min, q_max, v_max = sysd.q_min, sysd.q_max, sysd.v_max
    v_min, tau_max, dt_sym, tol, eps = -v_max, sysd.u_max, sysd.dt, sysd.tol, sysd.eps
    grav = nq == 2
    N = N_start
    draw = iter(float(v) for v in U[:IC_DRAWS[nq]])
    pick = lambda seq: seq[min(int(next(draw) * len(seq)), len(seq) - 1)]
    # ---- IC sampling, the reference's scalar arithmetic (:33-83) ----
    joint_sel = pick(list(range(nq)))
    vel_sel = pick([-1, 1])
    q_init_sel, q_fin_sel = (q_min, q_max) if vel_sel == -1 else (q_max, q_min)
    ran1 = vel_sel * next(draw)
    others = []
    for _ in range(nq - 1):
        sgn = pick([-1, 1])
        others.append(sgn * next(draw))
    norm_weights = norm(np.array([ran1] + others))
    w = [r / norm_weights for r in [ran1] + others]
    pw = [0.0] * nq
    pw[joint_sel] = w[0]
    for c, v in zip([c for c in range(nq) if c != joint_sel], w[1:]):
        pw[c] = v
    p = np.array(pw + [0.])

    def clamp_eps(v):
        if v > q_max - eps:
            v = v - eps
        if v < q_min + eps:
            v = v + eps
        return v

    if grav:
        joint_oth = 1 - joint_sel
        ran = [ran1, others[0]]
        q_init_oth = clamp_eps(q_min + next(draw) * (q_max - q_min))
        store_ic = [vel_sel + 1 + joint_sel, ran[0], ran[1], q_init_oth]
        qpos = [q_init_oth] * nq
    else:
        qpos = [clamp_eps(q_min + next(draw) * (q_max - q_min)) for _ in range(nq)]
    q_init_lb = np.array(qpos + [v_min] * nq + [dt_sym])
    q_init_ub = np.array(qpos + [v_max] * nq + [dt_sym])
    sel0 = q_min + eps if q_init_sel == q_min else q_max - eps
    q_init_lb[joint_sel] = sel0
    q_init_ub[joint_sel] = sel0
    q_lb = np.array([q_min] * nq + [v_min] * nq + [dt_sym])
    q_ub = np.array([q_max] * nq + [v_max] * nq + [dt_sym])
    u_lb = np.array([-tau_max] * nq)
    u_ub = np.array([tau_max] * nq)
    q_fin_lb = np.array([q_min] * nq + [0.] * nq + [dt_sym])
    q_fin_ub = np.array([q_max] * nq + [0.] * nq + [dt_sym])

    def solve(Nc, xg, ug, pc, qi_lb, qi_ub):
        return Solve(Nc, xg, ug, pc.copy(), q_lb, q_ub, u_lb, u_ub, qi_lb.copy(), qi_ub.copy(), q_fin_lb, q_fin_ub)

    def straight_guess(Nc, qpos):
        xg = np.empty((Nc, NX + 1))
        ug = np.empty((Nc, nq))
        for i, tau in enumerate(np.linspace(0, 1, Nc)):
            x_guess = np.concatenate([qpos, np.zeros(nq), [dt_sym]])
            x_guess[joint_sel] = (1 - tau) * q_init_sel + tau * q_fin_sel
            x_guess[joint_sel + nq] = 2 * (1 - tau) * (q_fin_sel - q_init_sel)
            xg[i] = x_guess
            ug[i] = _gravity_u(sysd, x_guess) if grav else np.zeros(nq)
        return xg, ug

    x_sol_guess, u_sol_guess = straight_guess(N, np.array(qpos))

    # ---- horizon extension (:105-174) ----
    cost = 1e6
    all_ok = False
    sol = None
    for _ in range(10):
        res = yield solve(N, x_sol_guess, u_sol_guess, p, q_init_lb, q_init_ub)
        if res.status == 0:
            cost_new = res.cost
            if cost_new > cost - tol:
                all_ok = True
                sol = res
                break
            cost = cost_new
            x_sol_guess = np.empty((N + 1, NX + 1))
            u_sol_guess = np.empty((N + 1, nq))
            x_sol_guess[:N] = res.x[:N]
            u_sol_guess[:N] = res.u[:N]
            x_sol_guess[N] = res.x[N]
            u_sol_guess[N] = _gravity_u(sysd, x_sol_guess[N]) if grav else np.zeros(nq)
            N = N + 1
        else:
            if grav:
                ran[0] = ran[0] + rng.random() * rng.choice([-1, 1]) * 0.01
                ran[1] = ran[1] + rng.random() * rng.choice([-1, 1]) * 0.01
                norm_weights = norm(np.array(ran))
                p = (np.array([ran[0] / norm_weights, ran[1] / norm_weights, 0.]) if joint_sel == 0
                     else np.array([ran[1] / norm_weights, ran[0] / norm_weights, 0.]))
                q_init_oth = q_init_oth + rng.random() * rng.choice([-1, 1]) * 0.01
                if q_init_oth > q_max - eps:
                    q_init_oth = q_init_oth - eps
                if q_init_oth < q_min + eps:
                    q_init_oth = q_init_oth + eps
                q_init_lb[joint_oth] = q_init_oth
                q_init_ub[joint_oth] = q_init_oth
                store_ic = [vel_sel + 1 + joint_sel, ran[0], ran[1], q_init_oth]
            else:
                rans = []
                for k in range(nq):
                    rans.append(p[k] + rng.random() * rng.choice([-1, 1]) * 0.01)
                norm_weights = norm(np.array(rans))
                p = np.array([r / norm_weights for r in rans] + [0])
                dev = rng.random() * rng.choice([-1, 1]) * 0.01
                for j in range(nq):
                    if j != joint_sel:
                        val = q_init_lb[j] + dev
                        if val > q_max - eps:
                            val = val - eps
                        if val < q_min + eps:
                            val = val + eps
                        q_init_lb[j] = val
                        q_init_ub[j] = val
            x_sol_guess, u_sol_guess = straight_guess(N, q_init_lb[:nq])
            cost = 1e6

    if not all_ok:
        return (None, None, store_ic) if grav else None

    # ---- sweep along the optimal trajectory (:177-365) ----
    x_sol = np.array(sol.x[:N + 1], dtype=float)
    u_sol = np.array(sol.u[:N], dtype=float)
    x_sym = [None] * (N + 1)
    valid_data = [x_sol[0][:NX].tolist()]
    x_out = np.copy(x_sol[0][:NX])
    for j in range(nq):
        x_out[nq + j] = x_out[nq + j] - eps * p[j]

    def vel_out(xo):
        return any(xo[nq + j] > v_max or xo[nq + j] < v_min for j in range(nq))

    def pos_at_limit(xs):
        return any(xs[j] > q_max - eps or xs[j] < q_min + eps for j in range(nq))

    is_x_at_limit = vel_out(x_out)
    if not is_x_at_limit:
        x_sym[0] = x_out
    for f in range(1, N):
        if is_x_at_limit:
            x_out = np.copy(x_sol[f][:NX])
            norm_vel = norm(x_out[nq:])
            for j in range(nq):
                x_out[nq + j] = x_out[nq + j] + eps * x_out[nq + j] / norm_vel
            if pos_at_limit(x_sol[f]) or vel_out(x_out):
                is_x_at_limit = True
            else:
                is_x_at_limit = False
                if pos_at_limit(x_sol[f - 1]):
                    break
                # verification OCP from x_sol[f] (:245-339)
                N_test = N - f
                norm_weights = norm(np.array([x_sol[f][nq + j] for j in range(nq)]))
                p = np.array([-x_sol[f][nq + j] / norm_weights for j in range(nq)] + [0.])
                q_init_lb = np.concatenate([x_sol[f][:nq], [v_min] * nq, [dt_sym]])
                q_init_ub = np.concatenate([x_sol[f][:nq], [v_max] * nq, [dt_sym]])
                x_sol_guess = np.empty((N_test + 1, NX + 1))
                u_sol_guess = np.empty((N_test + 1, nq))
                for i in range(N_test):
                    x_sol_guess[i] = x_sol[i + f]
                    u_sol_guess[i] = u_sol[i + f]
                x_sol_guess[N_test] = x_sol[N]
                u_sol_guess[N_test] = _gravity_u(sysd, x_sol[N]) if grav else np.zeros(nq)
                norm_old = norm(np.array([x_sol[f][nq:NX]]))
                norm_bef = 0
                ok_v = False
                sol_v = None
                norm_new = None
                for _ in range(5):
                    res = yield solve(N_test, x_sol_guess, u_sol_guess, p, q_init_lb, q_init_ub)
                    if res.status == 0:
                        x0_new = res.x[0]
                        norm_new = norm(np.array([x0_new[nq:NX]]))
                        if norm_new < norm_bef + tol:
                            ok_v = True
                            sol_v = res
                            break
                        norm_bef = norm_new
                        x_sol_guess = np.empty((N_test + 1, NX + 1))
                        u_sol_guess = np.empty((N_test + 1, nq))
                        x_sol_guess[:N_test] = res.x[:N_test]
                        u_sol_guess[:N_test] = res.u[:N_test]
                        x_sol_guess[N_test] = res.x[N_test]
                        u_sol_guess[N_test] = _gravity_u(sysd, x_sol_guess[N_test]) if grav else np.zeros(nq)
                        N_test = N_test + 1
                    else:
                        break
                if ok_v:
                    if norm_new > norm_old + tol:   # the state is inside V
                        for i in range(N - f):
                            x_sol[i + f] = sol_v.x[i]
                            u_sol[i + f] = sol_v.u[i]
                        x_out = np.copy(x_sol[f][:NX])
                        for j in range(nq):
                            x_out[nq + j] = x_out[nq + j] + eps * x_out[nq + j] / norm_new
                        if vel_out(x_out):
                            is_x_at_limit = True
                        else:
                            is_x_at_limit = False
                            x_sym[f] = x_out
                    else:                            # the state is on dV
                        is_x_at_limit = False
                        x_out = np.copy(x_sol[f][:NX])
                        for j in range(nq):
                            x_out[nq + j] = x_out[nq + j] - eps * p[j]
                        if x_out[joint_sel + nq] > v_max:
                            x_out[joint_sel + nq] = v_max
                        if x_out[joint_sel + nq] < v_min:
                            x_out[joint_sel + nq] = v_min
                        x_sym[f] = x_out
                else:
                    # unresolved: the reference appends x_sol[f] once per later state at a velocity
                    # limit (quirk A.3, :333-337), then stops the sweep
                    for r in range(f, N):
                        if any(abs(x_sol[r][nq + j]) > v_max - eps for j in range(nq)):
                            valid_data.append(x_sol[f][:NX].tolist())
                    break
        else:
            x_out = yield Rk4(np.array(x_sym[f - 1], dtype=float), np.copy(u_sol[f - 1]), dt_sym)
            x_sym[f] = x_out
            is_x_at_limit = (any(x_out[j] > q_max or x_out[j] < q_min for j in range(nq)) or vel_out(x_out))
        if (all(q_min + eps < x_sol[f][j] < q_max - eps for j in range(nq))
                and all(abs(x_sol[f][nq + j]) > tol for j in range(nq))):
            valid_data.append(x_sol[f][:NX].tolist())
    return (valid_data, store_ic, None) if grav else valid_data


# ------------------------------------------------------------------------------------------------
# held-out test-set state machine (a restatement of the reference's `testing`)
# ------------------------------------------------------------------------------------------------
# draws of `testing` from the problem's first uniform block (ics.uniforms stream 1, the block
# ics.heldout_ics uses): (choice, random) per joint, then one position per joint; the pendulum draws
# choice, then its position (triplependulum_testdata.py:19-28, doublependulum_testdata.py:19-27,
# pendulum_testdata.py:14-18)
TEST_DRAWS = {3: 9, 2: 6, 1: 2}
TEST_STREAM = 3          # the restart perturbations of `testing` (stream 2 is data_generation's)
MAX_TEST_RESTARTS = 100  # the reference retries forever (`while True`, :41); a problem still failing
                         # after this many perturbed restarts returns None


def testing_problem(nq, pid, U, rng, N_start, max_restarts=MAX_TEST_RESTARTS):
    """Generator for one held-out problem (triplependulum_testdata.py:9-125, the double
    doublependulum_testdata.py:9-121; the pendulum pendulum_testdata.py:7-53 solves once).
    U: the problem's first uniform block (stream 1), drawn in the reference's order; rng: its restart
    stream.  Yields Solve requests and returns x_0[:2nq] of the accepted solution (None if the
    pendulum's single solve fails or the restart cap is hit)."""
    sysd = system(nq)
    NX = 2 * nq
    q_min, q_max, v_max = sysd.q_min, sysd.q_max, sysd.v_max
    v_min, tau_max, dt_sym = -v_max, sysd.u_max, sysd.dt
    grav = nq == 2
    draw = iter(float(v) for v in U[:TEST_DRAWS[nq]])
    pick = lambda seq: seq[min(int(next(draw) * len(seq)), len(seq) - 1)]
    q_lb = np.array([q_min] * nq + [v_min] * nq + [dt_sym])
    q_ub = np.array([q_max] * nq + [v_max] * nq + [dt_sym])
    u_lb = np.array([-tau_max] * nq)
    u_ub = np.array([tau_max] * nq)
    q_fin_lb = np.array([q_min] * nq + [0.] * nq + [dt_sym])
    q_fin_ub = np.array([q_max] * nq + [0.] * nq + [dt_sym])

    if nq == 1:
        ran = pick([-1, 1])
        p = np.array([ran, 0.])
        q_init = q_min + next(draw) * (q_max - q_min)
        x0b = np.array([q_init, v_min, dt_sym]), np.array([q_init, v_max, dt_sym])
        xg = np.full((N_start, 3), np.array([q_init, 0., dt_sym]))
        res = yield Solve(N_start, xg, np.zeros((N_start, 1)), p, q_lb, q_ub, u_lb, u_ub, x0b[0], x0b[1],
                          q_fin_lb, q_fin_ub)
        return res.x[0][:2].copy() if res.status == 0 else None

    rans = []
    for _ in range(nq):
        c = pick([-1, 1])
        rans.append(c * next(draw))

    def direction(rs):
        nw = norm(np.array(rs))
        return np.array([r / nw for r in rs] + [0.])

    def start(qs):
        xg = np.full((N_start, NX + 1), np.array(qs + [0.] * nq + [dt_sym]))
        ug = np.full((N_start, nq), _gravity_u(sysd, qs) if grav else np.zeros(nq))
        return (np.array(qs + [v_min] * nq + [dt_sym]), np.array(qs + [v_max] * nq + [dt_sym]), xg, ug)

    p = direction(rans)
    qs = [q_min + next(draw) * (q_max - q_min) for _ in range(nq)]
    q_init_lb, q_init_ub, x_sol_guess, u_sol_guess = start(qs)
    fmt, dec = ("{:.4f}", 1e-4) if grav else ("{:.3f}", 1e-3)   # doublependulum_testdata.py:80 / :82
    N = N_start
    cost = 1e6
    restarts = 0
    while True:
        res = yield Solve(N, x_sol_guess, u_sol_guess, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub,
                          q_fin_lb, q_fin_ub)
        if res.status == 0:
            cost_new = res.cost
            if cost_new > float(fmt.format(cost)) - dec:
                return res.x[0][:NX].copy()
            cost = cost_new
            x_sol_guess = np.empty((N + 1, NX + 1))
            u_sol_guess = np.empty((N + 1, nq))
            x_sol_guess[:N] = res.x[:N]
            u_sol_guess[:N] = res.u[:N]
            x_sol_guess[N] = res.x[N]
            u_sol_guess[N] = _gravity_u(sysd, x_sol_guess[N]) if grav else np.zeros(nq)
            N = N + 1
        else:
            restarts += 1
            if restarts > max_restarts:
                return None
            N = N_start
            for j in range(nq):
                rans[j] = rans[j] + rng.random() * rng.choice([-1, 1]) * 0.01
            p = direction(rans)
            for j in range(nq):
                qs[j] = qs[j] + rng.random() * rng.choice([-1, 1]) * 0.01
            q_init_lb, q_init_ub, x_sol_guess, u_sol_guess = start(qs)
            cost = 1e6


# ------------------------------------------------------------------------------------------------
# scheduler + backends
# ------------------------------------------------------------------------------------------------
class GpuBackend:
    """The product backend: batched OCP solves and twin steps on the GPU (libvboc_amd)."""

    def __init__(self, nq, nmax=200, device=0, path_constraint=None, **options):
        """path_constraint: systems.CartesianConstraint for the Cartesian double pendulum's OCP."""
        from . import lib
        self.lib = lib
        self.nq = nq
        self.nmax = nmax
        self.solver = lib.Solver(nq, nmax, device=device, **options)
        if path_constraint is not None:
            self.solver.set_path_constraint(path_constraint)

    def solve(self, batch, free_time=False):
        return self.solver.solve_host(batch, free_time=free_time)

    def rk4(self, x, u, T):
        return self.lib.rk4_host(self.nq, T, x, u)


def _pack(nq, reqs, nmax):
    """Solve requests -> one padded batch in the ics layout (rows beyond N unused)."""
    B = len(reqs)
    nx = 2 * nq + 1
    Nmax = max(r.N for r in reqs)
    if Nmax > nmax:
        raise ValueError(f"horizon {Nmax} exceeds the solver's nmax {nmax}")
    xg = np.zeros((B, Nmax + 1, nx))
    ug = np.zeros((B, Nmax, nq))
    for b, r in enumerate(reqs):
        xg[b, :r.N] = r.x_guess[:r.N]
        xg[b, r.N] = r.x_guess[-1]
        ug[b, :r.N] = r.u_guess[:r.N]
        xg[b, r.N + 1:] = xg[b, r.N]
    stack = lambda name: np.stack([getattr(r, name) for r in reqs]).astype(np.float64)
    return dict(N=np.array([r.N for r in reqs], dtype=np.int32), x_guess=xg, u_guess=ug, p=stack("p"),
                lbx=stack("q_lb"), ubx=stack("q_ub"), lbu=stack("u_lb"), ubu=stack("u_ub"),
                lbx0=stack("q_init_lb"), ubx0=stack("q_init_ub"), lbxe=stack("q_fin_lb"),
                ubxe=stack("q_fin_ub"))


def run_problems(nq, gens, backend, nmax=200):
    """Drive the generators to completion: every round, all pending OCP solves go to the backend as
    one batch and all pending twin steps as one batched call.  Returns the generators' results."""
    results = [None] * len(gens)
    pending = {}
    for i, g in enumerate(gens):
        try:
            pending[i] = next(g)
        except StopIteration as e:
            results[i] = e.value
    stats = dict(rounds=0, solves=0, rk4=0)
    while pending:
        stats["rounds"] += 1
        rk = [i for i, r in pending.items() if isinstance(r, Rk4)]
        sv = [i for i, r in pending.items() if isinstance(r, Solve)]
        answers = {}
        if rk:
            x = np.stack([pending[i].x for i in rk])
            u = np.stack([pending[i].u for i in rk])
            T = pending[rk[0]].T
            x1 = backend.rk4(x, u, T)
            for k, i in enumerate(rk):
                answers[i] = x1[k]
            stats["rk4"] += len(rk)
        if sv and not rk:
            # solves are the expensive part: batch them only once no twin steps are outstanding, so
            # problems that are sweeping catch up and join the next solve batch
            for ft in (False, True):
                grp = [i for i in sv if pending[i].free_time == ft]
                if not grp:
                    continue
                reqs = [pending[i] for i in grp]
                b = _pack(nq, reqs, nmax)
                out = backend.solve(b, free_time=True) if ft else backend.solve(b)
                for k, i in enumerate(grp):
                    Nk = reqs[k].N
                    answers[i] = Solution(int(out["status"][k]), out["x"][k, :Nk + 1], out["u"][k, :Nk],
                                          float(out["cost"][k]))
                stats["solves"] += len(grp)
        for i, a in answers.items():
            try:
                pending[i] = gens[i].send(a)
            except StopIteration as e:
                results[i] = e.value
                del pending[i]
    return results, stats


def data_generation_batch(nq, ids, backend, N_start=None, seed=SEED):
    """`data_generation(v)` for every problem id in `ids`, batched.  Returns
    (results, stats): results[i] is what the reference's call returns for problem ids[i]
    (triple: list of samples or None; double: 3-tuple)."""
    sysd = system(nq)
    N_start = N_start or sysd.N
    ids = np.asarray(ids)
    U = uniforms(ids, 3 * nq + 1, seed)
    gens = [data_generation_problem(nq, int(pid), U[b], ProblemRNG(int(pid), seed), N_start)
            for b, pid in enumerate(ids)]
    return run_problems(nq, gens, backend, nmax=getattr(backend, "nmax", 200))


def data_generation_device(nq, ids, solver, N_start=None, seed=SEED):
    """`data_generation(v)` for every problem id, with the WHOLE state machine on the GPU
    (vboc_data_generation: one wave per problem runs the IC sampling, the horizon-extension and
    verification solves and the twin steps of the sweep, dg.h).  Same return values as
    `data_generation_batch` - results[i] is what the reference's call returns for ids[i] (triple: list of
    samples or None; double: 3-tuple) - and stats (solves, rk4, sqp_iter totals).  `solver`: a
    lib.Solver for nq with nmax >= N_start + 12."""
    import torch
    ids_t = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=f"cuda:{solver.device}")
    out = solver.data_generation_device(ids_t, N_start=N_start, seed=seed)
    rows = out["rows"].cpu().numpy()
    off, cnt = out["row_off"].cpu().numpy(), out["row_cnt"].cpu().numpy()
    ic, slot = out["ic"].cpu().numpy(), out["ic_slot"].cpu().numpy()
    st = out["stats"].cpu().numpy()
    results = []
    for b in range(len(cnt)):
        if cnt[b] < -1:
            raise RuntimeError(f"problem {ids[b]}: row pool overflow")
        samples = None if cnt[b] < 0 else [r.tolist() for r in rows[off[b]:off[b] + cnt[b]]]
        if nq == 2:
            icb = [int(ic[b, 0])] + ic[b, 1:].tolist()
            results.append((samples, icb, None) if slot[b] == 1 else (None, None, icb))
        else:
            results.append(samples)
    stats = dict(solves=int(st[:, 0].sum()), rk4=int(st[:, 1].sum()), sqp_iter=int(st[:, 2].sum()), rounds=1,
                 per_problem=st, spec_solves=out["spec_solves"], spec_used=out["spec_used"])
    return results, stats


def testing_device(nq, ids, solver, N_start=None, seed=SEED, max_restarts=MAX_TEST_RESTARTS):
    """`testing(v)` for every problem id with the whole state machine on the GPU (vboc_testing: one wave per
    problem runs the draws, the horizon extension and the perturbed restarts, dg.h k_ts).  Same return values
    as `testing_batch`: results[i] = x_0[:2nq] of ids[i] or None, and stats.  `solver`: a lib.Solver for nq
    (double or triple) with nmax >= N_start + 12."""
    import torch
    ids_t = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=f"cuda:{solver.device}")
    out = solver.testing_device(ids_t, N_start=N_start, seed=seed, max_restarts=max_restarts)
    rows, cnt, st = out["rows"].cpu().numpy(), out["row_cnt"].cpu().numpy(), out["stats"].cpu().numpy()
    results = [rows[b].copy() if cnt[b] == 1 else None for b in range(len(cnt))]
    stats = dict(solves=int(st[:, 0].sum()), sqp_iter=int(st[:, 2].sum()), rounds=1, per_problem=st)
    return results, stats


def testing_batch(nq, ids, backend, N_start=None, seed=SEED, max_restarts=MAX_TEST_RESTARTS):
    """`testing(v)` for every problem id in `ids`, batched.  Returns (results, stats):
    results[i] is x_0[:2nq] of problem ids[i] (or None)."""
    sysd = system(nq)
    N_start = N_start or sysd.N
    ids = np.asarray(ids)
    U = uniforms(ids, 3 * nq + 1, seed, stream=1)
    gens = [testing_problem(nq, int(pid), U[b], ProblemRNG(int(pid), seed, stream=TEST_STREAM), N_start,
                            max_restarts) for b, pid in enumerate(ids)]
    return run_problems(nq, gens, backend, nmax=getattr(backend, "nmax", 200))


# ------------------------------------------------------------------------------------------------
# UR5 arm (BASELINE config 5): the main block of VBOC/UR5/vboc_multiprocessing_ur5.py fans
# `testing_test` (:369-466) out over Pool(30) for the 10k test set (:487-498) and the 1M training set
# (:506-528).  Each call extends the horizon while the cost still drops by more than tol and returns
# [x_0]; a failed solve returns None (no restarts).
# ------------------------------------------------------------------------------------------------
def ur5_problem(pid, U, N_start=100):
    """Generator for one `testing_test` problem; U: the problem's uniform block (ics.UR5_STREAM), drawn
    in the reference's order (random() before choice() in `random.random() * random.choice([-1, 1])`).
    Requests use the 9-column C-ABI layout (time step pinned in the dt column, p padded with 0)."""
    from .ics import UR5_DRAWS
    from .ur5 import DT, NQ, U_LIMITS, XMAX, XMIN
    tol = 1e-3                                   # nlp_solver_tol_stat (:483)
    draw = iter(float(v) for v in U[:UR5_DRAWS])
    pick = lambda seq: seq[min(int(next(draw) * len(seq)), len(seq) - 1)]
    p = np.empty(NQ)
    for j in range(NQ):
        r = next(draw)
        p[j] = r * pick([-1, 1])
    p = p / norm(p)
    q0 = np.empty(NQ)
    for j in range(NQ):
        q0[j] = XMIN[j] + next(draw) * (XMAX[j] - XMIN[j])
    col = lambda a: np.r_[a, DT]
    q_lb, q_ub = col(XMIN), col(XMAX)
    u_lb, u_ub = -U_LIMITS, U_LIMITS.copy()
    q_init_lb, q_init_ub = col(np.r_[q0, XMIN[NQ:]]), col(np.r_[q0, XMAX[NQ:]])
    q_fin_lb, q_fin_ub = col(np.r_[XMIN[:NQ], np.zeros(NQ)]), col(np.r_[XMAX[:NQ], np.zeros(NQ)])
    pp = np.r_[p, 0.0]
    N = N_start
    xg = np.tile(col(np.r_[q0, np.zeros(NQ)]), (N, 1))
    ug = np.zeros((N, NQ))
    cost_old = 1e6
    while True:
        res = yield Solve(N, xg, ug, pp, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb, q_fin_ub)
        if res.status != 0:
            return None
        if res.cost > cost_old - tol:
            return [res.x[0][:2 * NQ].copy()]
        cost_old = res.cost
        xg = np.empty((N + 1, 2 * NQ + 1))
        ug = np.empty((N + 1, NQ))
        xg[:N] = res.x[:N]
        ug[:N] = res.u[:N]
        xg[N] = res.x[N]
        ug[N] = 0.0
        N = N + 1


def ur5_testing_batch(ids, backend, N_start=100, seed=SEED):
    """`testing_test(v)` for every problem id in `ids`, batched.  Returns (results, stats): results[i] is
    [x_0] (8 floats) or None, as the reference's call returns."""
    from .ics import UR5_DRAWS, UR5_STREAM
    ids = np.asarray(ids)
    U = uniforms(ids, UR5_DRAWS, seed, stream=UR5_STREAM)
    gens = [ur5_problem(int(pid), U[b], N_start) for b, pid in enumerate(ids)]
    return run_problems(4, gens, backend, nmax=getattr(backend, "nmax", 200))


def _tt_results(out, ncols):
    rows, cnt, st = out["rows"].cpu().numpy(), out["row_cnt"].cpu().numpy(), out["stats"].cpu().numpy()
    results = [[rows[b, :ncols].copy()] if cnt[b] == 1 else None for b in range(len(cnt))]
    return results, dict(solves=int(st[:, 0].sum()), sqp_iter=int(st[:, 2].sum()), rounds=1, per_problem=st)


def ur5_testing_device(ids, solver, N_start=100, seed=SEED):
    """`testing_test(v)` of the UR5 driver for every problem id with the whole state machine on the GPU
    (vboc_testing_test: one wave per problem, dg.h k_tt).  Same return values as `ur5_testing_batch`.
    `solver`: a lib.Solver(4, nmax)."""
    import torch
    from .ics import UR5_STREAM
    from .ur5 import DT, NQ, U_LIMITS, XMAX, XMIN
    ids_t = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=f"cuda:{solver.device}")
    out = solver.testing_test_device(ids_t, N_start, seed, UR5_STREAM, 1e-3, DT, XMIN, XMAX, U_LIMITS)
    return _tt_results(out, 2 * NQ)


def cartesian_testing_device(ids, solver, N_start=100, seed=SEED):
    """`testing_test(v)` of the Cartesian driver for every problem id on the GPU (vboc_testing_test, k_tt with
    the keep-out circle).  Same return values as `cartesian_testing_batch` ([x_0] with the dt column, or None).
    `solver`: a lib.Solver(2, nmax) with set_path_constraint(systems.cartesian_constraint())."""
    import torch
    from .ics import CART_STREAM
    sysd = system(2)
    ids_t = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=f"cuda:{solver.device}")
    xlo = [sysd.q_min] * 2 + [-sysd.v_max] * 2
    xhi = [sysd.q_max] * 2 + [sysd.v_max] * 2
    out = solver.testing_test_device(ids_t, N_start, seed, CART_STREAM, sysd.tol, sysd.dt, xlo, xhi, [sysd.u_max] * 2)
    return _tt_results(out, 5)


def ur5_set(results):
    """X = np.array([i for f in X_temp for i in f]) over the non-None results (:493-495)."""
    rows = [row for t in results if t is not None for row in t]
    return np.array(rows, dtype=np.float64).reshape(len(rows), 8)


# ------------------------------------------------------------------------------------------------
# Cartesian double pendulum (VBOC/Cartesian constraints/): the main block of vboc_multiprocessing.py fans
# `testing_test` (:19-129) out over Pool(30) for the 1k test set (:557-562) and the 100k training set
# (:567-585), on OCPdoublependulumINIT with the end-effector keep-out circle (the solver backend must carry
# systems.cartesian_constraint()).  Same state machine as the UR5's: extend N while the cost drops by more
# than tol, return [x_0] (5 values, dt included: ocp_solver.get(0, "x")); a failed solve returns None.
# ------------------------------------------------------------------------------------------------
def cartesian_problem(pid, U, N_start=100):
    """Generator for one Cartesian `testing_test` problem; U: the problem's uniform block
    (ics.CART_STREAM), drawn in the reference's order (:33-50)."""
    from .ics import CART_DRAWS
    sysd = system(2)
    tol = sysd.tol                                # nlp_solver_tol_stat (:547)
    v_max, v_min, q_max, q_min, tau_max, dt = sysd.v_max, -sysd.v_max, sysd.q_max, sysd.q_min, sysd.u_max, sysd.dt
    draw = iter(float(v) for v in U[:CART_DRAWS])
    pick = lambda seq: seq[min(int(next(draw) * len(seq)), len(seq) - 1)]
    p = np.zeros(3)
    for j in range(2):
        r = next(draw)
        p[j] = r * pick([-1, 1])
    p = p / norm(p)
    q_init_lb, q_init_ub = np.full(5, v_min), np.full(5, v_max)
    q_init_lb[-1] = q_init_ub[-1] = dt
    q0 = np.empty(2)
    for j in range(2):
        q0[j] = q_min + next(draw) * (q_max - q_min)
        q_init_lb[j] = q_init_ub[j] = q0[j]
    q_lb, q_ub = q_init_lb.copy(), q_init_ub.copy()
    q_lb[:2], q_ub[:2] = q_min, q_max
    u_lb, u_ub = np.full(2, -tau_max), np.full(2, tau_max)
    q_fin_lb, q_fin_ub = q_lb.copy(), q_ub.copy()
    q_fin_lb[2:4] = q_fin_ub[2:4] = 0.0
    N = N_start
    x_guess = np.zeros(5)
    x_guess[:2] = q0
    x_guess[-1] = dt
    xg = np.tile(x_guess, (N, 1))
    ug = np.zeros((N, 2))
    cost_old = 1e6
    while True:
        res = yield Solve(N, xg, ug, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb, q_fin_ub)
        if res.status != 0:
            return None
        if res.cost > cost_old - tol:
            return [res.x[0].copy()]
        cost_old = res.cost
        xg = np.empty((N + 1, 5))
        ug = np.empty((N + 1, 2))
        xg[:N] = res.x[:N]
        ug[:N] = res.u[:N]
        xg[N] = res.x[N]
        ug[N] = 0.0
        N = N + 1


def cartesian_testing_batch(ids, backend, N_start=100, seed=SEED):
    """`testing_test(v)` of the Cartesian driver for every problem id, batched.  Returns (results, stats):
    results[i] is [x_0] (5 floats) or None.  `backend` solves with the keep-out circle."""
    from .ics import CART_DRAWS, CART_STREAM
    ids = np.asarray(ids)
    U = uniforms(ids, CART_DRAWS, seed, stream=CART_STREAM)
    gens = [cartesian_problem(int(pid), U[b], N_start) for b, pid in enumerate(ids)]
    return run_problems(2, gens, backend, nmax=getattr(backend, "nmax", 200))


# ------------------------------------------------------------------------------------------------
# pendulum VBOC data generation (free-time OCPs)
# ------------------------------------------------------------------------------------------------
PEND_N_START, PEND_EPS = 50, 1e-3   # VBOC/pendulum_vboc.py:21, :47


def pendulum_sweep_problem(v_sel_max, N_start=PEND_N_START, eps=PEND_EPS):
    """Generator for one of the two sweeps of the pendulum's simplified data generation
    (VBOC/pendulum_vboc.py:52-205, `for v_sel in [v_min, v_max]`).  Yields free-time Solve requests
    (OCPpendulum.OCP_solve); returns the rows it appends to X_save (lists [theta, dtheta]).
    Kept as in the reference: the horizon loop re-solves with N + 1 while |dtheta_0| grows by more
    than 1e-4 (:96-138); the verification solve is warm-started from the FIRST N_test + 1 rows of
    x_sol (:181), its status is not read (the test at :183 sees the horizon loop's status, SURVEY
    App. A.6), and a failed horizon solve raises like the reference (:138)."""
    sysd = system(1)
    v_max, q_max, q_min = sysd.v_max, sysd.q_max, sysd.q_min
    v_min = -v_max
    v_sel = v_max if v_sel_max else v_min
    N = N_start
    dt = 1e-2
    if v_sel == v_min:
        q_init, q_fin = q_max, q_min
        lb, ub = np.array([q_min, v_min, 0.]), np.array([q_max, 0., 1e-2])
        cost_dir = 1.
    else:
        q_init, q_fin = q_min, q_max
        lb, ub = np.array([q_min, 0., 0.]), np.array([q_max, v_max, 1e-2])
        cost_dir = -1.
    u_lb, u_ub = np.array([-sysd.u_max]), np.array([sysd.u_max])

    def solve(Nc, xg, ug, qi):
        # OCPpendulum.OCP_solve: stages i < Nc from the guess rows, stage Nc from row Nc
        return Solve(Nc, np.array(xg[:Nc + 1], dtype=float), np.array(ug[:Nc], dtype=float),
                     np.array([cost_dir, 1.]), lb, ub, u_lb, u_ub, np.array([qi, -v_max, 0.]),
                     np.array([qi, v_max, 1e-2]), np.array([q_fin, 0., 0.]), np.array([q_fin, 0., 1e-2]),
                     free_time=True)

    x_guess = np.empty((N + 1, 3))
    u_guess = np.zeros((N, 1))
    q_guess = np.linspace(q_init, q_fin, N + 1, endpoint=True)
    for i in range(N + 1):
        x_guess[i] = [q_guess[i], v_sel, dt]
    norm_old = v_max
    while True:
        if x_guess.shape[0] < N + 1:
            raise IndexError("stage-N guess row missing (the reference's OCP_solve indexes x_sol_guess[N])")
        res = yield solve(N, x_guess, u_guess, q_init)
        status = res.status
        if status != 0:
            raise RuntimeError("Sorry, the solver failed")
        norm_new = abs(res.x[0][1])
        if norm_new > norm_old + 1e-4:
            norm_old = norm_new
            x_guess = np.empty((N + 1, 3))
            u_guess = np.empty((N + 1, 1))
            x_guess[:N] = res.x[:N]
            u_guess[:N] = res.u[:N]
            x_guess[N] = res.x[N]
            u_guess[N] = 0.
            N = N + 1
        else:
            x_sol = np.array(res.x[:N + 1], dtype=float)
            u_sol = np.array(res.u[:N], dtype=float)
            break
    rows = [x_sol[0][:2].tolist()]
    x_out = np.copy(x_sol[0][:2])
    x_out[1] = x_out[1] - eps * cost_dir
    x_at_limit = bool(x_out[1] > v_max or x_out[1] < v_min)
    for f in range(1, N):
        if x_at_limit:
            v_out = x_sol[f][1] - eps * cost_dir
            if v_out > v_max or v_out < v_min:
                rows.append(x_sol[f][:2].tolist())
            else:
                norm_old = abs(x_sol[f][1])
                N_test = N - f
                ver = yield solve(N_test, x_sol, u_sol, x_sol[f][0])
                if status == 0:          # the horizon loop's status (quirk A.6): always 0 here
                    x0_new = ver.x[0]
                    norm_new = abs(x0_new[1])
                    if norm_new > norm_old + 1e-4:
                        for i in range(N - f):
                            x_sol[i + f] = ver.x[i]
                            u_sol[i + f] = ver.u[i]
                        x_out = np.copy(x0_new[:2])
                        x_out[1] = x_out[1] - eps * cost_dir
                        x_at_limit = bool(x_out[1] > v_max or x_out[1] < v_min)
                    else:
                        x_at_limit = False
                    rows.append(x_sol[f][:2].tolist())
        else:
            if abs(x_sol[f][0] - q_fin) <= 1e-3:
                break
            rows.append(x_sol[f][:2].tolist())
    return rows


def pendulum_data_generation(backend, N_start=PEND_N_START, eps=PEND_EPS):
    """X_save of VBOC/pendulum_vboc.py:50-205: both sweeps (v_min, then v_max) run as one batch of two
    problems.  Returns (X_save [n x 2] float64, stats)."""
    gens = [pendulum_sweep_problem(False, N_start, eps), pendulum_sweep_problem(True, N_start, eps)]
    res, stats = run_problems(1, gens, backend, nmax=getattr(backend, "nmax", 200))
    rows = res[0] + res[1]
    return np.array(rows, dtype=np.float64).reshape(len(rows), 2), stats


def heldout_set(nq, results):
    """The saved held-out array: np.array(data) (triplependulum_testdata.py:144); the pendulum drops the
    failed problems first (pendulum_testdata.py:68)."""
    rows = [r for r in results if r is not None]
    if nq > 1 and len(rows) != len(results):
        raise ValueError("a problem hit the restart cap; the reference would still be retrying it")
    return np.array(rows, dtype=np.float64).reshape(len(rows), 2 * nq)
