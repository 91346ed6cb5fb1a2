"""Safe MPC with the VBOC network as terminal constraint (VBOC/Safe MPC/), on the batched
solver.

The reference (`VBOC/Safe MPC/triplependulum_class_vboc.py`) wraps MODELtriplependulum (:8-78, nx 6, nu 3, the
VBOC triple's dynamics without the dt state) in an ACADOS OCP over tot_time / time_step intervals (:91-161):
  cost      LINEAR_LS, W = blockdiag(Q, R) at stages 0..N-1, W_e = Q at N (:108-134), Gauss-Newton Hessian:
            Q = diag(1e-4, 1e4, 1e-4, 1e-4, 1e-4, 1e-4), R = 1e-4 I, yref = [pi, thetamax - 0.05, pi, 0...]
  bounds    theta in [3pi/4, 5pi/4], |dtheta| <= 10 on the path and at N, |C| <= 10 (:136-151)
  options   qp_solver_iter_max 100, nlp_solver_max_iter 1000, MERIT_BACKTRACKING 0.3 / 1e-2,
            levenberg_marquardt 1e-2 (:153-161); the drivers pass "SQP_RTI"
            (hard_terminal_constraints/3dof_sym.py:96)
  OCP_solve(x0, x_sol_guess, u_sol_guess): x_0 fixed by constraints_set(0, lbx / ubx, x0), guesses at every
            stage (:163-181)
  HardTerm  the terminal row 0 <= NN(x_N) - max(|x_N[2:]|, 1e-3) <= 1e6 (:197-240; x[2:] includes theta_3 in the
            reference - kept)
The restatement: the free-time solver's model (dt a state, here pinned by x_0 and unbounded on the path - an
exact reformulation), its SQP / merit / Mehrotra IPM / Riccati recursion with the tracking cost's Gauss-Newton
Hessian and gradient and the terminal row handled like the Cartesian rows (oracle/vboc_oracle_ft.c,
vboc_amd/csrc/ft.h).  ACADOS' cost_scaling (stage costs times the time step in current releases, 1 in older
ones) is unpinned: `cost_scale` states the choice (default: the time step).  Under it the stage slack weights zl / Zl
of stages 0..N-1 are scaled too (stage N stays at 1), as ACADOS scales them; the receding driver, whose path slack
weights are large (10^(6(1 - ri/N)), 1e12), depends on that choice, so its closed-loop parity is unpinned as well.
"""
import math

import numpy as np

from .systems import system


class MpcSpec:
    """The OCP data of OCPtriplependulum (Safe MPC/triplependulum_class_vboc.py:91-161) for a time step / horizon."""

    def __init__(self, time_step=4e-3, tot_time=0.148, cost_scale=None):
        s = system(3)
        self.nq = 3
        self.time_step, self.tot_time = float(time_step), float(tot_time)
        self.N = int(self.tot_time / self.time_step)                     # :105 dims.N = int(tot_time / time_step)
        self.thetamax, self.thetamin = math.pi / 4 + math.pi, -math.pi / 4 + math.pi   # :125-127
        self.dthetamax, self.Cmax = 10.0, 10.0
        self.Q = np.array([1e-4, 1e4, 1e-4, 1e-4, 1e-4, 1e-4])          # :111-112
        self.R = np.array([1e-4, 1e-4, 1e-4])
        self.W = np.concatenate([self.Q, self.R])
        self.W_e = self.Q.copy()
        self.yref = np.array([math.pi, self.thetamax - 0.05, math.pi, 0., 0., 0., 0., 0., 0.])   # :130-131
        self.yref_e = self.yref[:6].copy()
        self.xmax = np.array([self.thetamax] * 3 + [self.dthetamax] * 3)
        self.xmin = np.array([self.thetamin] * 3 + [-self.dthetamax] * 3)
        self.umax = np.full(3, self.Cmax)
        self.umin = -self.umax
        self.cost_scale = self.time_step if cost_scale is None else float(cost_scale)
        self.lm = 1e-2
        self.g, self.m, self.l = s.g, s.m, s.l


def nn_params(model):
    """The six NeuralNetDIR parameters (list(model.parameters()), the reference's nn_params) as float64 arrays:
    CasADi's SX(param.tolist()) takes the float32 values exactly."""
    return [np.ascontiguousarray(p.detach().cpu().numpy().astype(np.float64)) for p in model.parameters()]


def nn_row(params, mean, std, x, safety_margin=None):
    """h(x) = nn_decisionfunction(params, mean, std, x) (:208-230) for one state x [6] (numpy); with safety_margin
    the SoftTraj class's nn_decisionfunction_conservative (:284-304): out * (100 - safety_margin) / 100 - vn.  The
    receding driver evaluates it on the previous solution's states (receiding_hard_constraints/3dof_sym.py:32-35)."""
    x = np.asarray(x, dtype=np.float64)
    vn = max(float(np.linalg.norm(x[2:])), 1e-3)
    z = np.concatenate([(x[:3] - mean) / std, x[3:] / vn])
    W0, b0, W1, b1, W2, b2 = params
    a = np.maximum(W0 @ z + b0, 0.0)
    a = np.maximum(W1 @ a + b1, 0.0)
    out = float((W2 @ a + b2)[0])
    if safety_margin is not None:
        out = out * (100 - safety_margin) / 100
    return out - vn


# ------------------------------------------------------------------------------------------------
# drop-in classes (Safe MPC/triplependulum_class_vboc.py:81-240) on the GPU solver, batch of one
# ------------------------------------------------------------------------------------------------
class _Dims:
    def __init__(self, N, nx, nu):
        self.N, self.nx, self.nu = N, nx, nu


class _Ocp:
    def __init__(self, spec):
        self.dims = _Dims(spec.N, 6, 3)


class _OcpSolver:
    """The ocp_solver accessors the Safe-MPC drivers use: get(i, 'x' | 'u') of the last OCP_solve."""

    def __init__(self):
        self.x = self.u = None
        self.cost = None

    def get(self, i, field):
        return np.copy(self.x[i] if field == "x" else self.u[i])

    def get_cost(self):
        return self.cost


class OCPtriplependulum:
    """OCPtriplependulum (:81-181) on the batched GPU solver (vboc_mpc_solve_batch): OCP_solve(x0, x_sol_guess,
    u_sol_guess) -> status, results through ocp_solver.get.  nn_params None: OCPtriplependulumSTD (no terminal row)."""

    def __init__(self, nlp_solver_type, time_step, tot_time, nn_params=None, mean=0.0, std=1.0, regenerate=False,
                 cost_scale=None, device=0):
        import torch
        from .lib import Solver
        self.spec = MpcSpec(time_step, tot_time, cost_scale)
        self.N = self.spec.N
        self.ocp = _Ocp(self.spec)
        self.rti = nlp_solver_type == "SQP_RTI"
        self.thetamax, self.thetamin, self.dthetamax, self.Cmax = (self.spec.thetamax, self.spec.thetamin,
                                                                   self.spec.dthetamax, self.spec.Cmax)
        self.Xmax_limits, self.Xmin_limits = self.spec.xmax, self.spec.xmin
        self.dev = torch.device("cuda", device)
        self.solver = Solver(3, max(self.N, 2), device=device)
        self.solver.set_option("levenberg_marquardt", self.spec.lm)
        self.solver.set_option("nlp_solver_tol_stat", 1e-6)       # ACADOS defaults (the class sets no tolerance)
        self.solver.set_option("qp_solver_tol_stat", 1e-8)
        self.params = None
        if nn_params is not None:
            self.params = [torch.as_tensor(np.asarray(p, dtype=np.float64), device=self.dev) for p in nn_params]
        self.mean, self.std = float(mean), float(std)
        self.ocp_solver = _OcpSolver()

    def solve_batch(self, x0, x_guess, u_guess):
        """Batched OCP_solve: numpy [B, 6], [B, N+1, 6], [B, N, 3] -> dict of numpy results."""
        import torch
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=self.dev)
        out = self.solver.mpc_solve_device(self.spec, T(x0), T(x_guess), T(u_guess), self.params, self.mean,
                                           self.std, rti=self.rti)
        torch.cuda.synchronize(self.dev)
        return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}

    def OCP_solve(self, x0, x_sol_guess, u_sol_guess):
        r = self.solve_batch(np.asarray(x0)[None], np.asarray(x_sol_guess)[None], np.asarray(u_sol_guess)[None])
        self.ocp_solver.x, self.ocp_solver.u, self.ocp_solver.cost = r["x"][0], r["u"][0], float(r["cost"][0])
        return int(r["status"][0])


class OCPtriplependulumHardTerm(OCPtriplependulum):
    """The hard terminal constraint class (:197-240): NN(x_N) - max(|x_N[2:]|, 1e-3) in [0, 1e6]."""

    def __init__(self, nlp_solver_type, time_step, tot_time, nn_params, mean, std, regenerate=False, **kw):
        super().__init__(nlp_solver_type, time_step, tot_time, nn_params=[np.asarray(p.detach().cpu().numpy()
                         if hasattr(p, "detach") else p, dtype=np.float64) for p in nn_params],
                         mean=float(mean), std=float(std), regenerate=regenerate, **kw)


class _SoftOcpSolver(_OcpSolver):
    """The SoftTraj drivers' accessors: get(i, 'x' | 'u') and cost_set(i, 'Zl' | 'zl' | 'W', value) - the per-stage
    slack weights (soft_traj_constraints/3dof_sym.py:102-105, receiding_hard_constraints/3dof_sym.py:41-46) and stage
    weights (:36-40), kept until changed, as ACADOS keeps them in the solver."""

    def __init__(self, ocp):
        super().__init__()
        self.ocp = ocp

    def cost_set(self, i, field, value):
        o, N = self.ocp, self.ocp.N
        if not 0 <= i <= N:
            raise ValueError(f"stage {i} outside 0..{N}")
        v = np.asarray(value, dtype=np.float64)
        if field in ("Zl", "zl"):
            getattr(o, field)[i] = float(v.reshape(-1)[0])
        elif field == "W":
            if np.abs(v - np.diag(np.diag(v))).max() > 0.0:
                raise NotImplementedError("cost_set(W): diagonal weights only (the drivers' block_diag(Q, R))")
            if i < N:
                o.W[i] = np.diag(v)
            else:
                o.We[:] = np.diag(v)
        else:
            raise NotImplementedError(f"cost_set field {field!r}")


class OCPtriplependulumSoftTraj(OCPtriplependulum):
    """The soft-constraint class (:242-304): the row nn_decisionfunction_conservative = NN(x) (100 - safety_margin) /
    100 - max(|x[2:]|, 1e-3) on every stage 0..N (con_h_expr and con_h_expr_e, lh = 0, uh = 1e6), soft on its lower
    side (idxsh / idxsh_e) with zl = Zl = zu = Zu = 0 until the driver sets them (ocp_solver.cost_set).  GPU:
    vboc_mpc_soft_solve_batch (ft.h)."""

    def __init__(self, nlp_solver_type, time_step, tot_time, nn_params, mean, std, safety_margin, regenerate=False,
                 **kw):
        super().__init__(nlp_solver_type, time_step, tot_time, nn_params=[np.asarray(p.detach().cpu().numpy()
                         if hasattr(p, "detach") else p, dtype=np.float64) for p in nn_params],
                         mean=float(mean), std=float(std), regenerate=regenerate, **kw)
        self.safety_margin = float(safety_margin)
        N = self.N
        self.Zl, self.zl = np.zeros(N + 1), np.zeros(N + 1)     # ocp.cost.Zl / zl / Zl_e / zl_e = 0 (:265-282)
        self.W = np.tile(self.spec.W, (N, 1))
        self.We = self.spec.W_e.copy()
        self.ocp_solver = _SoftOcpSolver(self)

    def nn_decisionfunction_conservative(self, params, mean, std, safety_margin, x):
        """The row at one state (:284-304), numerically (the receding driver's use, :32-35)."""
        P = [np.asarray(p.detach().cpu().numpy() if hasattr(p, "detach") else p, dtype=np.float64) for p in params]
        return nn_row(P, float(mean), float(std), x, safety_margin=safety_margin)

    def weights(self, B):
        """The solver's current weights as per-problem arrays (Zl, zl [B, N+1], W [B, 9], We [B, 6])."""
        if np.abs(self.W - self.W[0]).max() > 0.0:
            raise NotImplementedError("different stage weights W on different stages")
        return dict(Zl=np.tile(self.Zl, (B, 1)), zl=np.tile(self.zl, (B, 1)), W=np.tile(self.W[0], (B, 1)),
                    We=np.tile(self.We, (B, 1)))

    def solve_batch(self, x0, x_guess, u_guess, weights=None):
        """Batched OCP_solve: numpy [B, 6], [B, N+1, 6], [B, N, 3]; weights: per-problem arrays (Zl, zl, W, We;
        default: the solver's, cost_set)."""
        import torch
        B = np.asarray(x0).shape[0]
        w = self.weights(B)
        if weights is not None:
            w.update({k: np.asarray(v, dtype=np.float64) for k, v in weights.items() if v is not None})
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=self.dev)
        soft = dict(margin=self.safety_margin, **{k: T(v) for k, v in w.items()})
        out = self.solver.mpc_solve_device(self.spec, T(x0), T(x_guess), T(u_guess), self.params, self.mean,
                                           self.std, rti=self.rti, soft=soft)
        torch.cuda.synchronize(self.dev)
        return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}


class _Integrator:
    def __init__(self, T):
        self.T, self.x, self.u, self.out = T, None, None, None

    def set(self, field, v):
        if field == "T":
            self.T = float(v)
        else:
            setattr(self, field, np.asarray(v, dtype=np.float64))

    def solve(self):
        from .lib import rk4_host
        self.out = rk4_host(3, self.T, self.x[None], self.u[None])[0]
        return 0

    def get(self, field):
        return np.copy(self.out)


class SYMtriplependulum:
    """SYMtriplependulum (:70-78): one ERK4 step of T = time_step (vboc_rk4_batch)."""

    def __init__(self, time_step, tot_time, regenerate=False):
        self.acados_integrator = _Integrator(time_step)


# ------------------------------------------------------------------------------------------------
# the closed-loop driver (hard_terminal_constraints/3dof_sym.py:15-72) for a batch of initial states
# ------------------------------------------------------------------------------------------------
def simulate_batch(solve, rk4, spec, x0s, x_guess, u_guess, tot_steps=100, weights=None, log=None):
    """The reference's simulate(p) for every initial state at once: each MPC step solves the OCPs of the problems
    still running in one batched call (solve(x0 [b, 6], xg [b, N+1, 6], ug [b, N, 3]) -> dict(status, x, u)),
    applies the reference's guess shifting and failure bookkeeping per problem (failed_iter, :37-62), and steps the
    plant with one RK4 of time_step (rk4(x [b, 6], u [b, 3]) -> x1).  Returns (res_steps [B] - the step at which each
    problem stopped, as simulate returns f -, simX [B, tot_steps + 1, 6], solves).
    weights (the receding driver): weights(f, failed [b], last_x [b, N+1, 6]) -> per-problem solver weights for the
    step, passed as solve(x0, xg, ug, weights); last_x is each problem's previous solve's result (ocp_solver.get).
    log (dict, optional) receives 'u' [B, tot_steps, 3]: the control applied to the plant at each step (NaN after the
    stop)."""
    x0s = np.asarray(x0s, dtype=np.float64)
    B, N = x0s.shape[0], spec.N
    xg = np.array(x_guess, dtype=np.float64, copy=True)
    ug = np.array(u_guess, dtype=np.float64, copy=True)
    simX = np.zeros((B, tot_steps + 1, 6))
    simX[:, 0] = x0s
    failed = np.full(B, -1)
    res = np.full(B, tot_steps - 1)
    live = np.ones(B, dtype=bool)
    last_x = np.array(xg, copy=True)
    appliedU = np.full((B, tot_steps, 3), np.nan)
    solves = 0
    for f in range(tot_steps):
        idx = np.flatnonzero(live)
        if idx.size == 0:
            break
        if weights is None:
            r = solve(simX[idx, f], xg[idx], ug[idx])
        else:
            r = solve(simX[idx, f], xg[idx], ug[idx], weights(f, failed[idx], last_x[idx]))
        last_x[idx] = r["x"]
        solves += idx.size
        simU = np.zeros((idx.size, 3))
        keep = np.ones(idx.size, dtype=bool)
        for j, b in enumerate(idx):
            if r["status"][j] != 0:
                if failed[b] >= N - 1 or failed[b] < 0:
                    res[b] = f
                    live[b] = False
                    keep[j] = False
                    continue
                failed[b] += 1
                simU[j] = ug[b, 0]
                xg[b, :N - 1] = xg[b, 1:N].copy()
                ug[b, :N - 1] = ug[b, 1:N].copy()
                xg[b, N - 1] = xg[b, N]
            else:
                failed[b] = 0
                simU[j] = r["u"][j, 0]
                xg[b, :N - 1] = r["x"][j, 1:N]
                ug[b, :N - 1] = r["u"][j, 1:N]
                xg[b, N - 1] = r["x"][j, N]
                xg[b, N] = xg[b, N - 1]
                ug[b, N - 1] = ug[b, N - 2]
        step = idx[keep]
        if step.size:
            simX[step, f + 1] = rk4(simX[step, f], simU[keep])
            appliedU[step, f] = simU[keep]
    if log is not None:
        log["u"] = appliedU
    return res, simX, solves


# ------------------------------------------------------------------------------------------------
# the soft-constraint drivers (VBOC/Safe MPC/soft_traj_constraints/3dof_sym.py, receiding_hard_constraints/3dof_sym.py)
# ------------------------------------------------------------------------------------------------
def soft_traj_weights(N):
    """soft_traj_constraints/3dof_sym.py:102-105: Zl = 0 on stages 1..N-1, 1e6 at N (stage 0 keeps the class's 0)."""
    Zl = np.zeros(N + 1)
    Zl[N] = 1e6
    return Zl


def receding_weights(params, mean, std, safety_margin, N):
    """receiding_hard_constraints/3dof_sym.py:26-46 for the problems of one MPC step: the receding index from the
    previous solution (the last stage i in 1..N whose state satisfies the row, when the previous solve succeeded),
    receiding_iter = N - failed_iter - receiding, Q = diag(1e-2 + 10^(2 receiding_iter / N), 1e-4, ...), R = 1e-4 I,
    Zl = 1e12 at stage receiding_iter and 10^(6 (1 - receiding_iter / N)) elsewhere.  Returns weights(f, failed,
    last_x) for simulate_batch."""
    def weights(f, failed, last_x):
        b = failed.shape[0]
        Zl, W, We = np.empty((b, N + 1)), np.empty((b, 9)), np.empty((b, 6))
        for j in range(b):
            receiding = 0
            fi = int(failed[j])
            if fi == 0 and f > 0:
                for i in range(1, N + 1):
                    if nn_row(params, mean, std, last_x[j, i], safety_margin=safety_margin) >= 0.:
                        receiding = N - i + 1
            ri = N - fi - receiding
            Q = np.array([1e-2 + pow(10, ri / N * 2), 1e-4, 1e-4, 1e-4, 1e-4, 1e-4])
            W[j] = np.r_[Q, [1e-4, 1e-4, 1e-4]]
            We[j] = Q
            Zl[j] = pow(10, (1 - ri / N) * 6)
            if 0 <= ri <= N:
                Zl[j, ri] = 1e12
        return dict(Zl=Zl, W=W, We=We)
    return weights


def halton_states(spec, test_num=100):
    """The drivers' initial states (:98-103): a Halton sequence (scipy.stats.qmc, unscrambled) of the positions
    scaled to [Xmin, Xmax], zero velocities."""
    from scipy.stats import qmc
    sample = qmc.Halton(d=3, scramble=False).random(n=test_num)
    data = qmc.scale(sample, spec.xmin[:3], spec.xmax[:3])
    x0 = np.zeros((test_num, 6))
    x0[:, :3] = data
    return x0


def compare_steps(res_steps_traj, res_steps):
    """The drivers' comparison with the unconstrained MPC (:158-172): better / equal / worse counts."""
    d = np.asarray(res_steps_traj) - np.asarray(res_steps)
    return int((d > 0).sum()), int((d == 0).sum()), int((d < 0).sum())
