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
ones) is unpinned: `cost_scale` states the choice (default: the time step).
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
def simulate_batch(solve, rk4, spec, x0s, x_guess, u_guess, tot_steps=100):
    """The reference's simulate(p) for every initial state at once: each MPC step solves the OCPs of the problems
    still running in one batched call (solve(x0 [b, 6], xg [b, N+1, 6], ug [b, N, 3]) -> dict(status, x, u)),
    applies the reference's guess shifting and failure bookkeeping per problem (failed_iter, :37-62), and steps the
    plant with one RK4 of time_step (rk4(x [b, 6], u [b, 3]) -> x1).  Returns (res_steps [B] - the step at which each
    problem stopped, as simulate returns f -, simX [B, tot_steps + 1, 6], solves)."""
    x0s = np.asarray(x0s, dtype=np.float64)
    B, N = x0s.shape[0], spec.N
    xg = np.array(x_guess, dtype=np.float64, copy=True)
    ug = np.array(u_guess, dtype=np.float64, copy=True)
    simX = np.zeros((B, tot_steps + 1, 6))
    simX[:, 0] = x0s
    failed = np.full(B, -1)
    res = np.full(B, tot_steps - 1)
    live = np.ones(B, dtype=bool)
    solves = 0
    for f in range(tot_steps):
        idx = np.flatnonzero(live)
        if idx.size == 0:
            break
        r = solve(simX[idx, f], xg[idx], ug[idx])
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
    return res, simX, solves
