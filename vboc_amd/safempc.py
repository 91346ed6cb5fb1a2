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


def nn_row(params, mean, std, x):
    """h(x) = nn_decisionfunction(params, mean, std, x) (:208-230) for one state x [6] (numpy, for tests)."""
    x = np.asarray(x, dtype=np.float64)
    vn = max(float(np.linalg.norm(x[2:])), 1e-3)
    z = np.concatenate([(x[:3] - mean) / std, x[3:] / vn])
    W0, b0, W1, b1, W2, b2 = params
    a = np.maximum(W0 @ z + b0, 0.0)
    a = np.maximum(W1 @ a + b1, 0.0)
    return float((W2 @ a + b2)[0]) - vn
