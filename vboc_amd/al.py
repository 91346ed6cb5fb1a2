"""Active learning's labelling OCP on the batched solver (AL/).

The reference (`AL/triplependulum_class_al.py`) labels a state x0 = (q0, v0) by ONE call of ACADOS on the OCP of
OCPtriplependulum (:82-144) with the terminal rest of OCPtriplependulumINIT (:204-222):
  model     the triple pendulum, nx 6 (no dt state), nu 3, ERK4 on tf = 1 over N = 100 intervals (:85-89)
  cost      LINEAR_LS 1/2 |[x; u]|^2_W, W = blockdiag(Q, R), Q = 2 diag(0, 0, 0, 1, 1, 1), R = 0; W_e = Q (:97-115)
  bounds    theta in [3pi/4, 5pi/4], |dtheta| <= 10, |C| <= 10 on the path and at N (:118-141); terminal
            velocities fixed to 0 (lbx_e = ubx_e = 0, :210-216)
  options   none set: ACADOS' defaults - SQP_RTI (ONE QP at the reset point and its full step), GAUSS_NEWTON,
            levenberg_marquardt 0, qp_solver_iter_max 50 (PARTIAL_CONDENSING_HPIPM)
  compute_problem(q0, v0) (:148-169): reset (u = 0, multipliers 0), x_0 fixed by lbx = ubx, every stage's x guess
            (q0, 0); returns 1 if the solve's status is 0, 0 if it is 4 (QP failure), 2 otherwise.
The single QP's feasibility is the label.  The restatement (oracle/vboc_oracle_ft.c vboc_oracle_al_solve_batch,
vboc_amd/csrc/ft.h through vboc_al_solve_batch) solves that QP with the Safe-MPC solver's interior-point method and
counts a QP the IPM has not finished after qp_solver_iter_max iterations as a failure (status 4); HPIPM's own
status on such a QP is unpinned (ACADOS / HPIPM are not in this image).  The tests pin the label against an
independent LP feasibility check of the same linearised QP (tests/test_al.py).  The driver `testing(s0)`
(AL/triplependulum_al.py:24-42) is `testing_batch` below; with the guess network (compute_problem_nnguess, :171-201) the
same function restates `testing_guess(s0)` (:44-62).
"""
import math

import numpy as np


class AlSpec:
    """The OCP data of OCPtriplependulumINIT (AL/triplependulum_class_al.py:82-144, 204-222)."""

    def __init__(self, cost_scale=None):
        self.nq, self.nx, self.nu = 3, 6, 3
        self.Tf = 1.0                                   # :85
        self.N = int(100 * self.Tf)                     # :88
        self.time_step = self.Tf / self.N
        self.Cmax = 10.0                                # :118
        self.thetamax = math.pi / 4 + math.pi           # :119
        self.thetamin = -math.pi / 4 + math.pi          # :120
        self.dthetamax = 10.0                           # :121
        self.Q = 2.0 * np.array([0.0, 0.0, 0.0, 1.0, 1.0, 1.0])   # :98
        self.R = 2.0 * np.zeros(3)                                 # :99
        self.W = np.concatenate([self.Q, self.R])
        self.W_e = self.Q.copy()
        self.xmax = np.array([self.thetamax] * 3 + [self.dthetamax] * 3)
        self.xmin = np.array([self.thetamin] * 3 + [-self.dthetamax] * 3)
        self.umax = np.full(3, self.Cmax)
        self.umin = -self.umax
        self.xmax_e, self.xmin_e = self.xmax.copy(), self.xmin.copy()
        self.xmax_e[3:] = self.xmin_e[3:] = 0.0         # :210-216 zero final velocity
        # ACADOS' cost_scaling: stage costs times the time step in current releases, 1 in older ones - unpinned; the
        # choice matters for the step's trajectory, not for the QP's feasibility (the label)
        self.cost_scale = self.time_step if cost_scale is None else float(cost_scale)
        self.lm = 0.0                                   # ACADOS default levenberg_marquardt
        self.qp_iter_max = 50                           # ACADOS default qp_solver_iter_max


class _OcpSolver:
    """The accessors the AL driver uses after compute_problem: get(i, 'x' | 'u')."""

    def __init__(self):
        self.x = self.u = None
        self.status = None

    def get(self, i, field):
        return np.copy(self.x[i] if field == "x" else self.u[i])

    def get_status(self):
        return self.status


class OCPtriplependulumINIT:
    """AL's OCPtriplependulumINIT (AL/triplependulum_class_al.py:204-222) on the batched GPU solver: compute_problem
    (q0, v0) -> 1 / 0 / 2 and ocp_solver.get(i, 'x') of the step (vboc_al_solve_batch); compute_problem_batch for
    many states at once."""

    def __init__(self, device=0, cost_scale=None):
        from .lib import Solver
        self.spec = AlSpec(cost_scale)
        s = self.spec
        self.N, self.nx, self.nu = s.N, s.nx, s.nu
        self.Tf, self.Cmax, self.thetamax, self.thetamin, self.dthetamax = (s.Tf, s.Cmax, s.thetamax, s.thetamin,
                                                                            s.dthetamax)
        self.device = device
        self.solver = Solver(3, self.N, device=device)
        self.solver.set_option("levenberg_marquardt", s.lm)
        self.solver.set_option("qp_solver_iter_max", s.qp_iter_max)
        self.solver.set_option("nlp_solver_tol_stat", 1e-6)    # ACADOS defaults (the class sets no tolerance)
        self.solver.set_option("qp_solver_tol_stat", 1e-8)
        self.ocp_solver = _OcpSolver()

    def compute_problem_batch(self, x0):
        """compute_problem for every row of x0 [B, 6] (numpy): dict(label, status, x [B, N+1, 6], u [B, N, 3],
        qp_iter) as numpy arrays."""
        import torch
        dev = torch.device("cuda", self.device)
        t = torch.as_tensor(np.ascontiguousarray(x0, dtype=np.float64), device=dev)
        out = self.solver.al_solve_device(self.spec, t)
        torch.cuda.synchronize(dev)
        return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}

    def labels(self, X):
        """(labels [B], trajectories [B, N+1, 6]) of compute_problem for every state of X: testing_batch's label_fn."""
        r = self.compute_problem_batch(X)
        return r["label"], r["x"]

    def compute_problem(self, q0, v0):
        x0 = np.array([q0[0], q0[1], q0[2], v0[0], v0[1], v0[2]], dtype=np.float64)   # :152
        r = self.compute_problem_batch(x0[None])
        self.ocp_solver.x, self.ocp_solver.u, self.ocp_solver.status = r["x"][0], r["u"][0], int(r["status"][0])
        return int(r["label"][0])

    def compute_problem_nnguess_batch(self, x0, model, mean, std):
        """compute_problem_nnguess (:171-201) for every row of x0 [B, 6]: the guess network's trajectory as every
        stage's x guess (nn_guess), then the same RTI step.  Returns the dict of compute_problem_batch."""
        import torch
        x0 = np.ascontiguousarray(x0, dtype=np.float64)
        xg = np.stack([nn_guess(self.N, s[:3], s[3:], model, mean, std) for s in x0]) if len(x0) else \
            np.zeros((0, self.N + 1, 6))
        dev = torch.device("cuda", self.device)
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)
        out = self.solver.al_solve_device(self.spec, T(x0), x_guess=T(xg))
        torch.cuda.synchronize(dev)
        return {k: v.cpu().numpy() for k, v in out.items() if not k.startswith("_")}

    def compute_problem_nnguess(self, q0, v0, model, mean, std):
        x0 = np.array([q0[0], q0[1], q0[2], v0[0], v0[1], v0[2]], dtype=np.float64)   # :175
        r = self.compute_problem_nnguess_batch(x0[None], model, mean, std)
        self.ocp_solver.x, self.ocp_solver.u, self.ocp_solver.status = r["x"][0], r["u"][0], int(r["status"][0])
        return int(r["label"][0])

    def labels_nnguess(self, model, mean, std):
        """testing_batch's label_fn for the driver's testing_guess (AL/triplependulum_al.py:44-62)."""
        def fn(X):
            r = self.compute_problem_nnguess_batch(X, model, mean, std)
            return r["label"], r["x"]
        return fn


def nn_guess(N, q0, v0, model, mean, std):
    """The stage guesses of compute_problem_nnguess (AL/triplependulum_class_al.py:180-192): the guess network
    (NeuralNetCLS(6, 500, 6 N), FP32) evaluated on the normalised state exactly as the reference does it - one [1, 6]
    float32 tensor, (x - mean) / std, model, * std + mean, reshaped to [N, 6] - and x0 at stage 0.  Evaluated on the
    model's device (the reference's is the CPU, where the FP32 arithmetic is the reference's own)."""
    import torch
    dev = next(model.parameters()).device
    with torch.no_grad():
        inp = torch.Tensor([[q0[0], q0[1], q0[2], v0[0], v0[1], v0[2]]]).to(dev)
        inp = (inp - mean) / std
        out = model(inp)
        out = out * std + mean
        out = out.cpu().numpy()
    out = np.reshape(out, (N, 6))
    xg = np.empty((N + 1, 6))
    xg[0] = [q0[0], q0[1], q0[2], v0[0], v0[1], v0[2]]
    xg[1:] = out
    return xg


def out_of_bounds(spec, s0):
    """testing's pre-check (AL/triplependulum_al.py:27): a position outside [thetamin, thetamax] or a velocity outside
    [-dthetamax, dthetamax] on any joint."""
    q0, v0 = s0[:3], s0[3:]
    q_min, q_max, v_min, v_max = spec.thetamin, spec.thetamax, -spec.dthetamax, spec.dthetamax
    return any(q0[j] < q_min or q0[j] > q_max or v0[j] < v_min or v0[j] > v_max for j in range(3))


def testing_batch(spec, S0, label_fn):
    """The AL driver's testing(s0) (AL/triplependulum_al.py:24-42) for every state of S0 [B, 6] at once:
    label_fn(x0 [b, 6]) -> (labels [b], x [b, N+1, 6]) solves the in-bounds states in one batch (compute_problem).
    Returns the list of testing's return values: ([q0, v0, 1, 0], None) for an out-of-bounds state or label 0,
    ([q0, v0, 0, 1], trajectory list of (N+1)*6) for label 1, and None for label 2 (testing falls off its if/elif)."""
    S0 = np.asarray(S0, dtype=np.float64)
    out = [None] * S0.shape[0]
    run = []
    for b, s0 in enumerate(S0):
        if out_of_bounds(spec, s0):
            out[b] = ([*map(float, s0), 1, 0], None)
        else:
            run.append(b)
    if run:
        labels, X = label_fn(S0[run])
        for j, b in enumerate(run):
            s0 = S0[b]
            if labels[j] == 1:
                out[b] = ([*map(float, s0), 0, 1], np.reshape(X[j], ((spec.N + 1) * 6,)).tolist())
            elif labels[j] == 0:
                out[b] = ([*map(float, s0), 1, 0], None)
    return out


def unlabeled_states(spec, n, rng):
    """Samples in the driver's unlabeled box (AL/triplependulum_al.py:115-123): positions in [thetamin, thetamax],
    velocities in [-dthetamax, dthetamax] widened by 1/20 of the range on each side, uniform."""
    v_min, v_max = -spec.dthetamax, spec.dthetamax
    lo = [spec.thetamin] * 3 + [v_min - (v_max - v_min) / 20] * 3
    hi = [spec.thetamax] * 3 + [v_max + (v_max - v_min) / 20] * 3
    return rng.uniform(low=lo, high=hi, size=(n, 6))
