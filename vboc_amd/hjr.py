"""The HJR variant's one-step OCP on the GPU: drop-in copies of the reference's HJR classes and the HJR labelling
step, batched.

Reference: HJR/triplependulum_hjr_class.py (OCPtriplependulum(mean, std, params), compute_problem(x0), :7-152),
HJR/doublependulum_hjr_class.py (compute_problem(x0)), HJR/pendulum_hjr_class.py (compute_problem(q0, v0)); the
labelling function data_generation(v) of HJR/triplependulum_hjr.py:21-40 (its Pool.map over the candidate
states, :161-176).  The OCP: x0 fixed, one ERK4 step of 1e-2 with u0 in the torque box, the terminal cost the
classifier's logit 0 at x1 (NeuralNetCLS, my_nn.py:4-18); the solve runs one problem per GPU lane
(vboc_hjr_solve_batch, csrc/hjr.h).  `compute_problem` keeps the reference's return value (1 iff ACADOS status 0)
and `ocp_solver.get_cost()` / `get(stage, "x" | "u")` read the last solution, so the HJR driver changes only its
import.  `hjr_labels` is the labelling step for a whole candidate set at once.
"""
import numpy as np

from . import lib

# bounds of the HJR classes (HJR/triplependulum_hjr_class.py:84-87; pendulum_hjr_class.py:74-77)
THETA_MIN, THETA_MAX, DTHETA_MAX = -np.pi / 4 + np.pi, np.pi / 4 + np.pi, 10.0
U_MAX = {1: 3.0, 2: 10.0, 3: 10.0}


class _Access:
    """The ocp_solver subset the HJR drivers read after compute_problem."""

    def __init__(self, owner):
        self._o = owner

    def get_cost(self):
        return float(self._o._last["cost"])

    def get_status(self):
        return int(self._o._last["status"])

    def get(self, stage, field):
        last = self._o._last
        if field == "x":
            return np.array(last["x0"] if stage == 0 else last["x1"])
        if field == "u" and stage == 0:
            return np.array(last["u"])
        raise KeyError(f"{field} at stage {stage}")


class _HjrOcp:
    nq = 3

    def __init__(self, mean, std, params, device=0):
        import torch
        self.mean, self.std = float(mean), float(std)
        # SX(param.tolist()) of nn_decisionfunction: the float32 parameters as doubles
        self.weights = [torch.as_tensor(np.asarray(p.detach().cpu().numpy() if hasattr(p, "detach") else p,
                                                   dtype=np.float64), device=f"cuda:{device}") for p in params]
        if len(self.weights) != 6:
            raise ValueError("params: the six tensors of NeuralNetCLS (Linear, ReLU, Linear, ReLU, Linear)")
        self.N = 1
        self.Cmax = U_MAX[self.nq]
        self.thetamax, self.thetamin, self.dthetamax = THETA_MAX, THETA_MIN, DTHETA_MAX
        self.device = device
        self.solver = lib.Solver(self.nq, 1, device=device)
        self.ocp_solver = _Access(self)
        self._last = None

    def compute_problems(self, X0):
        """compute_problem for every row of X0 [B, 2nq] in one launch: returns (labels [B] = 1 iff status 0,
        dict of numpy arrays status, cost, u, x1, sqp_iter, qp_iter)."""
        import torch
        x0 = torch.as_tensor(np.ascontiguousarray(X0, dtype=np.float64).reshape(-1, 2 * self.nq),
                             device=f"cuda:{self.device}")
        out = self.solver.hjr_solve_device(x0, self.weights, self.mean, self.std, self.Cmax)
        out.pop("_keep")
        res = {k: v.cpu().numpy() for k, v in out.items()}
        return (res["status"] == 0).astype(np.int64), res

    def _one(self, x0):
        lab, res = self.compute_problems(np.asarray(x0, dtype=np.float64)[None, :])
        self._last = dict(x0=np.asarray(x0, dtype=np.float64), **{k: v[0] for k, v in res.items()})
        return int(lab[0])


class OCPtriplependulum(_HjrOcp):
    """HJR/triplependulum_hjr_class.py:7-134: compute_problem(x0) -> 1 if the solve succeeded, else 0."""
    nq = 3

    def compute_problem(self, x0):
        return self._one(x0)


class OCPdoublependulum(_HjrOcp):
    """HJR/doublependulum_hjr_class.py: compute_problem(x0)."""
    nq = 2

    def compute_problem(self, x0):
        return self._one(x0)


class OCPpendulum(_HjrOcp):
    """HJR/pendulum_hjr_class.py: compute_problem(q0, v0) (undamped pendulum, force box 3, lm 1e-2)."""
    nq = 1

    def compute_problem(self, q0, v0):
        return self._one(np.array([q0, v0], dtype=np.float64))


def hjr_labels(ocp, Xu_iter, y_pred, q_min=THETA_MIN, q_max=THETA_MAX, v_max=DTHETA_MAX):
    """data_generation(v) of HJR/triplependulum_hjr.py:21-40 for every candidate v at once.  A candidate inside
    the state box that the classifier predicts viable (y_pred == 1) is solved (compute_problem): solved ->
    (x0, [0, 1] if get_cost() < 0 else [1, 0]), not solved -> (None, None); every other candidate -> (x0, [1, 0]).
    Returns the list of (state, output) pairs in candidate order, as the reference's Pool.map does."""
    X = np.asarray(Xu_iter, dtype=np.float64)
    nq = X.shape[1] // 2
    v_min = -v_max
    pos = X[:, :nq]
    vel = X[:, nq:]
    inside = np.all((pos >= q_min) & (pos <= q_max), axis=1) & np.all((vel >= v_min) & (vel <= v_max), axis=1)
    ask = inside & (np.asarray(y_pred) == 1)
    out = [(X[i], [1, 0]) for i in range(X.shape[0])]
    idx = np.flatnonzero(ask)
    if idx.size:
        lab, res = ocp.compute_problems(X[idx])
        for k, i in enumerate(idx):
            if lab[k] == 1:
                out[i] = (X[i], [0, 1] if res["cost"][k] < 0.0 else [1, 0])
            else:
                out[i] = (None, None)
    return out
