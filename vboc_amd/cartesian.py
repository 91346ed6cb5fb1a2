"""Drop-in replacement for the Cartesian-constraint double pendulum
(VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py): `OCPdoublependulumINIT` and
`SYMdoublependulumINIT` with the interface of that module, so `vboc_multiprocessing.py` only changes its import
(`from vboc_amd.cartesian import OCPdoublependulumINIT, SYMdoublependulumINIT`).

The OCP is the double pendulum's boundary OCP (VBOC/doublependulum_class_vboc.py, identical model, cost,
bounds and solver options) plus the nonlinear path constraint of :154-160,
    lh = radius^2 <= (l1 sin th1 + l2 sin th2 - x_c)^2 + (l1 cos th1 + l2 cos th2 - y_c)^2 <= uh = 1e6,
radius = l2 / 4, (x_c, y_c) = (0, -l1 - l2 / 2): the end effector stays out of a circle below the pivot.
The solver handle carries it (vboc_set_path_constraint); each OCP_solve is a batch-of-one call.
"""
from types import SimpleNamespace

import numpy as np

from . import ocp as _ocp
from .systems import cartesian_constraint


class _CartSolver(_ocp.OcpSolver):
    def __init__(self, ocp_def, constraint):
        self._hc = constraint
        super().__init__(ocp_def)

    def _bind(self):
        return _ocp._shared_solver(self.nq, self.NMAX, self._hc)


class OCPdoublependulum(_ocp.OCPdoublependulum):
    def __init__(self):
        super().__init__()
        c = cartesian_constraint()
        self.radius = self.l2 / 4
        self.x_c = c.x_c
        self.y_c = c.y_c
        self.ocp.constraints.lh = np.array([c.lh])
        self.ocp.constraints.uh = np.array([c.uh])
        self.ocp.constraints.C = np.zeros((2, 5))
        self.ocp.constraints.D = np.zeros((2, 2))
        self.ocp.model = SimpleNamespace(con_h_expr="(l1 sin th1 + l2 sin th2 - x_c)^2 + (l1 cos th1 + l2 cos th2 - y_c)^2")
        self.constraint = c


class OCPdoublependulumINIT(_ocp._InitBase):
    """OCP_solve(x_sol_guess, u_sol_guess, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb, q_fin_ub)
    -> status, as in :184-219; the solver sees the keep-out circle on every solve."""

    def __init__(self):
        base = OCPdoublependulum()
        self.__dict__.update({k: v for k, v in base.__dict__.items()})
        self.Cmax = base.Cmax
        self.ocp_solver = _CartSolver(self, base.constraint)


class SYMdoublependulumINIT(_ocp.SYMdoublependulumINIT):
    """The twin integrator (:222-308): the unconstrained double pendulum model."""
