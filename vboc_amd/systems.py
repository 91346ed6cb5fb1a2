"""Physical constants and box constraints of the reference systems.

  pendulum : VBOC/pendulum_class_vboc.py:14-17 (m, g, d, b), :55-67 (N, Fmax, bounds)
  double   : VBOC/doublependulum_class_vboc.py:14-18, :107-118
  triple   : VBOC/triplependulum_class_vboc.py:15-21, :74, :90-93
Driver constants: dt_sym = 1e-2, tol = nlp_solver_tol_stat = 1e-3, eps = 10 tol
(VBOC/triplependulum_vboc.py:388-393).
"""
from dataclasses import dataclass, field

import numpy as np


@dataclass(frozen=True)
class System:
    nq: int
    name: str
    N: int
    q_min: float
    q_max: float
    v_max: float
    u_max: float
    g: float = 9.81
    m: tuple = ()
    l: tuple = ()
    dt: float = 1e-2
    tol: float = 1e-3
    eps: float = 1e-2
    gravity_guess: bool = False

    @property
    def nx(self):
        return 2 * self.nq + 1   # reference layout: (theta, dtheta, dt)

    @property
    def nu(self):
        return self.nq

    @property
    def np(self):
        return self.nq + 1


_SYS = {
    1: System(1, "pendulum", 50, np.pi - np.pi / 4, np.pi + np.pi / 4, 10.0, 3.0, m=(0.5,), l=(0.3,)),
    2: System(2, "doublependulum", 100, np.pi - np.pi / 4, np.pi + np.pi / 4, 10.0, 10.0,
              m=(0.4, 0.4), l=(0.8, 0.8), gravity_guess=True),
    3: System(3, "triplependulum", 100, np.pi - np.pi / 4, np.pi + np.pi / 4, 10.0, 10.0,
              m=(0.4, 0.4, 0.4), l=(0.8, 0.8, 0.8)),
}


def system(nq):
    return _SYS[int(nq)]


@dataclass(frozen=True)
class CartesianConstraint:
    """End-effector keep-out circle of the Cartesian double pendulum
    (VBOC/Cartesian constraints/doublependulum_class_fixedveldir.py:154-160):
    lh <= (l1 sin th1 + l2 sin th2 - x_c)^2 + (l1 cos th1 + l2 cos th2 - y_c)^2 <= uh on the path stages.
    The constants are evaluated with the reference's expressions (radius = l2/4, y_c = -l1 - l2/2)."""
    x_c: float
    y_c: float
    lh: float
    uh: float


def cartesian_constraint():
    l1, l2 = _SYS[2].l
    radius = l2 / 4
    return CartesianConstraint(x_c=0.0, y_c=-l1 - l2 / 2, lh=radius ** 2, uh=1e6)
