"""Drop-in replacements for the reference's OCP classes, backed by the HIP solver.

Reference interface (kept verbatim so the reference drivers run unchanged):
  OCPtriplependulum / OCPtriplependulumINIT / SYMtriplependulumINIT
      VBOC/triplependulum_class_vboc.py:7-239
  OCPdoublependulum / OCPdoublependulumINIT / SYMdoublependulumINIT
      VBOC/doublependulum_class_vboc.py:6-304
  OCPpendulum (solver built in the constructor) VBOC/pendulum_class_vboc.py:6-130

Attributes the drivers read: .N (mutable), .ocp.dims.nx/nu/N, .ocp.solver_options.*,
.thetamax/.thetamin/.dthetamax/.Cmax (.Fmax for the pendulum), .g/.l1/.m1...; methods
.OCP_solve(...) -> status and .ocp_solver with the AcadosOcpSolver subset the drivers call
(reset, set, get, constraints_set, solve, get_cost, get_stats, set_new_time_steps,
update_qp_solver_cond_N - SURVEY.md section 8b).  `SYM<sys>INIT().acados_integrator` offers
set('x'|'u'|'T'), solve(), get('x') of AcadosSimSolver.

Each solve() is a batch-of-one call of the C ABI (vboc_solve_batch_host); the batched drivers
(vboc_amd.drivers) call the library directly with whole batches.  Structures outside what the
boundary-OCP solver implements raise NotImplementedError (loudly - no silent fallback).
"""
from types import SimpleNamespace

import numpy as np

from . import lib
from .systems import system

_SOLVERS = {}
_BACKEND = None


def use_backend(backend):
    """Test hook: route subsequently created solvers / integrators through `backend` (an object with
    solve_host(batch) -> dict and rk4(nq, T, x, u) -> x1), e.g. the CPU oracle in tests/.  None (the
    default) = the HIP library; there is no automatic fallback."""
    global _BACKEND
    _BACKEND = backend


def _shared_solver(nq, nmax, path_constraint=None):
    """One HIP handle per (nq, nmax, path constraint) per process (the reference builds one solver per
    process).  path_constraint: systems.CartesianConstraint of the Cartesian double pendulum, or None."""
    if _BACKEND is not None:
        return _BACKEND if path_constraint is None else _BACKEND.with_path_constraint(path_constraint)
    key = (nq, nmax, path_constraint)
    if key not in _SOLVERS:
        s = lib.Solver(nq, nmax, slots=256)
        if path_constraint is not None:
            s.set_path_constraint(path_constraint)
        _SOLVERS[key] = s
    return _SOLVERS[key]


class SolverOptions(SimpleNamespace):
    pass


def _solver_options(N):
    # VBOC/triplependulum_class_vboc.py:129-141 (identical in the double / pendulum classes)
    return SolverOptions(tf=N, nlp_solver_type="SQP", hessian_approx="EXACT", exact_hess_constr=0,
                         exact_hess_dyn=0, nlp_solver_tol_stat=1e-3, nlp_solver_tol_eq=1e-6,
                         nlp_solver_tol_ineq=1e-6, nlp_solver_tol_comp=1e-6, qp_solver_tol_stat=1e-3,
                         qp_solver_iter_max=100, nlp_solver_max_iter=1000, globalization="MERIT_BACKTRACKING",
                         alpha_reduction=0.3, alpha_min=1e-2, levenberg_marquardt=1e-5,
                         integrator_type="ERK", qp_solver="PARTIAL_CONDENSING_HPIPM")


_OPT_FIELDS = ("nlp_solver_tol_stat", "nlp_solver_tol_eq", "nlp_solver_tol_ineq", "nlp_solver_tol_comp",
               "qp_solver_tol_stat", "qp_solver_iter_max", "nlp_solver_max_iter", "alpha_reduction",
               "alpha_min", "levenberg_marquardt")


class OcpSolver:
    """The AcadosOcpSolver subset used by the VBOC drivers, for one OCP at a time."""

    NMAX = 512   # horizon capacity of the shared handle (drivers extend N from 100 by +1 steps)

    def __init__(self, ocp_def):
        self._def = ocp_def
        self.nq = ocp_def.nq
        self.nx = 2 * self.nq + 1
        self.nu = self.nq
        self.N = ocp_def.ocp.dims.N
        self._lib = self._bind()
        self._stats = dict(sqp_iter=0, qp_iter=0, time_tot=0.0, status=0)
        self.reset()

    def _bind(self):
        return _shared_solver(self.nq, self.NMAX)

    # -- AcadosOcpSolver API ----------------------------------------------------------------------
    def reset(self):
        N, nx, nu = self.N, self.nx, self.nu
        c = self._def.ocp.constraints
        self._x = np.zeros((N + 1, nx))
        self._u = np.zeros((N, nu))
        self._p = np.tile(np.asarray(self._def.ocp.parameter_values, float), (N + 1, 1))
        self._lbx = np.tile(c.lbx, (N + 1, 1))
        self._ubx = np.tile(c.ubx, (N + 1, 1))
        self._lbx[0], self._ubx[0] = c.lbx_0, c.ubx_0
        self._lbx[N], self._ubx[N] = c.lbx_e, c.ubx_e
        self._lbu = np.tile(c.lbu, (N, 1))
        self._ubu = np.tile(c.ubu, (N, 1))
        ng = self.nq if c.C is not None else 0
        self._C = np.zeros((N, ng, nx))
        self._D = np.zeros((N, ng, nu))
        self._lg = np.zeros((N, ng))
        self._ug = np.zeros((N, ng))
        self._x_sol = self._x.copy()
        self._u_sol = self._u.copy()
        self._cost = 0.0

    def set_new_time_steps(self, steps):
        steps = np.asarray(steps, dtype=float)
        if not np.all(steps == 1.0):
            raise NotImplementedError("only unit shooting intervals (tf = N) are supported")
        if len(steps) > self.NMAX:
            raise NotImplementedError(f"horizon {len(steps)} exceeds {self.NMAX}")
        self.N = len(steps)
        self.reset()

    def update_qp_solver_cond_N(self, N):
        # partial condensing with cond_N = N is no condensing: the Riccati sweep needs nothing
        if int(N) != self.N:
            raise ValueError(f"cond_N {N} != N {self.N}")

    def set(self, stage, field, value):
        v = np.asarray(value, dtype=float)
        if field == "x":
            self._x[stage] = v
        elif field == "u":
            self._u[stage] = v
        elif field == "p":
            self._p[stage] = v
        else:
            raise ValueError(f"set: unsupported field '{field}'")

    def constraints_set(self, stage, field, value, api="warn"):
        v = np.asarray(value, dtype=float)
        if field == "lbx":
            self._lbx[stage] = v
        elif field == "ubx":
            self._ubx[stage] = v
        elif field == "lbu":
            self._lbu[stage] = v
        elif field == "ubu":
            self._ubu[stage] = v
        elif field == "C":
            self._C[stage] = v.reshape(self._C.shape[1:])
        elif field == "D":
            self._D[stage] = v.reshape(self._D.shape[1:])
        elif field == "lg":
            self._lg[stage] = v
        elif field == "ug":
            self._ug[stage] = v
        else:
            raise ValueError(f"constraints_set: unsupported field '{field}'")

    def get(self, stage, field):
        if field == "x":
            return self._x_sol[stage].copy()
        if field == "u":
            return self._u_sol[stage].copy()
        raise ValueError(f"get: unsupported field '{field}'")

    def get_cost(self):
        return float(self._cost)

    def get_stats(self, field):
        if field not in self._stats:
            raise ValueError(f"get_stats: unsupported field '{field}'")
        return self._stats[field]

    def solve(self):
        b, free_time = self._pack()
        r = self._lib.solve_host(b, free_time=True) if free_time else self._lib.solve_host(b)
        N = self.N
        self._x_sol = r["x"][0, :N + 1].copy()
        self._u_sol = r["u"][0, :N].copy()
        self._cost = r["cost"][0]
        self._stats.update(sqp_iter=int(r["sqp_iter"][0]), qp_iter=int(r["qp_iter"][0]),
                           status=int(r["status"][0]))
        return int(r["status"][0])

    # -- structure checks + packing into the C-ABI layout -----------------------------------------
    def _pack(self):
        N, nq = self.N, self.nq
        for name, arr, st in (("p", self._p, slice(0, N + 1)), ("lbx", self._lbx, slice(1, N)),
                              ("ubx", self._ubx, slice(1, N)), ("lbu", self._lbu, slice(0, N)),
                              ("ubu", self._ubu, slice(0, N))):
            a = arr[st]
            if len(a) and not np.all(a == a[0]):
                raise NotImplementedError(f"stage-varying '{name}' is not supported by the batched solver")
        if np.any(self._D) or np.any(self._lg) or np.any(self._ug) or np.any(self._C[1:]):
            raise NotImplementedError("general constraints other than the stage-0 direction "
                                      "constraint (I - d d^T) dtheta_0 = 0 are not supported")
        p = self._p[0]
        dt = self._lbx[:, 2 * nq]
        if not (np.all(dt == self._ubx[:, 2 * nq]) and np.all(dt == dt[0])):
            return self._pack_free_time(p), True
        if nq > 1:
            d = p[:nq] / np.linalg.norm(p[:nq])
            Cexp = np.zeros((nq, 2 * nq + 1))
            Cexp[:, nq:2 * nq] = np.eye(nq) - np.outer(p[:nq], p[:nq])
            if np.any(self._C[0]) and not np.allclose(self._C[0], Cexp, atol=1e-12):
                raise NotImplementedError("stage-0 C must be [0 | I - p p^T | 0] with p = params[:nq]")
            if not np.any(self._C[0]) and not np.allclose(d, np.eye(nq)[np.argmax(np.abs(d))]):
                raise NotImplementedError("stage-0 velocity direction constraint is required")
        lbx0, ubx0 = self._lbx[0], self._ubx[0]
        if not np.all(lbx0[:nq] == ubx0[:nq]):
            raise NotImplementedError("stage-0 positions must be fixed (lbx_0 == ubx_0)")
        if not np.all(self._lbx[N, nq:2 * nq] == self._ubx[N, nq:2 * nq]):
            raise NotImplementedError("terminal velocities must be fixed (lbx_e == ubx_e)")
        xg = self._x.copy()
        return dict(N=np.array([N], np.int32), x_guess=xg[None], u_guess=self._u[None].copy(), p=p[None],
                    lbx=self._lbx[1 if N > 1 else 0][None], ubx=self._ubx[1 if N > 1 else 0][None],
                    lbu=self._lbu[0][None], ubu=self._ubu[0][None], lbx0=lbx0[None], ubx0=ubx0[None],
                    lbxe=self._lbx[N][None], ubxe=self._ubx[N][None]), False

    def _pack_free_time(self, p):
        """dt free somewhere: the free-time box OCP (vboc_solve_batch_ft, include/vboc.h) - what
        OCPpendulum.OCP_solve builds (VBOC/pendulum_class_vboc.py:107-130)."""
        N = self.N
        if np.any(self._C):
            raise NotImplementedError("free-time OCPs with a general constraint C are not supported")
        lbx, ubx = self._lbx[1 if N > 1 else 0], self._ubx[1 if N > 1 else 0]
        if N > 1 and not np.all(lbx < ubx):
            raise NotImplementedError("free-time OCP: path bounds must satisfy lb < ub on every component")
        return dict(N=np.array([N], np.int32), x_guess=self._x.copy()[None], u_guess=self._u[None].copy(),
                    p=p[None], lbx=lbx[None], ubx=ubx[None], lbu=self._lbu[0][None], ubu=self._ubu[0][None],
                    lbx0=self._lbx[0][None], ubx0=self._ubx[0][None], lbxe=self._lbx[N][None],
                    ubxe=self._ubx[N][None])


class _Constraints(SimpleNamespace):
    pass


class _OcpDef:
    """Stand-in for AcadosOcp: dims, constraints, solver_options, parameter_values."""

    def __init__(self, nq, N):
        s = system(nq)
        nx, nu = 2 * nq + 1, nq
        self.dims = SimpleNamespace(N=N, nx=nx, nu=nu, np=nq + 1)
        self.solver_options = _solver_options(N)
        self.parameter_values = np.zeros(nq + 1) if nq > 1 else np.array([0.0, 1.0])
        q = [s.q_min] * nq
        Q = [s.q_max] * nq
        v = [s.v_max] * nq
        self.constraints = _Constraints(
            lbu=np.full(nu, -s.u_max), ubu=np.full(nu, s.u_max), idxbu=np.arange(nu),
            lbx=np.r_[q, [-x for x in v], 0.0], ubx=np.r_[Q, v, 1e-2], idxbx=np.arange(nx),
            lbx_e=np.r_[q, [-x for x in v], 0.0], ubx_e=np.r_[Q, v, 0.0 if nq > 1 else 1e-2],
            lbx_0=np.r_[q, [-x for x in v], 0.0], ubx_0=np.r_[Q, v, 0.0 if nq > 1 else 1e-2],
            C=np.zeros((nq, nx)) if nq > 1 else None, D=np.zeros((nq, nu)) if nq > 1 else None,
            lg=np.zeros(nq) if nq > 1 else None, ug=np.zeros(nq) if nq > 1 else None)


class _Base:
    def __init__(self, nq):
        s = system(nq)
        self.nq = nq
        self.N = s.N
        self.g = s.g
        for i, (m, l) in enumerate(zip(s.m, s.l), start=1):
            setattr(self, f"m{i}", m)
            setattr(self, f"l{i}", l)
        self.thetamax = s.q_max
        self.thetamin = s.q_min
        self.dthetamax = s.v_max
        self.ocp = _OcpDef(nq, self.N)


class _InitBase(_Base):
    def __init__(self, nq):
        super().__init__(nq)
        self.ocp_solver = OcpSolver(self)

    def OCP_solve(self, x_sol_guess, u_sol_guess, p, q_lb, q_ub, u_lb, u_ub, q_init_lb, q_init_ub, q_fin_lb,
                  q_fin_ub):
        """Same contract as VBOC/triplependulum_class_vboc.py:155-191 (and the double :183-219)."""
        S = self.ocp_solver
        if S.N != self.N:
            S.set_new_time_steps(np.full((self.N,), 1.0))
        S.reset()
        nq = self.nq
        for i in range(self.N):
            S.set(i, "x", x_sol_guess[i])
            S.set(i, "u", u_sol_guess[i])
            S.set(i, "p", p)
            S.constraints_set(i, "lbx", q_lb)
            S.constraints_set(i, "ubx", q_ub)
            S.constraints_set(i, "lbu", u_lb)
            S.constraints_set(i, "ubu", u_ub)
        C = np.zeros((nq, 2 * nq + 1))
        d = np.asarray(p[:nq], float)
        C[:, nq:2 * nq] = np.eye(nq) - np.outer(d, d)
        S.constraints_set(0, "C", C, api="new")
        S.constraints_set(0, "lbx", q_init_lb)
        S.constraints_set(0, "ubx", q_init_ub)
        S.constraints_set(self.N, "lbx", q_fin_lb)
        S.constraints_set(self.N, "ubx", q_fin_ub)
        S.set(self.N, "x", x_sol_guess[-1])
        S.set(self.N, "p", p)
        return S.solve()


class OCPtriplependulum(_Base):
    def __init__(self):
        super().__init__(3)
        self.Cmax = system(3).u_max


class OCPtriplependulumINIT(_InitBase):
    def __init__(self):
        super().__init__(3)
        self.Cmax = system(3).u_max


class OCPdoublependulum(_Base):
    def __init__(self):
        super().__init__(2)
        self.Cmax = system(2).u_max


class OCPdoublependulumINIT(_InitBase):
    def __init__(self):
        super().__init__(2)
        self.Cmax = system(2).u_max


class OCPpendulum(_Base):
    """VBOC/pendulum_class_vboc.py:6-130 - the solver is built in the constructor."""

    def __init__(self):
        super().__init__(1)
        s = system(1)
        self.m, self.d, self.b = s.m[0], s.l[0], 0.01
        self.Fmax = s.u_max
        self.ocp_solver = OcpSolver(self)

    def OCP_solve(self, x_sol_guess, u_sol_guess, cost_dir, q_lb, q_ub, q_init, q_fin):
        """Same contract as VBOC/pendulum_class_vboc.py:107-130: a free-time OCP (dt a state in
        [0, 1e-2], cost cost_dir * dtheta_0 + sum_k dt_k), solved by vboc_solve_batch_ft."""
        S = self.ocp_solver
        if S.N != self.N:
            S.set_new_time_steps(np.full((self.N,), 1.0))
        S.reset()
        N = self.N
        for i in range(N):
            S.set(i, "x", np.array(x_sol_guess[i]))
            S.set(i, "u", np.array(u_sol_guess[i]))
            S.set(i, "p", np.array([cost_dir, 1.0]))
            S.constraints_set(i, "lbx", q_lb)
            S.constraints_set(i, "ubx", q_ub)
        S.constraints_set(0, "lbx", np.array([q_init, -self.dthetamax, 0.0]))
        S.constraints_set(0, "ubx", np.array([q_init, self.dthetamax, 1e-2]))
        S.constraints_set(N, "lbx", np.array([q_fin, 0.0, 0.0]))
        S.constraints_set(N, "ubx", np.array([q_fin, 0.0, 1e-2]))
        S.set(N, "x", np.array(x_sol_guess[N]))
        S.set(N, "p", np.array([cost_dir, 1.0]))
        return S.solve()


class _Integrator:
    """AcadosSimSolver subset: ERK4, 4 stages, one step (VBOC/triplependulum_class_vboc.py:235-239)."""

    def __init__(self, nq, T=1e-2):
        self.nq = nq
        self.T = T
        self.x = np.zeros(2 * nq)
        self.u = np.zeros(nq)
        self.xo = np.zeros(2 * nq)

    def set(self, field, value):
        if field == "x":
            self.x = np.asarray(value, dtype=float).copy()
        elif field == "u":
            self.u = np.asarray(value, dtype=float).copy()
        elif field == "T":
            self.T = float(value)
        else:
            raise ValueError(f"integrator set: unsupported field '{field}'")

    def solve(self):
        if _BACKEND is not None:
            self.xo = np.asarray(_BACKEND.rk4(self.nq, self.T, self.x, self.u), dtype=float)
        else:
            self.xo = lib.rk4_host(self.nq, self.T, self.x[None], self.u[None])[0]
        return 0

    def get(self, field):
        if field != "x":
            raise ValueError(f"integrator get: unsupported field '{field}'")
        return self.xo.copy()


class SYMtriplependulumINIT(OCPtriplependulum):
    def __init__(self):
        super().__init__()
        self.acados_integrator = _Integrator(3)


class SYMdoublependulumINIT(OCPdoublependulum):
    def __init__(self):
        super().__init__()
        self.acados_integrator = _Integrator(2)
