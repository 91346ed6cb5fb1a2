"""ORACLE - TEST INFRASTRUCTURE ONLY.

ctypes binding of the plain-C FP64 restatement (oracle/vboc_oracle.c).  Importable by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg only; the product package vboc_amd never
imports it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("VBOC_ORACLE_LIB") or os.path.join(HERE, "libvboc_oracle.so")   # tools/oracle_asan.sh: the ASan build


class Opts(ctypes.Structure):
    _fields_ = [("tol_stat", ctypes.c_double), ("tol_eq", ctypes.c_double),
                ("tol_ineq", ctypes.c_double), ("tol_comp", ctypes.c_double),
                ("max_iter", ctypes.c_int), ("qp_max_iter", ctypes.c_int),
                ("alpha_min", ctypes.c_double), ("alpha_reduction", ctypes.c_double),
                ("lm", ctypes.c_double), ("mu0", ctypes.c_double), ("ipm_push", ctypes.c_double),
                ("ipm_tau", ctypes.c_double), ("qp_tol_stat", ctypes.c_double),
                ("qp_tol_eq", ctypes.c_double), ("qp_tol_comp", ctypes.c_double),
                ("hc", ctypes.c_int), ("hc_xc", ctypes.c_double), ("hc_yc", ctypes.c_double),
                ("hc_lh", ctypes.c_double), ("hc_uh", ctypes.c_double)]


RESULT_DTYPE = np.dtype([("status", "i4"), ("sqp_iter", "i4"), ("qp_iter", "i4"), ("pad", "i4"),
                         ("cost", "f8"), ("res_stat", "f8"), ("res_eq", "f8"), ("res_ineq", "f8"),
                         ("res_comp", "f8")])

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        _lib.vboc_oracle_solve_batch.restype = ctypes.c_int
    return _lib


def default_opts(**kw):
    o = Opts()
    lib().vboc_oracle_default_opts(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def model(nq, th, om, u):
    th, om, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (th, om, u))
    acc = np.zeros(nq)
    Jth, Jom, Ju = np.zeros((nq, nq)), np.zeros((nq, nq)), np.zeros((nq, nq))
    lib().vboc_oracle_model(nq, _p(th), _p(om), _p(u), _p(acc), _p(Jth), _p(Jom), _p(Ju))
    return acc, Jth, Jom, Ju


def rk4(nq, h, x, u):
    x, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, u))
    x1 = np.zeros(2 * nq)
    lib().vboc_oracle_rk4(nq, ctypes.c_double(h), _p(x), _p(u), _p(x1))
    return x1


def rk4_sens(nq, h, x, u):
    x, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, u))
    x1, A, B = np.zeros(2 * nq), np.zeros((2 * nq, 2 * nq)), np.zeros((2 * nq, nq))
    lib().vboc_oracle_rk4_sens(nq, ctypes.c_double(h), _p(x), _p(u), _p(x1), _p(A), _p(B))
    return x1, A, B


def ft_rk4_sens(nq, x, u):
    """Shooting map of the free-time model (x = [q, v, dt]) and its Jacobians (vboc_oracle_ft.c)."""
    x, u = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, u))
    nx = 2 * nq + 1
    x1, A, B = np.zeros(nx), np.zeros((nx, nx)), np.zeros((nx, nq))
    lib().vboc_oracle_ft_rk4_sens(nq, _p(x), _p(u), _p(x1), _p(A), _p(B))
    return x1, A, B


def solve_batch(nq, N, x_guess, u_guess, p, lbx, ubx, lbu, ubu, lbx0, ubx0, lbxe, ubxe,
                opts=None, nthreads=None, free_time=False):
    """Problem-major batch in the reference layout (see vboc_oracle.c).  Returns
    (x_out, u_out, results).  free_time: the free-time box OCP of vboc_oracle_ft.c
    (OCPpendulum.OCP_solve); an unsupported structure there gives status 5."""
    N = np.ascontiguousarray(N, dtype=np.int32)
    B = N.shape[0]
    arrs = [np.ascontiguousarray(a, dtype=np.float64)
            for a in (x_guess, u_guess, p, lbx, ubx, lbu, ubu, lbx0, ubx0, lbxe, ubxe)]
    Nmax = arrs[0].shape[1] - 1
    assert arrs[1].shape[1] == Nmax
    x_out = np.zeros_like(arrs[0])
    u_out = np.zeros_like(arrs[1])
    res = np.zeros(B, dtype=RESULT_DTYPE)
    # the UR5 OCP sets levenberg_marquardt = 1e-2 (VBOC/UR5/ur5reduced_class_fixedveldir.py:135)
    o = opts if opts is not None else default_opts(**({"lm": 1e-2} if nq == 4 else {}))
    nthreads = nthreads or os.cpu_count()
    fn = lib().vboc_oracle_ft_solve_batch if free_time else lib().vboc_oracle_solve_batch
    rc = fn(nq, B, Nmax, _p(N), *[_p(a) for a in arrs], ctypes.byref(o),
                                       int(nthreads), _p(x_out), _p(u_out), _p(res))
    if rc != 0:
        raise RuntimeError(f"oracle solve_batch failed rc={rc}")
    return x_out, u_out, res


def solve_mult(nq, b, i, opts=None):
    """Problem i of batch b (ics.Batch layout) with the NLP multipliers at the final iterate
    (vboc_oracle_solve_mult): returns dict(x [N+1, 2nq], u [N, nq], status, cost, res_stat, pi [N, 2nq],
    lam_l / lam_u [N+1, 3nq] in the stage layout z_0 = (s, u_0), z_k = (x_k, u_k), z_N = x_N, nu [nq], s)."""
    N = int(b["N"][i])
    nx, nz, nxr = 2 * nq, 3 * nq, 2 * nq + 1
    arrs = [np.ascontiguousarray(b[k][i], dtype=np.float64) for k in
            ("x_guess", "u_guess", "p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")]
    x_out, u_out = np.zeros((N + 1, nxr)), np.zeros((N, nq))
    row = nx + 2 * nz
    mult = np.zeros((N + 1) * row + nq + 1)
    res = np.zeros(1, dtype=RESULT_DTYPE)
    o = opts if opts is not None else default_opts(**({"lm": 1e-2} if nq == 4 else {}))
    rc = lib().vboc_oracle_solve_mult(nq, N, *[_p(a) for a in arrs], ctypes.byref(o), _p(x_out), _p(u_out),
                                      _p(res), _p(mult))
    if rc != 0:
        raise RuntimeError(f"oracle solve_mult failed rc={rc}")
    m = mult[:(N + 1) * row].reshape(N + 1, row)
    return dict(x=x_out[:, :nx], u=u_out, status=int(res["status"][0]), cost=float(res["cost"][0]),
                res_stat=float(res["res_stat"][0]), sqp_iter=int(res["sqp_iter"][0]), pi=m[:N, :nx],
                lam_l=m[:, nx:nx + nz], lam_u=m[:, nx + nz:], nu=mult[(N + 1) * row:(N + 1) * row + nq],
                s=float(mult[(N + 1) * row + nq]))


def hjr_solve_batch(nq, x0, weights, mean, std, u_max=None, opts=None, nthreads=None):
    """The HJR one-step OCP (compute_problem of HJR/<sys>_hjr_class.py) for every row of x0 [B, 2nq]
    (vboc_oracle_hjr.c).  weights: the NeuralNetCLS parameters in model.parameters() order (W0, b0, W1, b1, W2,
    b2).  Returns dict(status, cost, sqp_iter, qp_iter, res_stat, u [B, nq], x1 [B, 2nq], pi, lam_l, lam_u)."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B = x0.shape[0]
    W = [np.ascontiguousarray(np.asarray(w, dtype=np.float64)) for w in weights]
    h = W[0].shape[0]
    if opts is None:
        opts = Opts()
        lib().vboc_oracle_hjr_default_opts(nq, ctypes.byref(opts))
    u_max = float(u_max if u_max is not None else (3.0 if nq == 1 else 10.0))
    u, x1 = np.zeros((B, nq)), np.zeros((B, 2 * nq))
    mult = np.zeros((B, 2 * nq + 2 * nq))
    res = np.zeros(B, dtype=RESULT_DTYPE)
    rc = lib().vboc_oracle_hjr_solve_batch(nq, B, _p(x0), h, *[_p(w) for w in W], ctypes.c_double(mean),
                                           ctypes.c_double(std), ctypes.c_double(u_max), ctypes.byref(opts),
                                           int(nthreads or os.cpu_count()), _p(u), _p(x1), _p(mult), _p(res))
    if rc != 0:
        raise RuntimeError(f"oracle hjr_solve_batch failed rc={rc}")
    nx = 2 * nq
    return dict(status=np.array(res["status"]), cost=np.array(res["cost"]), sqp_iter=np.array(res["sqp_iter"]),
                qp_iter=np.array(res["qp_iter"]), res_stat=np.array(res["res_stat"]), u=u, x1=x1, pi=mult[:, :nx],
                lam_l=mult[:, nx:nx + nq], lam_u=mult[:, nx + nq:])


def cartesian_opts():
    """vboc_opts_t fields of the Cartesian double pendulum's keep-out circle (vboc_amd.systems)."""
    from vboc_amd.systems import cartesian_constraint
    c = cartesian_constraint()
    return dict(hc=1, hc_xc=c.x_c, hc_yc=c.y_c, hc_lh=c.lh, hc_uh=c.uh)


def hc_value(x):
    """h(x) of the keep-out circle for rows x[..., :2] (the chain tip's squared distance to the centre)."""
    from vboc_amd.systems import cartesian_constraint, system
    c, l = cartesian_constraint(), system(2).l
    X = l[0] * np.sin(x[..., 0]) + l[1] * np.sin(x[..., 1])
    Y = l[0] * np.cos(x[..., 0]) + l[1] * np.cos(x[..., 1])
    return (X - c.x_c) ** 2 + (Y - c.y_c) ** 2


def data_generation(nq, ids, N_start=None, seed=None, fail_mod=0, nthreads=None):
    """The reference's data_generation(v) for every problem id (vboc_dg.c: the C restatement, one problem per
    OpenMP thread, the oracle as solver and twin integrator).  Returns (results, stats) in the format of
    vboc_amd.drivers.data_generation_batch: results[i] = list of saved rows or None (triple), the 3-tuple
    (samples | None, ic | None, ic | None) (double); stats = dict(solves, rk4, sqp_iter, per_problem [B, 3])."""
    from vboc_amd.ics import SEED
    from vboc_amd.systems import system
    sd = system(nq)
    N_start = int(N_start or sd.N)
    seed = SEED if seed is None else int(seed)
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    B, nx = ids.shape[0], 2 * nq
    max_rows = 2 * (N_start + 16) + 2
    m = (list(sd.m) + [0.0, 0.0])[:2]
    l = (list(sd.l) + [0.0, 0.0])[:2]
    params = np.array([sd.q_min, sd.q_max, sd.v_max, sd.u_max, sd.dt, sd.tol, sd.eps, sd.g, l[0], l[1], m[0], m[1]])
    rows = np.zeros((B, max_rows, nx))
    cnt = np.zeros(B, np.int32)
    ic = np.zeros((B, 4))
    slot = np.zeros(B, np.int32)
    st = np.zeros((B, 3), np.int64)
    rc = lib().vboc_oracle_data_generation(nq, B, _p(ids), ctypes.c_ulonglong(seed), N_start, _p(params), int(fail_mod),
                                          int(nthreads or os.cpu_count()), max_rows, _p(rows), _p(cnt), _p(ic),
                                          _p(slot), _p(st))
    if rc != 0 or (cnt > max_rows).any():
        raise RuntimeError(f"oracle data_generation failed rc={rc}")
    results = []
    for b in range(B):
        samples = None if cnt[b] < 0 else [r.tolist() for r in rows[b, :cnt[b]]]
        if nq == 2:
            icb = [int(ic[b, 0])] + ic[b, 1:].tolist()
            results.append((samples, icb, None) if slot[b] == 1 else (None, None, icb))
        else:
            results.append(samples)
    return results, dict(solves=int(st[:, 0].sum()), rk4=int(st[:, 1].sum()), sqp_iter=int(st[:, 2].sum()),
                         per_problem=st)


class DriverBackend:
    """The oracle behind the batched drivers' backend interface (vboc_amd.drivers: solve(batch),
    rk4(x, u, T)) - the CPU baseline of bench.py's dg-loop leg and the tests' reference runs."""
    nmax = 512

    def __init__(self, nq, nthreads=None, **opts):
        """opts: vboc_opts_t fields, e.g. the Cartesian keep-out circle (cartesian_opts())."""
        self.nq, self.nthreads = nq, nthreads
        self.opts = opts

    def solve(self, b, free_time=False):
        o = default_opts(**self.opts) if self.opts else None
        xo, uo, r = solve_batch(self.nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], opts=o, nthreads=self.nthreads,
                                free_time=free_time)
        return dict(status=np.array(r["status"]), x=xo, u=uo, cost=np.array(r["cost"]),
                    sqp_iter=np.array(r["sqp_iter"]), qp_iter=np.array(r["qp_iter"]))

    def rk4(self, x, u, T):
        return np.stack([rk4(self.nq, T, x[i], u[i]) for i in range(x.shape[0])])


class MpcNN(ctypes.Structure):
    """vboc_mpc_nn_t (vboc_oracle.h): the terminal row's network."""
    _fields_ = [("hid", ctypes.c_int)] + [(n, ctypes.c_void_p) for n in ("W0", "b0", "W1", "b1", "W2", "b2")] + \
               [(n, ctypes.c_double) for n in ("mean", "std", "lh", "uh")]


def mpc_solve_batch(spec, x0, x_guess, u_guess, params=None, mean=0.0, std=1.0, rti=False, opts=None,
                    nthreads=None, lh=0.0, uh=1e6):
    """The Safe-MPC OCP_solve (vboc_oracle_ft.c vboc_oracle_mpc_solve) for every row of x0 [B, 6]: spec a
    vboc_amd.safempc.MpcSpec, guesses [B, N+1, 6] / [B, N, 3], params the NeuralNetDIR weights (float64, None = no
    terminal row).  Returns (x, u, results, h(x_N))."""
    x0, xg, ug = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, x_guess, u_guess))
    B, N = x0.shape[0], spec.N
    assert xg.shape == (B, N + 1, 6) and ug.shape == (B, N, 3)
    x_out, u_out = np.zeros_like(xg), np.zeros_like(ug)
    res = np.zeros(B, dtype=RESULT_DTYPE)
    hrow = np.zeros(B)
    if opts is None:
        opts = default_opts(lm=spec.lm, tol_stat=1e-6, qp_tol_stat=1e-8)
    vec = [np.ascontiguousarray(a, dtype=np.float64) for a in
           (spec.xmin, spec.xmax, spec.umin, spec.umax, spec.xmin, spec.xmax, spec.W, spec.W_e, spec.yref, spec.yref_e)]
    nnp = None
    keep = None
    if params is not None:
        keep = [np.ascontiguousarray(p, dtype=np.float64) for p in params]
        nnp = MpcNN(hid=keep[0].shape[0], mean=float(mean), std=float(std), lh=float(lh), uh=float(uh),
                    **{n: p.ctypes.data for n, p in zip(("W0", "b0", "W1", "b1", "W2", "b2"), keep)})
    rc = lib().vboc_oracle_mpc_solve_batch(3, B, N, ctypes.c_double(spec.time_step), _p(x0), _p(xg), _p(ug),
                                           *[_p(a) for a in vec], ctypes.c_double(spec.cost_scale),
                                           ctypes.byref(nnp) if nnp is not None else None, int(bool(rti)),
                                           ctypes.byref(opts), int(nthreads or os.cpu_count()), _p(x_out), _p(u_out),
                                           _p(res), _p(hrow))
    if rc != 0:
        raise RuntimeError(f"oracle mpc_solve_batch failed rc={rc}")
    del keep
    return x_out, u_out, res, hrow


def _mpc_nn(params, mean, std, lh=0.0, uh=1e6):
    keep = [np.ascontiguousarray(p, dtype=np.float64) for p in params]
    return MpcNN(hid=keep[0].shape[0], mean=float(mean), std=float(std), lh=float(lh), uh=float(uh),
                 **{n: p.ctypes.data for n, p in zip(("W0", "b0", "W1", "b1", "W2", "b2"), keep)}), keep


def mpc_soft_solve_batch(spec, x0, x_guess, u_guess, params, mean, std, margin, Zl, zl=None, W=None, We=None,
                         rti=True, opts=None, nthreads=None, lh=0.0, uh=1e6):
    """OCPtriplependulumSoftTraj's OCP_solve (vboc_oracle_ft.c vboc_oracle_mpc_soft_solve_batch): the row
    NN(x) (100 - margin) / 100 - vn(x) on every stage, soft lower sides with the per-problem per-stage weights Zl / zl
    [B, N+1]; W [B, 9] / We [B, 6] per-problem stage weights (default: the spec's).  Returns (x, u, results, h(x_N))."""
    x0, xg, ug = (np.ascontiguousarray(a, dtype=np.float64) for a in (x0, x_guess, u_guess))
    B, N = x0.shape[0], spec.N
    assert xg.shape == (B, N + 1, 6) and ug.shape == (B, N, 3)
    Zl = np.ascontiguousarray(np.broadcast_to(np.asarray(Zl, dtype=np.float64), (B, N + 1)))
    zl = np.zeros((B, N + 1)) if zl is None else np.ascontiguousarray(np.broadcast_to(np.asarray(zl, float), (B, N + 1)))
    W = np.ascontiguousarray(np.broadcast_to(np.asarray(spec.W if W is None else W, float), (B, 9)))
    We = np.ascontiguousarray(np.broadcast_to(np.asarray(spec.W_e if We is None else We, float), (B, 6)))
    x_out, u_out = np.zeros_like(xg), np.zeros_like(ug)
    res = np.zeros(B, dtype=RESULT_DTYPE)
    hrow = np.zeros(B)
    if opts is None:
        opts = default_opts(lm=spec.lm, tol_stat=1e-6, qp_tol_stat=1e-8)
    vec = [np.ascontiguousarray(a, dtype=np.float64) for a in (spec.xmin, spec.xmax, spec.umin, spec.umax, spec.xmin,
                                                               spec.xmax)]
    nnp, keep = _mpc_nn(params, mean, std, lh, uh)
    rc = lib().vboc_oracle_mpc_soft_solve_batch(
        3, B, N, ctypes.c_double(spec.time_step), _p(x0), _p(xg), _p(ug), *[_p(a) for a in vec], _p(W), _p(We),
        _p(np.ascontiguousarray(spec.yref, dtype=np.float64)), _p(np.ascontiguousarray(spec.yref_e, dtype=np.float64)),
        ctypes.c_double(spec.cost_scale), ctypes.byref(nnp), ctypes.c_double(float(margin)), _p(zl), _p(Zl),
        int(bool(rti)), ctypes.byref(opts), int(nthreads or os.cpu_count()), _p(x_out), _p(u_out), _p(res), _p(hrow))
    if rc != 0:
        raise RuntimeError(f"oracle mpc_soft_solve_batch failed rc={rc}")
    del keep
    return x_out, u_out, res, hrow


def mpc_row(x, params, mean, std, margin=-1.0):
    """The Safe-MPC row at states x [B, 6] (vboc_oracle_mpc_row): margin >= 0 the SoftTraj (conservative) row."""
    x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float64)
    out = np.zeros(x.shape[0])
    nnp, keep = _mpc_nn(params, mean, std)
    lib().vboc_oracle_mpc_row(3, x.shape[0], _p(x), ctypes.byref(nnp), ctypes.c_double(float(margin)), _p(out))
    del keep
    return out


def al_solve_batch(spec, x0, x_guess=None, opts=None, nthreads=None):
    """AL's compute_problem (vboc_oracle_ft.c vboc_oracle_al_solve_batch) for every row of x0 [B, 6]: spec a
    vboc_amd.al.AlSpec; x_guess [B, N+1, 6] (optional): compute_problem_nnguess's stage guesses.  Returns
    dict(label, status, qp_iter, x [B, N+1, 6], u [B, N, 3])."""
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    B, N = x0.shape[0], spec.N
    xg = None if x_guess is None else np.ascontiguousarray(x_guess, dtype=np.float64)
    assert xg is None or xg.shape == (B, N + 1, 6)
    x_out, u_out = np.zeros((B, N + 1, 6)), np.zeros((B, N, 3))
    res = np.zeros(B, dtype=RESULT_DTYPE)
    label = np.zeros(B, np.int32)
    if opts is None:
        opts = default_opts(lm=spec.lm, tol_stat=1e-6, qp_tol_stat=1e-8, qp_max_iter=spec.qp_iter_max)
    vec = [np.ascontiguousarray(a, dtype=np.float64) for a in
           (spec.xmin, spec.xmax, spec.umin, spec.umax, spec.xmin_e, spec.xmax_e, spec.W, spec.W_e)]
    rc = lib().vboc_oracle_al_solve_batch(3, B, N, ctypes.c_double(spec.time_step), _p(x0),
                                          _p(xg) if xg is not None else None, *[_p(a) for a in vec],
                                          ctypes.c_double(spec.cost_scale), ctypes.byref(opts),
                                          int(nthreads or os.cpu_count()), _p(x_out), _p(u_out), _p(res), _p(label))
    if rc != 0:
        raise RuntimeError(f"oracle al_solve_batch failed rc={rc}")
    return dict(label=label, status=np.array(res["status"]), qp_iter=np.array(res["qp_iter"]), x=x_out, u=u_out)
