"""ctypes binding of libvboc_amd.so (the C ABI declared in include/vboc.h).

The product path: every solve goes through the HIP library.  There is no CPU fallback - if the
library is missing or cannot be loaded, `load()` raises.  PyTorch is used only for device memory
and streams (`solve_device`).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
# VBOC_LIB selects another in-tree build of the same sources (e.g. the phase-profiling build
# libvboc_amd_prof.so made with -DVBOC_COOP_PROF); default: the product library.  Only builds inside this repository
# are accepted (bench.py records `library.variant` when one is used).
LIB_PATH = os.environ.get("VBOC_LIB") or os.path.join(HERE, "libvboc_amd.so")
if os.environ.get("VBOC_LIB") and not os.path.realpath(LIB_PATH).startswith(os.path.realpath(ROOT) + os.sep):
    raise RuntimeError(f"VBOC_LIB={LIB_PATH}: only solver builds inside {ROOT} may replace the product library")
SRC = os.path.join(HERE, "csrc", "vboc_solver.hip")

EXPORTS = ("vboc_create", "vboc_destroy", "vboc_set_option", "vboc_get_option", "vboc_solve_batch",
           "vboc_solve_batch_host", "vboc_solve_batch_ft", "vboc_solve_batch_ft_host", "vboc_rk4_batch", "vboc_rk4_batch_host",
           "vboc_rk4_sens_batch_host", "vboc_last_kernel_ms",
           "vboc_kernel_stats", "vboc_debug_counters", "vboc_data_generation", "vboc_data_generation_async",
           "vboc_data_generation_wait", "vboc_testing", "vboc_testing_test", "vboc_hjr_solve_batch",
           "vboc_set_path_constraint", "vboc_mpc_solve_batch", "vboc_mpc_soft_solve_batch",
           "vboc_al_solve_batch", "vboc_last_error")

STATUS = {0: "success", 1: "nan", 2: "max_iter", 3: "min_step", 4: "qp_failure", 5: "unsupported"}


class VbocError(RuntimeError):
    pass


class Batch(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("nmax", ctypes.c_int), ("N", ctypes.c_void_p),
                ("x_guess", ctypes.c_void_p), ("u_guess", ctypes.c_void_p), ("p", ctypes.c_void_p),
                ("lbx", ctypes.c_void_p), ("ubx", ctypes.c_void_p), ("lbu", ctypes.c_void_p),
                ("ubu", ctypes.c_void_p), ("lbx_0", ctypes.c_void_p), ("ubx_0", ctypes.c_void_p),
                ("lbx_e", ctypes.c_void_p), ("ubx_e", ctypes.c_void_p), ("status", ctypes.c_void_p),
                ("x_out", ctypes.c_void_p), ("u_out", ctypes.c_void_p), ("cost", ctypes.c_void_p),
                ("sqp_iter", ctypes.c_void_p), ("qp_iter", ctypes.c_void_p)]


class DgBatch(ctypes.Structure):
    """vboc_dg_batch_t (include/vboc.h): the device data-generation call."""
    _fields_ = [("B", ctypes.c_int), ("ids", ctypes.c_void_p), ("seed", ctypes.c_ulonglong),
                ("N_start", ctypes.c_int)] + \
               [(n, ctypes.c_double) for n in ("q_min", "q_max", "v_max", "u_max", "dt", "tol", "eps", "g", "l1", "l2",
                                              "m1", "m2")] + \
               [("rows", ctypes.c_void_p), ("rows_cap", ctypes.c_longlong), ("row_off", ctypes.c_void_p),
                ("row_cnt", ctypes.c_void_p), ("ic", ctypes.c_void_p), ("ic_slot", ctypes.c_void_p),
                ("stats", ctypes.c_void_p), ("rows_used", ctypes.c_longlong), ("spec_solves", ctypes.c_longlong),
                ("spec_used", ctypes.c_longlong)]


class HjrBatch(ctypes.Structure):
    """vboc_hjr_batch_t (include/vboc.h): the HJR one-step OCP batch."""
    _fields_ = [("B", ctypes.c_int), ("hidden", ctypes.c_int), ("x0", ctypes.c_void_p)] + \
               [(n, ctypes.c_void_p) for n in ("W0", "b0", "W1", "b1", "W2", "b2")] + \
               [(n, ctypes.c_double) for n in ("mean", "std", "u_max")] + \
               [(n, ctypes.c_void_p) for n in ("status", "cost", "u", "x1", "sqp_iter", "qp_iter")]


class TtBatch(ctypes.Structure):
    """vboc_tt_batch_t (include/vboc.h): the device testing_test call (UR5, Cartesian)."""
    _fields_ = [("B", ctypes.c_int), ("ids", ctypes.c_void_p), ("seed", ctypes.c_ulonglong), ("N_start", ctypes.c_int),
                ("draw_stream", ctypes.c_int), ("tol", ctypes.c_double), ("dt", ctypes.c_double),
                ("xlo", ctypes.c_double * 8), ("xhi", ctypes.c_double * 8), ("ulim", ctypes.c_double * 4),
                ("rows", ctypes.c_void_p), ("row_cnt", ctypes.c_void_p), ("stats", ctypes.c_void_p)]


class MpcBatch(ctypes.Structure):
    """vboc_mpc_batch_t (include/vboc.h): Safe-MPC OCP_solve batch (W, We, yref, yref_e are host arrays)."""
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("rti", ctypes.c_int), ("hidden", ctypes.c_int),
                ("h", ctypes.c_double), ("cost_scale", ctypes.c_double)] + \
               [(n, ctypes.c_void_p) for n in ("x0", "x_guess", "u_guess", "lbx", "ubx", "lbu", "ubu", "lbx_e", "ubx_e",
                                               "W", "We", "yref", "yref_e", "W0", "b0", "W1", "b1", "W2", "b2")] + \
               [(n, ctypes.c_double) for n in ("mean", "std", "lh", "uh")] + \
               [(n, ctypes.c_void_p) for n in ("status", "x_out", "u_out", "cost", "sqp_iter", "qp_iter", "h_out")]


class MpcSoft(ctypes.Structure):
    """vboc_mpc_soft_t (include/vboc.h): OCPtriplependulumSoftTraj's soft rows (device arrays)."""
    _fields_ = [("safety_margin", ctypes.c_double)] + [(n, ctypes.c_void_p) for n in ("Zl", "zl", "W_b", "We_b")]


class AlBatch(ctypes.Structure):
    """vboc_al_batch_t (include/vboc.h): AL compute_problem batch (W, We are host arrays)."""
    _fields_ = [("B", ctypes.c_int), ("N", ctypes.c_int), ("h", ctypes.c_double), ("cost_scale", ctypes.c_double)] + \
               [(n, ctypes.c_void_p) for n in ("x0", "x_guess", "lbx", "ubx", "lbu", "ubu", "lbx_e", "ubx_e", "W", "We",
                                               "label", "status", "x_out", "u_out", "qp_iter")]


# per problem (vboc_dg_batch_t.stats); t0 / t1: the problem's start / end on its wave, 100 MHz ticks
DG_STATS = ("solves", "rk4", "sqp_iter", "n_sqp_iter", "n_qp_iter", "t0", "t1", "first_status", "first_sqp_iter",
            "t_last_job", "spec_taken", "spec_wait", "spec_lag")
DG_CLOCK_HZ = 100e6


def build(verbose=False, extra_flags=(), out=None):
    """hipcc the solver for gfx950 into vboc_amd/libvboc_amd.so (in-tree, -O3, one translation unit).
    `extra_flags` / `out` build an instrumented variant next to it (e.g. -DVBOC_COOP_PROF)."""
    out = out or LIB_PATH
    cmd = ["hipcc", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-O3", "-shared", *extra_flags, SRC, "-o", out]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return out


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VbocError(f"{LIB_PATH} not built - run __graft_entry__.build() (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name in EXPORTS:
        getattr(lib, name)  # raises AttributeError if a symbol is missing
    lib.vboc_last_error.restype = ctypes.c_char_p
    lib.vboc_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_void_p)]
    lib.vboc_destroy.argtypes = [ctypes.c_void_p]
    lib.vboc_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double]
    lib.vboc_set_path_constraint.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_double] * 4
    lib.vboc_get_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]
    lib.vboc_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch), ctypes.c_void_p]
    lib.vboc_solve_batch_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch)]
    lib.vboc_solve_batch_ft.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch), ctypes.c_void_p]
    lib.vboc_solve_batch_ft_host.argtypes = [ctypes.c_void_p, ctypes.POINTER(Batch)]
    lib.vboc_rk4_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.vboc_rk4_batch_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p]
    lib.vboc_rk4_sens_batch_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double] + [ctypes.c_void_p] * 5
    lib.vboc_last_kernel_ms.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_int)]
    lib.vboc_debug_counters.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    lib.vboc_data_generation.argtypes = [ctypes.c_void_p, ctypes.POINTER(DgBatch), ctypes.c_void_p]
    lib.vboc_data_generation_async.argtypes = [ctypes.c_void_p, ctypes.POINTER(DgBatch), ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_void_p]
    lib.vboc_data_generation_wait.argtypes = [ctypes.c_void_p, ctypes.POINTER(DgBatch), ctypes.c_void_p]
    lib.vboc_hjr_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(HjrBatch), ctypes.c_void_p]
    lib.vboc_testing.argtypes = [ctypes.c_void_p, ctypes.POINTER(DgBatch), ctypes.c_int, ctypes.c_void_p]
    lib.vboc_testing_test.argtypes = [ctypes.c_void_p, ctypes.POINTER(TtBatch), ctypes.c_void_p]
    lib.vboc_mpc_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(MpcBatch), ctypes.c_void_p]
    lib.vboc_mpc_soft_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(MpcBatch), ctypes.POINTER(MpcSoft),
                                              ctypes.c_void_p]
    lib.vboc_al_solve_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(AlBatch), ctypes.c_void_p]
    lib.vboc_kernel_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_double)]
    _lib = lib
    return lib


def _check(rc):
    if rc != 0:
        raise VbocError(f"vboc error {rc}: {load().vboc_last_error().decode()}")


FIELDS_IN = ("x_guess", "u_guess", "p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")
_CFIELD = {"lbx0": "lbx_0", "ubx0": "ubx_0", "lbxe": "lbx_e", "ubxe": "ubx_e"}


class Solver:
    """One HIP solver handle (one device, horizons up to nmax)."""

    def __init__(self, nq, nmax, slots=0, device=0, **options):
        self.lib = load()
        self.nq, self.nmax = int(nq), int(nmax)
        h = ctypes.c_void_p()
        _check(self.lib.vboc_create(self.nq, self.nmax, int(slots), int(device), ctypes.byref(h)))
        self.h = h
        self.device = device
        for k, v in options.items():
            self.set_option(k, v)

    def close(self):
        if getattr(self, "h", None):
            self.lib.vboc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, field, value):
        _check(self.lib.vboc_set_option(self.h, field.encode(), float(value)))

    def set_path_constraint(self, c=None):
        """The OCP's nonlinear path constraint (vboc_set_path_constraint): c = systems.CartesianConstraint
        (the keep-out circle of VBOC/Cartesian constraints/), None = none."""
        if c is None:
            _check(self.lib.vboc_set_path_constraint(self.h, 0, 0.0, 0.0, 0.0, 0.0))
        else:
            _check(self.lib.vboc_set_path_constraint(self.h, 1, float(c.x_c), float(c.y_c), float(c.lh), float(c.uh)))

    def get_option(self, field):
        v = ctypes.c_double()
        _check(self.lib.vboc_get_option(self.h, field.encode(), ctypes.byref(v)))
        return v.value

    # -- host path --------------------------------------------------------------------------------
    def solve_host(self, batch, free_time=False):
        """batch: dict with N, x_guess[B,nmax+1,nx], u_guess[B,nmax,nu], p, bounds (ics.Batch).
        Returns dict(status, x, u, cost, sqp_iter, qp_iter).  free_time: the free-time box OCP
        (vboc_solve_batch_ft_host, OCPpendulum.OCP_solve) instead of the boundary OCP."""
        N = np.ascontiguousarray(batch["N"], dtype=np.int32)
        B = N.shape[0]
        arrs = {k: np.ascontiguousarray(batch[k], dtype=np.float64) for k in FIELDS_IN}
        nmax = arrs["x_guess"].shape[1] - 1
        x_out = np.array(arrs["x_guess"], copy=True)
        u_out = np.array(arrs["u_guess"], copy=True)
        status = np.zeros(B, np.int32)
        sqp_iter = np.zeros(B, np.int32)
        qp_iter = np.zeros(B, np.int32)
        cost = np.zeros(B, np.float64)
        b = Batch(B=B, nmax=nmax, N=N.ctypes.data, status=status.ctypes.data,
                  x_out=x_out.ctypes.data, u_out=u_out.ctypes.data, cost=cost.ctypes.data,
                  sqp_iter=sqp_iter.ctypes.data, qp_iter=qp_iter.ctypes.data)
        for k, a in arrs.items():
            setattr(b, _CFIELD.get(k, k), a.ctypes.data)
        fn = self.lib.vboc_solve_batch_ft_host if free_time else self.lib.vboc_solve_batch_host
        _check(fn(self.h, ctypes.byref(b)))
        return dict(status=status, x=x_out, u=u_out, cost=cost, sqp_iter=sqp_iter, qp_iter=qp_iter)

    # -- device path (torch tensors resident in HBM) ---------------------------------------------
    def solve_device(self, tb, out=None, stream=None, free_time=False):
        """tb: dict of torch cuda tensors (float64 / int32 for N).  Asynchronous on `stream`
        (default: torch's current stream).  Returns the output tensor dict.  free_time: the
        free-time box OCP (vboc_solve_batch_ft)."""
        import torch
        N = tb["N"]
        B = N.shape[0]
        nmax = tb["x_guess"].shape[1] - 1
        if out is None:
            out = dict(x=tb["x_guess"].clone(), u=tb["u_guess"].clone(),
                       status=torch.empty(B, dtype=torch.int32, device=N.device),
                       cost=torch.empty(B, dtype=torch.float64, device=N.device),
                       sqp_iter=torch.empty(B, dtype=torch.int32, device=N.device),
                       qp_iter=torch.empty(B, dtype=torch.int32, device=N.device))
        b = Batch(B=B, nmax=nmax, N=N.data_ptr(), status=out["status"].data_ptr(),
                  x_out=out["x"].data_ptr(), u_out=out["u"].data_ptr(), cost=out["cost"].data_ptr(),
                  sqp_iter=out["sqp_iter"].data_ptr(), qp_iter=out["qp_iter"].data_ptr())
        for k in FIELDS_IN:
            t = tb[k]
            assert t.is_cuda and t.dtype == torch.float64 and t.is_contiguous(), k
            setattr(b, _CFIELD.get(k, k), t.data_ptr())
        st = stream if stream is not None else torch.cuda.current_stream()
        fn = self.lib.vboc_solve_batch_ft if free_time else self.lib.vboc_solve_batch
        _check(fn(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        return out

    # -- device data generation (the whole data_generation state machine per problem on the GPU) ----
    def data_generation_device(self, ids, N_start=None, seed=None, rows_cap=None, stream=None, done_flag=None,
                               cancel=None, wait=True):
        """`data_generation(v)` for every problem id of the int64 cuda tensor `ids` (vboc_data_generation,
        dg.h).  Returns a dict of device tensors: rows [rows_used, 2nq] (blocks per problem), row_off,
        row_cnt (-1: None), ic / ic_slot (double pendulum), stats [B, 5] (DG_STATS).
        wait=False (vboc_data_generation_async): returns once the launch is queued; done_flag (int32 cuda
        tensor [B], zeroed) gets 1 per finished problem, cancel (int32 cuda tensor [1]) skips the problems not
        yet started once set; finish with data_generation_wait(out)."""
        import torch
        from .ics import SEED
        from .systems import system
        sysd = system(self.nq)
        N_start = int(N_start or sysd.N)
        seed = SEED if seed is None else int(seed)
        assert ids.is_cuda and ids.dtype == torch.int64 and ids.is_contiguous()
        B = ids.shape[0]
        dev = ids.device
        nx = 2 * self.nq
        if rows_cap is None:
            rows_cap = B * (2 * (N_start + 12) + 2)   # a problem saves at most 2N rows (quirk A.3 included)
        rows = torch.empty((max(rows_cap, 1), nx), dtype=torch.float64, device=dev)
        out = dict(row_off=torch.empty(B, dtype=torch.int64, device=dev), row_cnt=torch.empty(B, dtype=torch.int32, device=dev),
                   ic=torch.zeros((B, 4), dtype=torch.float64, device=dev), ic_slot=torch.zeros(B, dtype=torch.int32, device=dev),
                   stats=torch.empty((B, len(DG_STATS)), dtype=torch.float64, device=dev))
        m = (list(sysd.m) + [0.0, 0.0])[:2]
        l = (list(sysd.l) + [0.0, 0.0])[:2]
        b = DgBatch(B=B, ids=ids.data_ptr(), seed=seed, N_start=N_start, q_min=sysd.q_min, q_max=sysd.q_max,
                    v_max=sysd.v_max, u_max=sysd.u_max, dt=sysd.dt, tol=sysd.tol, eps=sysd.eps, g=sysd.g,
                    l1=l[0], l2=l[1], m1=m[0], m2=m[1], rows=rows.data_ptr(), rows_cap=rows_cap,
                    row_off=out["row_off"].data_ptr(), row_cnt=out["row_cnt"].data_ptr(), ic=out["ic"].data_ptr(),
                    ic_slot=out["ic_slot"].data_ptr(), stats=out["stats"].data_ptr(), rows_used=0, spec_solves=0,
                    spec_used=0)
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        out["rows_all"] = rows
        if not wait:
            for t in (done_flag, cancel):
                assert t is None or (t.is_cuda and t.dtype == torch.int32 and t.is_contiguous())
            _check(self.lib.vboc_data_generation_async(
                self.h, ctypes.byref(b), ctypes.c_void_p(done_flag.data_ptr() if done_flag is not None else 0),
                ctypes.c_void_p(cancel.data_ptr() if cancel is not None else 0), ctypes.c_void_p(st.cuda_stream)))
            out["_batch"], out["_stream"], out["_keep"] = b, st, (ids, done_flag, cancel)
            return out
        _check(self.lib.vboc_data_generation(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        out["rows"] = rows[:b.rows_used]
        out["spec_solves"], out["spec_used"] = b.spec_solves, b.spec_used
        return out

    def data_generation_wait(self, out):
        """End a launch started with data_generation_device(wait=False)."""
        b, st = out.pop("_batch"), out.pop("_stream")
        out.pop("_keep", None)
        _check(self.lib.vboc_data_generation_wait(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        out["rows"] = out["rows_all"][:b.rows_used]
        out["spec_solves"], out["spec_used"] = b.spec_solves, b.spec_used
        return out

    def testing_device(self, ids, N_start=None, seed=None, max_restarts=100, stream=None):
        """The held-out set's `testing(v)` for every problem id of the int64 cuda tensor `ids` (vboc_testing,
        dg.h k_ts).  Returns a dict of device tensors: rows [B, 2nq] (row b = problem b's x0), row_cnt (1, or -1
        for None), stats [B, len(DG_STATS)]."""
        import torch
        from .ics import SEED
        from .systems import system
        sysd = system(self.nq)
        N_start = int(N_start or sysd.N)
        seed = SEED if seed is None else int(seed)
        assert ids.is_cuda and ids.dtype == torch.int64 and ids.is_contiguous()
        B, dev = ids.shape[0], ids.device
        rows = torch.zeros((max(B, 1), 2 * self.nq), dtype=torch.float64, device=dev)
        out = dict(row_off=torch.empty(B, dtype=torch.int64, device=dev), row_cnt=torch.empty(B, dtype=torch.int32, device=dev),
                   stats=torch.empty((B, len(DG_STATS)), dtype=torch.float64, device=dev))
        m = (list(sysd.m) + [0.0, 0.0])[:2]
        l = (list(sysd.l) + [0.0, 0.0])[:2]
        b = DgBatch(B=B, ids=ids.data_ptr(), seed=seed, N_start=N_start, q_min=sysd.q_min, q_max=sysd.q_max,
                    v_max=sysd.v_max, u_max=sysd.u_max, dt=sysd.dt, tol=sysd.tol, eps=sysd.eps, g=sysd.g,
                    l1=l[0], l2=l[1], m1=m[0], m2=m[1], rows=rows.data_ptr(), rows_cap=B,
                    row_off=out["row_off"].data_ptr(), row_cnt=out["row_cnt"].data_ptr(), ic=0, ic_slot=0,
                    stats=out["stats"].data_ptr(), rows_used=0, spec_solves=0, spec_used=0)
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        _check(self.lib.vboc_testing(self.h, ctypes.byref(b), int(max_restarts), ctypes.c_void_p(st.cuda_stream)))
        out["rows"] = rows[:B]
        return out

    def testing_test_device(self, ids, N_start, seed, draw_stream, tol, dt, xlo, xhi, ulim, stream=None):
        """`testing_test(v)` for every problem id of the int64 cuda tensor `ids` (vboc_testing_test, dg.h k_tt): the
        UR5 arm (nq 4) or the Cartesian double pendulum (nq 2, handle with the circle).  Returns a dict of device
        tensors: rows [B, 2nq + 1] (x0 with the dt column), row_cnt (1, or -1 for None), stats [B, len(DG_STATS)]."""
        import torch
        assert ids.is_cuda and ids.dtype == torch.int64 and ids.is_contiguous()
        B, dev, nx = ids.shape[0], ids.device, 2 * self.nq
        out = dict(rows=torch.zeros((max(B, 1), nx + 1), dtype=torch.float64, device=dev),
                   row_cnt=torch.empty(B, dtype=torch.int32, device=dev),
                   stats=torch.empty((B, len(DG_STATS)), dtype=torch.float64, device=dev))
        pad = lambda v, n: (ctypes.c_double * n)(*(list(map(float, v)) + [0.0] * (n - len(v))))
        b = TtBatch(B=B, ids=ids.data_ptr(), seed=int(seed), N_start=int(N_start), draw_stream=int(draw_stream),
                    tol=float(tol), dt=float(dt), xlo=pad(xlo, 8), xhi=pad(xhi, 8), ulim=pad(ulim, 4),
                    rows=out["rows"].data_ptr(), row_cnt=out["row_cnt"].data_ptr(), stats=out["stats"].data_ptr())
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        _check(self.lib.vboc_testing_test(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        out["rows"] = out["rows"][:B]
        return out

    def hjr_solve_device(self, x0, weights, mean, std, u_max, stream=None):
        """The HJR one-step OCP (vboc_hjr_solve_batch, hjr.h) for every row of the float64 cuda tensor x0 [B, 2nq]:
        weights = the six NeuralNetCLS parameter tensors (float64, cuda, model.parameters() order).  Returns a
        dict of device tensors: status, cost, u, x1, sqp_iter, qp_iter."""
        import torch
        assert x0.is_cuda and x0.dtype == torch.float64 and x0.is_contiguous()
        W = [w.contiguous() for w in weights]
        for w in W:
            assert w.is_cuda and w.dtype == torch.float64
        B, dev = x0.shape[0], x0.device
        out = dict(status=torch.empty(B, dtype=torch.int32, device=dev), cost=torch.empty(B, dtype=torch.float64, device=dev),
                   u=torch.empty((B, self.nq), dtype=torch.float64, device=dev), x1=torch.empty_like(x0),
                   sqp_iter=torch.empty(B, dtype=torch.int32, device=dev), qp_iter=torch.empty(B, dtype=torch.int32, device=dev))
        b = HjrBatch(B=B, hidden=W[0].shape[0], x0=x0.data_ptr(), mean=float(mean), std=float(std), u_max=float(u_max),
                     **{n: w.data_ptr() for n, w in zip(("W0", "b0", "W1", "b1", "W2", "b2"), W)},
                     **{k: out[k].data_ptr() for k in ("status", "cost", "u", "x1", "sqp_iter", "qp_iter")})
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        _check(self.lib.vboc_hjr_solve_batch(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        out["_keep"] = W
        return out

    def mpc_solve_device(self, spec, x0, x_guess, u_guess, params=None, mean=0.0, std=1.0, rti=False, lh=0.0,
                         uh=1e6, stream=None, soft=None):
        """OCPtriplependulumHardTerm.OCP_solve (vboc_mpc_solve_batch, ft.h) for every row of the float64 cuda tensor
        x0 [B, 6]: guesses [B, N+1, 6] / [B, N, 3] (cuda, float64), spec a safempc.MpcSpec, params the NeuralNetDIR
        weights as float64 cuda tensors (None: no terminal row).  Returns a dict of device tensors: status, x, u, cost,
        sqp_iter, qp_iter, h (the row at the result's x_N).
        soft: OCPtriplependulumSoftTraj (vboc_mpc_soft_solve_batch) - dict(margin=..., Zl=[B, N+1], zl=[B, N+1] or
        None, W=[B, 9] or None, We=[B, 6] or None), float64 cuda tensors."""
        import torch
        B, N = x0.shape[0], spec.N
        for t_ in (x0, x_guess, u_guess):
            assert t_.is_cuda and t_.dtype == torch.float64 and t_.is_contiguous()
        assert tuple(x_guess.shape) == (B, N + 1, 6) and tuple(u_guess.shape) == (B, N, 3)
        dev = x0.device
        f64 = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)
        bnd = [f64(a) for a in (spec.xmin, spec.xmax, spec.umin, spec.umax, spec.xmin, spec.xmax)]
        host = [np.ascontiguousarray(a, dtype=np.float64) for a in (spec.W, spec.W_e, spec.yref, spec.yref_e)]
        out = dict(status=torch.empty(B, dtype=torch.int32, device=dev), x=torch.empty_like(x_guess),
                   u=torch.empty_like(u_guess), cost=torch.empty(B, dtype=torch.float64, device=dev),
                   sqp_iter=torch.empty(B, dtype=torch.int32, device=dev),
                   qp_iter=torch.empty(B, dtype=torch.int32, device=dev), h=torch.zeros(B, dtype=torch.float64, device=dev))
        W = [p_.contiguous() for p_ in params] if params is not None else []
        for w in W:
            assert w.is_cuda and w.dtype == torch.float64
        b = MpcBatch(B=B, N=N, rti=int(bool(rti)), hidden=W[0].shape[0] if W else 0, h=spec.time_step,
                     cost_scale=spec.cost_scale, x0=x0.data_ptr(), x_guess=x_guess.data_ptr(), u_guess=u_guess.data_ptr(),
                     mean=float(mean), std=float(std), lh=float(lh), uh=float(uh),
                     **{n: t_.data_ptr() for n, t_ in zip(("lbx", "ubx", "lbu", "ubu", "lbx_e", "ubx_e"), bnd)},
                     **{n: a.ctypes.data for n, a in zip(("W", "We", "yref", "yref_e"), host)},
                     **{n: w.data_ptr() for n, w in zip(("W0", "b0", "W1", "b1", "W2", "b2"), W)},
                     status=out["status"].data_ptr(), x_out=out["x"].data_ptr(), u_out=out["u"].data_ptr(),
                     cost=out["cost"].data_ptr(), sqp_iter=out["sqp_iter"].data_ptr(),
                     qp_iter=out["qp_iter"].data_ptr(), h_out=out["h"].data_ptr())
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        if soft is None:
            _check(self.lib.vboc_mpc_solve_batch(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
            out["_keep"] = (bnd, host, W)
            return out
        arrs = {}
        for k_, shp in (("Zl", (B, N + 1)), ("zl", (B, N + 1)), ("W", (B, 9)), ("We", (B, 6))):
            a = soft.get(k_)
            if a is None:
                continue
            assert a.is_cuda and a.dtype == torch.float64 and a.is_contiguous() and tuple(a.shape) == shp, (k_, a.shape)
            arrs[k_] = a
        sf = MpcSoft(safety_margin=float(soft["margin"]), Zl=arrs["Zl"].data_ptr(),
                     zl=arrs["zl"].data_ptr() if "zl" in arrs else None,
                     W_b=arrs["W"].data_ptr() if "W" in arrs else None,
                     We_b=arrs["We"].data_ptr() if "We" in arrs else None)
        _check(self.lib.vboc_mpc_soft_solve_batch(self.h, ctypes.byref(b), ctypes.byref(sf),
                                                  ctypes.c_void_p(st.cuda_stream)))
        out["_keep"] = (bnd, host, W, arrs)
        return out

    def al_solve_device(self, spec, x0, x_guess=None, stream=None):
        """AL's OCPtriplependulumINIT.compute_problem (vboc_al_solve_batch, ft.h) for every row of the float64 cuda
        tensor x0 [B, 6]; spec a vboc_amd.al.AlSpec; x_guess (float64 cuda [B, N+1, 6], optional):
        compute_problem_nnguess's stage guesses.  Returns a dict of device tensors: label (1 / 0 / 2), status,
        x [B, N+1, 6], u [B, N, 3], qp_iter."""
        import torch
        assert x0.is_cuda and x0.dtype == torch.float64 and x0.is_contiguous() and x0.shape[1] == 6
        B, N, dev = x0.shape[0], spec.N, x0.device
        if x_guess is not None:
            assert (x_guess.is_cuda and x_guess.dtype == torch.float64 and x_guess.is_contiguous()
                    and tuple(x_guess.shape) == (B, N + 1, 6))
        f64 = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)
        bnd = [f64(a) for a in (spec.xmin, spec.xmax, spec.umin, spec.umax, spec.xmin_e, spec.xmax_e)]
        host = [np.ascontiguousarray(a, dtype=np.float64) for a in (spec.W, spec.W_e)]
        out = dict(label=torch.empty(B, dtype=torch.int32, device=dev), status=torch.empty(B, dtype=torch.int32, device=dev),
                   x=torch.empty((B, N + 1, 6), dtype=torch.float64, device=dev),
                   u=torch.empty((B, N, 3), dtype=torch.float64, device=dev),
                   qp_iter=torch.empty(B, dtype=torch.int32, device=dev))
        b = AlBatch(B=B, N=N, h=spec.time_step, cost_scale=spec.cost_scale, x0=x0.data_ptr(),
                    x_guess=x_guess.data_ptr() if x_guess is not None else None,
                    **{n: t_.data_ptr() for n, t_ in zip(("lbx", "ubx", "lbu", "ubu", "lbx_e", "ubx_e"), bnd)},
                    W=host[0].ctypes.data, We=host[1].ctypes.data, label=out["label"].data_ptr(),
                    status=out["status"].data_ptr(), x_out=out["x"].data_ptr(), u_out=out["u"].data_ptr(),
                    qp_iter=out["qp_iter"].data_ptr())
        st = stream if stream is not None else torch.cuda.current_stream(dev)
        _check(self.lib.vboc_al_solve_batch(self.h, ctypes.byref(b), ctypes.c_void_p(st.cuda_stream)))
        out["_keep"] = (bnd, host, x0, x_guess)
        return out

    def kernel_stats(self):
        """(factor_ms_total, factor_launches, factor_algorithmic_bytes) of the last solve."""
        ms, n, by = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double()
        _check(self.lib.vboc_kernel_stats(self.h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(by)))
        return ms.value, n.value, by.value

    def last_kernel_ms(self):
        ms = ctypes.c_double()
        n = ctypes.c_int()
        _check(self.lib.vboc_last_kernel_ms(self.h, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value


def debug_counters():
    """Wave-solver phase cycles since the last call (zeros unless built with -DVBOC_COOP_PROF)."""
    buf = (ctypes.c_ulonglong * 16)()
    _check(load().vboc_debug_counters(buf))
    names = ("linearize", "qp_init", "prep", "factor", "vec", "fwd", "update", "costate", "linesearch",
             "sqp_iters", "ipm_iters", "split0", "split1", "split2", "split3", "split4")
    return {n: int(buf[i]) for i, n in enumerate(names)}


def rk4_host(nq, T, x, u):
    lib = load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    B = x.shape[0]
    xo = np.zeros_like(x)
    _check(lib.vboc_rk4_batch_host(int(nq), B, float(T), x.ctypes.data, u.ctypes.data, xo.ctypes.data))
    return xo


def rk4_sens_host(nq, T, x, u):
    """One ERK4 step with forward sensitivities per state (the solvers' linearisation): (x1, A, B)."""
    lib = load()
    x = np.ascontiguousarray(x, dtype=np.float64)
    u = np.ascontiguousarray(u, dtype=np.float64)
    B, nx = x.shape
    xo, A, Bm = np.zeros_like(x), np.zeros((B, nx, nx)), np.zeros((B, nx, nq))
    _check(lib.vboc_rk4_sens_batch_host(int(nq), B, float(T), x.ctypes.data, u.ctypes.data, xo.ctypes.data,
                                        A.ctypes.data, Bm.ctypes.data))
    return xo, A, Bm


def rk4_device(nq, T, x, u, stream=None):
    import torch
    lib = load()
    xo = torch.empty_like(x)
    st = stream if stream is not None else torch.cuda.current_stream()
    _check(lib.vboc_rk4_batch(int(nq), x.shape[0], float(T), x.data_ptr(), u.data_ptr(), xo.data_ptr(),
                              ctypes.c_void_p(st.cuda_stream)))
    return xo
