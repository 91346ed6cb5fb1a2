"""ctypes binding of libvboc_fit.so (include/vboc_fit.h): the VBOC loop's NN fit on the device.

`build()` compiles vboc_amd/csrc/fit.hip for gfx950 in-tree; `load()` raises when the library is missing (the
trainer has no CPU path of its own: CPU runs use learn.DirTrainer explicitly).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libvboc_fit.so")
SRC = os.path.join(HERE, "csrc", "fit.hip")
EXPORTS = ("vboc_fit_create", "vboc_fit_destroy", "vboc_fit_set_params", "vboc_fit_get_params", "vboc_fit_train",
           "vboc_fit_sample", "vboc_fit_info", "vboc_fit_last_error")
EUNSUPPORTED = -3


class FitError(RuntimeError):
    pass


class FitRun(ctypes.Structure):
    """vboc_fit_run_t"""
    _fields_ = [("F", ctypes.c_void_p), ("n", ctypes.c_longlong), ("n_new", ctypes.c_longlong), ("ld", ctypes.c_int),
                ("it_max", ctypes.c_longlong), ("val0", ctypes.c_double), ("stop_val", ctypes.c_double),
                ("beta", ctypes.c_double), ("lr", ctypes.c_double), ("poll", ctypes.c_int), ("graphs", ctypes.c_int),
                ("iterations", ctypes.c_void_p), ("val", ctypes.c_void_p), ("launched", ctypes.c_void_p),
                ("kernel_ms", ctypes.c_void_p)]


def build(verbose=False):
    cmd = ["hipcc", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-O3", "-shared", SRC, "-o", LIB_PATH]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return LIB_PATH


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FitError(f"{LIB_PATH} not built - run __graft_entry__.build()")
    lib = ctypes.CDLL(LIB_PATH)
    for name in EXPORTS:
        getattr(lib, name)
    lib.vboc_fit_last_error.restype = ctypes.c_char_p
    lib.vboc_fit_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_ulonglong,
                                    ctypes.POINTER(ctypes.c_void_p)]
    lib.vboc_fit_destroy.argtypes = [ctypes.c_void_p]
    lib.vboc_fit_set_params.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 7
    lib.vboc_fit_get_params.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 7
    lib.vboc_fit_train.argtypes = [ctypes.c_void_p, ctypes.POINTER(FitRun), ctypes.c_void_p]
    lib.vboc_fit_sample.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_longlong, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
    lib.vboc_fit_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                  ctypes.POINTER(ctypes.c_longlong), ctypes.POINTER(ctypes.c_ulonglong)]
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise FitError(f"vboc_fit error {rc}: {load().vboc_fit_last_error().decode()}")


def supported(inputs, hidden, minibatch):
    hp = (hidden + 63) // 64 * 64
    return (inputs, hp) in ((6, 512), (4, 320), (2, 128)) and minibatch % 32 == 0 and 32 <= minibatch <= 4096
