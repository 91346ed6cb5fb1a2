"""The C-ABI library builds for gfx950, loads, and exports every symbol include/vboc.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from vboc_amd import lib

HEADER = os.path.join(lib.ROOT, "include", "vboc.h")


def declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(vboc_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_abi():
    names = declared()
    assert set(names) == set(lib.EXPORTS), names


def test_library_exports_every_declared_symbol():
    assert os.path.exists(lib.LIB_PATH), "run __graft_entry__.build() first"
    so = ctypes.CDLL(lib.LIB_PATH)
    for n in declared():
        assert hasattr(so, n), n


def test_error_reporting_without_device():
    so = lib.load()
    h = ctypes.c_void_p()
    rc = so.vboc_create(7, 100, 0, 0, ctypes.byref(h))   # nq out of range -> argument error
    assert rc == -1
    assert b"nq" in so.vboc_last_error()
    assert so.vboc_rk4_batch(3, -1, 0.01, None, None, None, None) == -1
    assert so.vboc_al_solve_batch(None, None, None) == -1
    assert b"vboc_al_solve_batch" in so.vboc_last_error()
