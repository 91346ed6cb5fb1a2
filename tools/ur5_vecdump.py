"""UR5 bisect (round 4): the vector-pass outputs of workgroup 0's first solve (XS rows and the stage-0 value of
the first vector passes) of a -DVBOC_VEC_DUMP build, for the 96 parity problems at one SQP iteration and two QP
iterations (four vector passes).  Run once per build (VBOC_LIB) and compare the dumps:
python tools/ur5_vecdump.py <out.npz>"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from vboc_amd import lib
    from vboc_amd.ics import ur5_ics
    b = ur5_ics(np.arange(96))
    L = lib.load()
    buf = (ctypes.c_double * (8 * 1024 + 8 * 256))()
    calls = ctypes.c_uint()
    L.vboc_debug_dump(buf, ctypes.byref(calls))          # reset
    s = lib.Solver(4, int(np.max(b["N"])), slots=256)
    s.set_option("nlp_solver_max_iter", 1)
    s.set_option("qp_solver_iter_max", 2)
    g = s.solve_host(b)
    L.vboc_debug_dump(buf, ctypes.byref(calls))
    allb = np.frombuffer(buf, dtype=np.float64).copy()
    d = allb[:8 * 1024].reshape(8, 1024)
    d2 = allb[8 * 1024:].reshape(8, 256)
    np.savez(sys.argv[1], dump=d, dump2=d2, calls=calls.value, x=g["x"], u=g["u"], status=g["status"])
    print(os.path.basename(os.environ.get("VBOC_LIB") or "libvboc_amd.so"), "calls", calls.value,
          "dump sums", [float(np.abs(d[i]).sum()) for i in range(min(calls.value, 8))], flush=True)


if __name__ == "__main__":
    main()
