"""Truncated UR5 wave-solver solves for bisecting a build's divergence (verdict r03 item 1; the round-2 method of
profiles/r02p_ur5_merit_bisect.log): the 96 problems of tests/test_ur5.py's parity test, solved with
nlp_solver_max_iter / qp_solver_iter_max cut to (1, 1), (1, 2), (1, 5), (1, 100), (2, 100), (5, 100) and the
test's (300, 100).  Writes every output to <out>.npz and prints one JSON line per cut with a digest, so two
builds (VBOC_LIB) can be compared bit for bit: the first cut whose digests differ names the pass that diverges
(QP iterations -> the IPM passes; SQP iterations -> linearisation / line search).
usage: python tools/ur5_trunc.py <out prefix>
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CUTS = ((1, 1), (1, 2), (1, 5), (1, 100), (2, 100), (5, 100), (300, 100))


def main():
    from vboc_amd import lib
    from vboc_amd.ics import ur5_ics
    out = sys.argv[1]
    if "--pre" in sys.argv:     # run other kernels first (a triple first-solve batch): results that change with what
        from vboc_amd.ics import data_generation_ics     # ran before point at a read of uninitialised registers
        pre = lib.Solver(3, 120)
        pre.solve_host(data_generation_ics(3, np.arange(4096)))
        pre.close()
    b = ur5_ics(np.arange(96))
    save = {}
    for it, qp in CUTS:
        s = lib.Solver(4, int(np.max(b["N"])), slots=256)
        s.set_option("nlp_solver_max_iter", it)
        s.set_option("qp_solver_iter_max", qp)
        g = s.solve_host(b)
        s.close()
        h = hashlib.sha1()
        for k in ("status", "sqp_iter", "qp_iter", "cost", "x", "u"):
            h.update(np.ascontiguousarray(g[k]).tobytes())
            save[f"{k}_{it}_{qp}"] = g[k]
        print(json.dumps({"lib": os.path.basename(os.environ.get("VBOC_LIB") or "libvboc_amd.so"), "max_iter": it,
                          "qp_max": qp, "digest": h.hexdigest(), "ok": int((g["status"] == 0).sum()),
                          "sqp_sum": int(g["sqp_iter"].sum()), "qp_sum": int(g["qp_iter"].sum())}), flush=True)
    np.savez_compressed(out + ".npz", **save)


if __name__ == "__main__":
    main()
