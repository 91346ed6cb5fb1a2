"""Scratch: oracle reference for ur5_bisect.py.  usage: python tools/scratch/make_ref.py nq B max_iter out.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from vboc_amd.ics import data_generation_ics, ur5_ics  # noqa: E402

nq, B, mi = (int(a) for a in sys.argv[1:4])
b = ur5_ics(np.arange(B)) if nq == 4 else data_generation_ics(nq, np.arange(B))
xo, uo, r = oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"], b["ubu"],
                               b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"],
                               opts=oracle.default_opts(max_iter=mi, lm=1e-2 if nq == 4 else 1e-5))
np.savez(sys.argv[4], nq=nq, B=B, max_iter=mi, status=r["status"], sqp_iter=r["sqp_iter"], cost=r["cost"],
         x0=xo[:, 0, :])
print(np.bincount(r["status"]), np.percentile(r["sqp_iter"], [50, 90, 100]))
