"""Scratch: per-SQP-iteration divergence of the wave solver vs the oracle (x_out after max_iter = 1..K)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

B = 8
b = ur5_ics(np.arange(B))
s = lib.Solver(4, int(b["N"].max()), slots=256)
for mi in (0, 1, 2, 3, 5, 8):
    s.set_option("nlp_solver_max_iter", mi)
    g = s.solve_host(b)
    xo, uo, r = oracle.solve_batch(4, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"], b["ubu"],
                                   b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], opts=oracle.default_opts(max_iter=mi, lm=1e-2))
    dx = np.abs(g["x"][:, :, :8] - xo[:, :, :8]).max(axis=(1, 2))
    du = np.abs(g["u"] - uo).max(axis=(1, 2))
    print(f"{sys.argv[1]} max_iter {mi}: dx {np.array2string(dx, precision=1)} du {np.array2string(du, precision=1)} "
          f"qp {g['qp_iter'].tolist()} vs {r['qp_iter'].tolist()}", flush=True)
