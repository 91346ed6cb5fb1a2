"""Scratch: wave-mode UR5 (or chain) solve of the first B problems vs a stored oracle reference.
usage: VBOC_LIB=<variant .so> python tools/scratch/ur5_bisect.py <ref.npz> <label>"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics, ur5_ics  # noqa: E402

ref = np.load(sys.argv[1])
nq, B, mi = int(ref["nq"]), int(ref["B"]), int(ref["max_iter"])
b = ur5_ics(np.arange(B)) if nq == 4 else data_generation_ics(nq, np.arange(B))
s = lib.Solver(nq, int(b["N"].max()), slots=256)
s.set_option("nlp_solver_max_iter", mi)
t = time.time()
g = s.solve_host(b)
dt = time.time() - t
both = (g["status"] == 0) & (ref["status"] == 0)
dc = np.abs(g["cost"] - ref["cost"])[both]
nx = 2 * nq
dx = np.abs(g["x"][:, 0, :nx] - ref["x0"][:, :nx]).max(axis=1)[both] if both.any() else np.array([np.nan])
bad = np.nonzero(g["sqp_iter"] != ref["sqp_iter"])[0]
print(f"{sys.argv[2]}: {dt:.1f} s status agree {np.mean(g['status'] == ref['status']):.3f} iter agree "
      f"{np.mean(g['sqp_iter'] == ref['sqp_iter']):.3f} both {both.sum()} |dcost| max {dc.max() if dc.size else np.nan:.2e} "
      f"|dx0| max {np.nanmax(dx):.2e} first mismatches {bad[:8].tolist()} gpu it {g['sqp_iter'][bad[:8]].tolist()} "
      f"ref it {ref['sqp_iter'][bad[:8]].tolist()}", flush=True)
