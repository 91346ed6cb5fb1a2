"""Scratch: the UR5 wave solver on the same first solves with the batch padded to nmax = 100 / 120 / 200."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

ids = np.arange(300, 332)
b = ur5_ics(ids)
for nm in (100, 120, 200):
    bb = dict(b)
    bb["x_guess"] = np.concatenate([b["x_guess"], np.repeat(b["x_guess"][:, -1:], nm - 100, 1)], 1)
    bb["u_guess"] = np.concatenate([b["u_guess"], np.zeros((32, nm - 100, 4))], 1)
    for hn in (nm, 200):
        g = lib.Solver(4, hn).solve_host(bb)
        print(f"batch nmax {nm} handle nmax {hn}: status {g['status'].tolist()} sqp {g['sqp_iter'][:8].tolist()}", flush=True)
