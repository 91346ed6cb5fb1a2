"""Diagnostics: cost of UR5 problem argv[1] after 1..argv[2] SQP iterations (GPU library from VBOC_LIB)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

pid, n = int(sys.argv[1]), int(sys.argv[2])
s = lib.Solver(4, 100, slots=256)
b = ur5_ics(np.array([pid]))
for it in range(1, n + 1):
    s.set_option("nlp_solver_max_iter", it)
    g = s.solve_host(b)
    print(it, g["status"][0], g["sqp_iter"][0], g["qp_iter"][0], repr(g["cost"][0]), flush=True)
