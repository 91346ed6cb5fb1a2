"""Diagnostics: one UR5 problem (id argv[1]) on the GPU library selected by VBOC_LIB, max_iter argv[2]."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

pid, it = int(sys.argv[1]), int(sys.argv[2])
s = lib.Solver(4, 100, slots=256)
s.set_option("nlp_solver_max_iter", it)
g = s.solve_host(ur5_ics(np.array([pid])))
print("status", g["status"], "sqp", g["sqp_iter"], "cost", g["cost"], flush=True)
