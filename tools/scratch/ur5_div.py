"""Scratch: UR5 wave-solver outputs after truncated solves (nlp iterations x QP iterations), saved per build
to compare the product build with the debug build bit for bit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

tag = sys.argv[1]
b = ur5_ics(np.arange(300, 332))
out = {}
for nlp in (1, 2):
    for qp in (1, 2, 3, 4, 6, 10, 20, 50):
        s = lib.Solver(4, 100)
        s.set_option("wave_all", 1)
        s.set_option("nlp_solver_max_iter", nlp)
        s.set_option("qp_solver_iter_max", qp)
        g = s.solve_host(b)
        out[f"x_{nlp}_{qp}"] = g["x"]
        out[f"u_{nlp}_{qp}"] = g["u"]
        out[f"q_{nlp}_{qp}"] = g["qp_iter"]
        s.close()
np.savez(f"gpurun_out/ur5div_{tag}.npz", **out)
print(tag, "saved", flush=True)
