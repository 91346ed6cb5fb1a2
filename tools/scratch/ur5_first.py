"""Scratch: UR5 first solves of ids 300..331 (wave solver) vs the oracle's SQP iteration counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402

ORACLE = [12, 74, 65, 6, 14, 10, 11, 96, 9, 63, 536, 16, 11, 5, 5, 23, 6, 6, 20, 8, 122, 43, 441, 7, 45, 7, 5, 15, 194, 53,
          227, 6]
b = ur5_ics(np.arange(300, 332))
s = lib.Solver(4, 100)
s.set_option("wave_all", 1)
g = s.solve_host(b)
print(os.environ.get("VBOC_LIB", "product"), "iteration agreement with the oracle",
      np.mean(g["sqp_iter"] == np.array(ORACLE)), g["sqp_iter"].tolist(), flush=True)
