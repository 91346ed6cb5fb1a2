"""UR5: wave vs lane solver vs oracle on the first B problems (iterations, status, cost, x0)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402
import oracle  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 96
b = ur5_ics(np.arange(B))
xo, uo, r = oracle.solve_batch(4, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"], b["ubu"],
                               b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], opts=oracle.default_opts(max_iter=300, lm=1e-2))
for mode in ("wave", "lane"):
    s = lib.Solver(4, 100, slots=256)
    s.set_option("nlp_solver_max_iter", 300)
    s.set_option("wave_all", 1 if mode == "wave" else 0)
    t = time.time()
    g = s.solve_host(b)
    dt = time.time() - t
    both = (g["status"] == 0) & (r["status"] == 0)
    dc = np.abs(g["cost"] - r["cost"])[both]
    dx = np.abs(g["x"][:, 0, :8] - xo[:, 0, :8]).max(axis=1)[both]
    print(f"{mode}: {dt:.1f} s  status agree {np.mean(g['status'] == r['status']):.3f}  iter agree "
          f"{np.mean(g['sqp_iter'] == r['sqp_iter']):.3f}  both {both.sum()}  |dcost| med {np.median(dc):.2e} max "
          f"{dc.max():.2e}  |dx0| med {np.median(dx):.2e} max {dx.max():.2e}", flush=True)
    s.close()
