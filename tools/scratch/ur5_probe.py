"""Stepwise UR5 probe on the GPU (prints after every step): twin RK4, then solves of growing size."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

t0 = time.time()
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import ur5_ics  # noqa: E402
import oracle  # noqa: E402

print("import", round(time.time() - t0, 1), flush=True)
x = np.zeros((4, 8))
u = np.zeros((4, 4))
t = time.time()
x1 = lib.rk4_host(4, 1e-2, x, u)
print("rk4", round(time.time() - t, 2), np.abs(x1 - np.stack([oracle.rk4(4, 1e-2, x[i], u[i]) for i in range(4)])).max(),
      flush=True)
s = lib.Solver(4, 100, slots=256)
if os.environ.get("VBOC_MODE") == "lane":
    s.set_option("wave_all", 0)
    s.set_option("coop_threshold", 0)
print("create", s.get_option("wave_groups"), s.get_option("levenberg_marquardt"), os.environ.get("VBOC_MODE"),
      flush=True)
for B, it in [(int(a), int(b)) for a, b in (arg.split(":") for arg in sys.argv[1:])]:
    s.set_option("nlp_solver_max_iter", it)
    b = ur5_ics(np.arange(B))
    t = time.time()
    g = s.solve_host(b)
    ms, _ = s.last_kernel_ms()
    print(f"B={B} max_iter={it}: {time.time() - t:.2f} s (kernel {ms:.1f} ms) status {np.bincount(g['status'])} "
          f"sqp mean {g['sqp_iter'].mean():.1f} max {g['sqp_iter'].max()} qp {g['qp_iter'].mean():.1f}", flush=True)
    if B <= 16:
        xo, uo, r = oracle.solve_batch(4, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                       b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"],
                                       opts=oracle.default_opts(max_iter=it, lm=1e-2))
        print("  oracle status", r["status"], "sqp", r["sqp_iter"], "gpu sqp", g["sqp_iter"], flush=True)
        both = (g["status"] == 0) & (r["status"] == 0)
        if both.any():
            print("  |dcost| max", np.abs(g["cost"] - r["cost"])[both].max(), flush=True)
s.close()
