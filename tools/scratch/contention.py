"""Scratch: wave-solver phase cycles per IPM iteration against the number of resident problems (memory
contention vs instruction latency).  usage: VBOC_LIB=<-DVBOC_COOP_PROF build> python tools/scratch/contention.py B g1,g2,..."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics  # noqa: E402

B = int(sys.argv[1])
b = data_generation_ics(3, np.arange(B))
for groups in (int(x) for x in sys.argv[2].split(",")):
    s = lib.Solver(3, 100, slots=256)
    s.set_option("wave_groups", groups)
    s.set_option("nlp_solver_max_iter", 200)
    lib.debug_counters()
    g = s.solve_host(b)
    ms, _ = s.last_kernel_ms()
    dc = lib.debug_counters()
    ip = max(1, dc["ipm_iters"])
    ph = {k: round(v / ip) for k, v in dc.items() if k not in ("sqp_iters", "ipm_iters") and not k.startswith("split")}
    sp = [round(dc[f"split{i}"] / ip) for i in range(5)]
    print(f"groups {groups}: kernel {ms:.0f} ms -> {B / ms * 1e3:.0f} solves/s | cycles per IPM iteration {ph} "
          f"total {sum(ph.values())} split {sp}", flush=True)
    s.close()
