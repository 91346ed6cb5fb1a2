"""Scratch: wave-solver phase cycles per IPM iteration (needs a -DVBOC_COOP_PROF build via VBOC_LIB),
factor_mfma on / off.  usage: VBOC_LIB=... python tools/scratch/phase_ab.py nq B groups"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics  # noqa: E402

nq, B, groups = (int(a) for a in sys.argv[1:4])
b = data_generation_ics(nq, np.arange(B))
for fm in (1, 0, 1):
    s = lib.Solver(nq, 100, slots=65536)
    s.set_option("factor_mfma", fm)
    if groups:
        s.set_option("wave_groups", groups)
    lib.debug_counters()
    t = time.time()
    g = s.solve_host(b)
    ms, _ = s.last_kernel_ms()
    dc = lib.debug_counters()
    ip = max(1, dc["ipm_iters"])
    ph = {k: round(v / ip) for k, v in dc.items() if k not in ("sqp_iters", "ipm_iters") and not k.startswith("split")}
    print(f"nq {nq} B {B} groups {s.get_option('wave_groups'):.0f} factor_mfma {fm}: kernel {ms:.0f} ms -> "
          f"{B / ms * 1e3:.0f} solves/s, ipm/problem {g['qp_iter'].mean():.1f} | cycles per IPM iteration {ph} "
          f"total {sum(ph.values())}", flush=True)
    s.close()
