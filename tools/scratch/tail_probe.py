"""Tail probe (diagnostic): one batched wave-mode solve per size; saves per-problem SQP / IPM iteration
counts of the first size so that the persistent kernel's end-of-launch tail can be simulated offline.

usage: python tools/tail_probe.py <out.npz> [sizes, default 100000,200000] [nq]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics  # noqa: E402

out = sys.argv[1]
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [100_000, 200_000]
nq = int(sys.argv[3]) if len(sys.argv) > 3 else 3
saved = {}
for B in sizes:
    b = data_generation_ics(nq, np.arange(B))
    s = lib.Solver(nq, int(b["N"].max()), slots=65536)
    s.set_option("wave_all", 1)
    g = s.solve_host(b)
    ms, _ = s.last_kernel_ms()
    print(f"B={B}: device {ms:.1f} ms -> {B / (ms / 1e3):.0f} solves/s | sqp mean {g['sqp_iter'].mean():.1f} "
          f"max {g['sqp_iter'].max()} | ipm/sqp {g['qp_iter'].sum() / max(1, g['sqp_iter'].sum()):.2f}", flush=True)
    if not saved:
        saved = {"sqp_iter": g["sqp_iter"], "qp_iter": g["qp_iter"], "status": g["status"],
                 "device_ms": np.float64(ms), "B": np.int64(B)}
    s.close()
np.savez(out, **saved)
