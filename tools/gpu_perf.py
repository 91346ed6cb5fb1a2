"""Throughput probe: one batched solve at several sizes (diagnostic)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics, heldout_ics  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 3
sizes = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [4096]
slots = int(sys.argv[3]) if len(sys.argv) > 3 else 0
law = sys.argv[4] if len(sys.argv) > 4 else "dg"
max_iter = int(sys.argv[5]) if len(sys.argv) > 5 else 0
coops = [x for x in sys.argv[6].split(",")] if len(sys.argv) > 6 else [None]
for B, coop in [(B, c) for B in sizes for c in coops]:
    b = (data_generation_ics if law == "dg" else heldout_ics)(nq, np.arange(B))
    s = lib.Solver(nq, int(b["N"].max()), slots=slots)
    if coop is not None and coop.startswith("wave"):
        s.set_option("wave_all", 1)
        if coop[4:]:
            s.set_option("wave_groups", int(coop[4:]))
    elif coop is not None:
        s.set_option("coop_threshold", float(coop))
    if max_iter:
        s.set_option("nlp_solver_max_iter", max_iter)
    t = time.time()
    g = s.solve_host(b)
    tw = time.time() - t
    ms, nl = s.last_kernel_ms()
    it = g["sqp_iter"]
    print(f"nq={nq} law={law} B={B} coop={coop} ({s.get_option('coop_problems'):.0f}, groups "
          f"{s.get_option('wave_groups'):.0f}) "
          f"slots={s.get_option('slots'):.0f}: wall {tw:.2f}s device {ms:.1f} ms "
          f"launches {nl} -> {B / (ms / 1e3):.0f} solves/s | ok {np.mean(g['status'] == 0):.4f} "
          f"sqp mean {it.mean():.1f} p99 {np.percentile(it, 99):.0f} max {it.max()} | qp/sqp "
          f"{g['qp_iter'].sum() / max(1, it.sum()):.1f}", flush=True)
    dc = lib.debug_counters()
    if dc["sqp_iters"]:
        ip = max(1, dc["ipm_iters"])
        main = {k: v for k, v in dc.items() if k not in ("sqp_iters", "ipm_iters") and not k.startswith("split")}
        print("  wave phase cycles per IPM iteration:", {k: round(v / ip) for k, v in main.items()},
              "| per SQP iteration:", round(sum(main.values()) / dc["sqp_iters"]), flush=True)
        if any(dc[f"split{i}"] for i in range(5)):
            print("  split of the profiled pass, cycles per IPM iteration:",
                  [round(dc[f"split{i}"] / ip) for i in range(5)], flush=True)
    s.close()
