"""Quick GPU-vs-oracle check + timing (diagnostic; the real gates live in tests/)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics, heldout_ics  # noqa: E402


def compare(nq, law, B, slots=0):
    b = (data_generation_ics if law == "dg" else heldout_ics)(nq, np.arange(B))
    s = lib.Solver(nq, int(b["N"].max()), slots=slots)
    t = time.time()
    g = s.solve_host(b)
    tg = time.time() - t
    ms, _ = s.last_kernel_ms()
    t = time.time()
    xo, uo, r = oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"])
    tc = time.time() - t
    same = g["status"] == r["status"]
    ok = (g["status"] == 0) & (r["status"] == 0)
    dcost = np.abs(g["cost"] - r["cost"])[ok]
    dx0 = np.abs(g["x"][:, 0, :2 * nq] - xo[:, 0, :2 * nq]).max(axis=1)[ok]
    itsame = (g["sqp_iter"] == r["sqp_iter"])
    print(f"nq={nq} law={law} B={B}: gpu {tg:.3f}s (kernel {ms:.1f} ms) cpu {tc:.3f}s | status agree "
          f"{same.mean():.3f} gpu ok {np.mean(g['status'] == 0):.3f} cpu ok {np.mean(r['status'] == 0):.3f} | "
          f"sqp-iter agree {itsame.mean():.3f} | max|dcost| {dcost.max() if dcost.size else 0:.2e} "
          f"median {np.median(dcost) if dcost.size else 0:.2e} | max|dx0| {dx0.max() if dx0.size else 0:.2e}",
          flush=True)
    bad = np.where(~same)[0][:5]
    for i in bad:
        print("   mismatch", i, "gpu", g["status"][i], g["sqp_iter"][i], g["cost"][i], "cpu", r["status"][i],
              r["sqp_iter"][i], r["cost"][i])
    return g, r


def timing(nq, B, slots=0):
    b = data_generation_ics(nq, np.arange(B))
    s = lib.Solver(nq, int(b["N"].max()), slots=slots)
    t = time.time()
    g = s.solve_host(b)
    tg = time.time() - t
    ms, _ = s.last_kernel_ms()
    print(f"timing nq={nq} B={B} slots={s.get_option('slots'):.0f}: wall {tg:.2f}s kernel {ms:.1f} ms -> "
          f"{B / (ms / 1e3):.0f} solves/s; ok {np.mean(g['status'] == 0):.3f} mean sqp {g['sqp_iter'].mean():.1f} "
          f"max sqp {g['sqp_iter'].max()} qp/sqp {g['qp_iter'].sum() / max(1, g['sqp_iter'].sum()):.1f}", flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "parity"):
        compare(1, "test", 256)
        compare(2, "dg", 256)
        compare(3, "dg", 256)
        compare(3, "test", 128)
    if which in ("all", "timing"):
        for B in (4096, 32768):
            timing(3, B)
