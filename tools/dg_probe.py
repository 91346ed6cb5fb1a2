"""One data-generation launch (k_dg, the bench's dominant kernel) on a fixed id range, for driver-shape A/Bs.

The bench's timed launch is 400k problems; its rate is the bulk rate (every resident wave busy) plus one tail
(the slowest problem after the queue drains).  This probe reports both for a launch of B problems:
  kernel_ms     the whole launch (HIP events)
  bulk          solves per second while the queue still feeds every wave: solves of the problems that ended
                inside [t_first + 5 % of the drain time, queue drained] / that window (device real-time clock)
  drained_ms    when the last job (new problem or parked resume) was taken; last_ms when the last problem finished
  digest        sha1 of the per-problem rows / counts / solve statistics (variants that claim the same results
                must reproduce the product's digest)
Run once per library (VBOC_LIB=<variant .so>) and resident-problem count (--groups).
usage: python tools/dg_probe.py [--nq 3] [--B 100000] [--groups 0 ...] [--first 0]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import dg_flops, order_rows
    from vboc_amd import lib
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=3)
    ap.add_argument("--B", type=int, default=100_000)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--groups", type=int, nargs="*", default=[0])
    ap.add_argument("--park", type=int, nargs="*", default=[1],
                    help="dg_park option values to run (1: parked first solves, the product default; 0: off)")
    ap.add_argument("--window", type=int, nargs="*", default=[0],
                    help="dg_spec_window option values to run (0: off, the product default)")
    ap.add_argument("--spec-first", type=int, nargs="*", default=[2],
                    help="dg_spec_first option values to run (1: restart jobs before parked resumes)")
    ap.add_argument("--spec-crit", type=int, nargs="*", default=[0],
                    help="dg_spec_crit option values to run (1: the critical-path rule for restart jobs)")
    ap.add_argument("--spec-pause", type=int, nargs="*", default=[0],
                    help="dg_spec_pause option values to run (> 0: early events after that many SQP iterations)")
    ap.add_argument("--park-window", type=int, nargs="*", default=[0],
                    help="dg_park_window option values to run (0: the product default)")
    ap.add_argument("--save", default=None, help="write the per-problem stats (lib.DG_STATS) of each launch to "
                                                 "<save>_g<groups>.npy (scheduling studies)")
    a = ap.parse_args()
    s = lib.Solver(a.nq, 120, device=0)
    ids = torch.arange(a.first, a.first + a.B, dtype=torch.int64, device="cuda:0")
    for g, pk, wn, sf, sc, pw, sp in [(g, pk, wn, sf, sc, pw, sp) for sp in a.spec_pause for pw in a.park_window
                                      for sc in a.spec_crit for sf in a.spec_first for wn in a.window for pk in a.park
                                      for g in a.groups]:
        if any(a.spec_pause):   # the option exists from round 6's library on
            s.set_option("dg_spec_pause", sp)
        s.set_option("dg_park_window", pw)
        s.set_option("dg_spec_crit", sc)
        s.set_option("dg_spec_first", sf)
        s.set_option("wave_groups", g)
        s.set_option("dg_park", pk)
        s.set_option("dg_spec_window", wn)
        t = time.time()
        out = s.data_generation_device(ids)
        torch.cuda.synchronize()
        wall = time.time() - t
        ms, _ = s.last_kernel_ms()
        st = out["stats"].cpu().numpy()
        t0, t1 = st[:, 5], st[:, 6]
        base = t0.min()
        drained = st[:, 9].max() - base          # the last job taken (a new problem or a parked resume)
        lo = base + 0.05 * drained
        hi = base + drained
        inwin = (t1 >= lo) & (t1 <= hi)
        bulk = float(st[inwin, 0].sum()) / ((hi - lo) / lib.DG_CLOCK_HZ) if hi > lo else None
        h = hashlib.sha1()
        h.update(order_rows(out).cpu().numpy().tobytes())
        h.update(out["row_cnt"].cpu().numpy().tobytes())
        h.update(st[:, [0, 1, 2, 3, 4, 7, 8]].tobytes())
        rec = {"lib": os.path.basename(os.environ.get("VBOC_LIB") or "libvboc_amd.so"), "nq": a.nq, "B": a.B,
               "groups": int(s.get_option("last_groups")), "park": pk, "window": wn, "spec_first": sf, "spec_crit": sc, "park_window": pw, "spec_pause": sp, "kernel_ms": round(ms, 1), "wall_s": round(wall, 2),
               "solves": int(st[:, 0].sum()), "solves_per_s": round(float(st[:, 0].sum()) / (ms / 1e3), 1),
               "bulk_solves_per_s": round(bulk, 1) if bulk else None,
               "drained_ms": round(drained / lib.DG_CLOCK_HZ * 1e3, 1),
               "last_ms": round((t1.max() - base) / lib.DG_CLOCK_HZ * 1e3, 1),
               "stage_ipm_iters_per_s": round(float(st[:, 4].sum()) / (ms / 1e3), 1),
               "tflops": round(dg_flops(a.nq, st) / (ms / 1e3) / 1e12, 4),
               "spec_solves": int(out.get("spec_solves", -1)), "spec_used": int(out.get("spec_used", -1)),
               "digest": h.hexdigest()}
        print(json.dumps(rec), flush=True)
        if a.save:
            np.save(f"{a.save}_g{rec['groups']}_p{pk}_w{wn}_f{sf}_c{sc}.npy", st)


if __name__ == "__main__":
    main()
