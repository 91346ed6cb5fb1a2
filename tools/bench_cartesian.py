"""Throughput of the Cartesian double pendulum's OCP (keep-out circle) on one MI355X.

First solves of `testing_test` (ics.cartesian_ics, N = 100) through the C ABI with inputs resident in HBM
(vboc_solve_batch): the constrained OCP on the wave solver (and on a larger batch) and on the lane-mode kernels, beside the
same problems without the circle on both paths, and the CPU oracle (OpenMP over the host cores, a bounded sample)
with the circle.  Prints one JSON object.

usage: python tools/bench_cartesian.py [--batch 8192] [--cpu-sample 256]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--big", type=int, default=16384, help="batch of the extra wave-solver run with the circle")
    ap.add_argument("--cpu-sample", type=int, default=256)
    args = ap.parse_args()
    import torch
    from vboc_amd import lib
    from vboc_amd.ics import cartesian_ics
    from vboc_amd.systems import cartesian_constraint
    B = args.batch
    b = cartesian_ics(np.arange(B))
    dev = torch.device("cuda:0")
    tb = {k: torch.as_tensor(np.ascontiguousarray(v), device=dev) for k, v in b.items()}
    tw = {k: v[:256].contiguous() for k, v in tb.items()}
    out = {}
    s = lib.Solver(2, 100, slots=65536)

    def run(tag, hc, wave, tbx=None):
        tbx = tbx or tb
        nb = int(tbx["N"].shape[0])
        s.set_path_constraint(cartesian_constraint() if hc else None)
        s.set_option("wave_all", 1 if wave else 0)
        s.set_option("coop_threshold", 0)
        s.solve_device(tw)                       # warm-up (first launches) on a slice
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = s.solve_device(tbx)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        st = r["status"].cpu().numpy()
        out[tag] = dict(problems=nb, seconds=dt, solves_per_s=nb / dt, converged=float(np.mean(st == 0)),
                        status_counts=np.bincount(st, minlength=6).tolist(),
                        sqp_iter_mean=float(r["sqp_iter"].double().mean().item()))
        print(tag, out[tag], file=sys.stderr, flush=True)

    run("gpu_wave_circle", True, True)
    bb = cartesian_ics(np.arange(args.big))
    run("gpu_wave_circle_big", True, True,
        {k: torch.as_tensor(np.ascontiguousarray(v), device=dev) for k, v in bb.items()})
    run("gpu_lane_circle", True, False)
    run("gpu_lane_no_circle", False, False)
    run("gpu_wave_no_circle", False, True)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    n = min(args.cpu_sample, B)
    keys = ("N", "x_guess", "u_guess", "p", "lbx", "ubx", "lbu", "ubu", "lbx0", "ubx0", "lbxe", "ubxe")
    threads = min(16, os.cpu_count() or 1)
    t = time.perf_counter()
    _, _, r = oracle.solve_batch(2, *[b[k][:n] for k in keys], opts=oracle.default_opts(**oracle.cartesian_opts()),
                                 nthreads=threads)
    dt = time.perf_counter() - t
    out["cpu_oracle_circle"] = dict(seconds=dt, solves_per_s=n / dt, sample=n, cores=threads,
                                    converged=float(np.mean(r["status"] == 0)))
    g = out["gpu_wave_circle"]
    print(json.dumps(dict(workload="Cartesian double pendulum testing_test first solves (cartesian_ics, N=100)",
                          batch=B, dtype="f64", data="synthetic", results=out,
                          gpu_vs_cpu=g["solves_per_s"] / out["cpu_oracle_circle"]["solves_per_s"])))


if __name__ == "__main__":
    main()
