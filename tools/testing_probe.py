"""Time the test / training-set drivers on one GPU: the whole state machine on the device (one launch: vboc_testing
for the held-out set, vboc_testing_test for the UR5 and Cartesian sets) against the host-batched drivers (one
batched solve per round of the state machines, vboc_amd.drivers.run_problems) on the same ids.  Prints one JSON
line per case.
usage: python tools/testing_probe.py [--cases heldout3,cart100k,ur5] [--host-max 8192]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from vboc_amd import lib  # noqa: E402
from vboc_amd import drivers as D  # noqa: E402
from vboc_amd.systems import cartesian_constraint  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.time()
    r = fn()
    torch.cuda.synchronize()
    return r, time.time() - t


def line(case, mode, n, res, st, sec):
    rows = sum(r is not None for r in res)
    print(json.dumps(dict(case=case, mode=mode, problems=n, rows=rows, solves=st["solves"], seconds=round(sec, 3),
                          solves_per_s=round(st["solves"] / sec, 1), problems_per_s=round(n / sec, 1),
                          rounds=st.get("rounds"))), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="heldout3,cart100k,ur5")
    ap.add_argument("--host-max", type=int, default=8192)
    a = ap.parse_args()
    for case in a.cases.split(","):
        if case == "heldout3":           # configs[2]'s 10k held-out set of the triple (triplependulum_testdata.py)
            ids = np.arange(10**7, 10**7 + 10000)
            s = lib.Solver(3, 140)
            D.testing_device(3, ids[:256], s, N_start=100)          # warm-up (code objects, allocations)
            (res, st), sec = timed(lambda: D.testing_device(3, ids, s, N_start=100))
            line(case, "device", len(ids), res, st, sec)
            (res, st), sec = timed(lambda: D.testing_batch(3, ids, D.GpuBackend(3, nmax=140), N_start=100))
            line(case, "host-rounds", len(ids), res, st, sec)
        elif case.startswith("cart"):   # the Cartesian main block's training set (vboc_multiprocessing.py:567-585)
            n = 100000 if case == "cart100k" else int(case[4:])
            ids = np.arange(1000, 1000 + n)
            s = lib.Solver(2, 200)
            s.set_path_constraint(cartesian_constraint())
            D.cartesian_testing_device(ids[:256], s, N_start=100)
            (res, st), sec = timed(lambda: D.cartesian_testing_device(ids, s, N_start=100))
            line(case, "device", n, res, st, sec)
            m = min(n, a.host_max)
            be = D.GpuBackend(2, nmax=200, path_constraint=cartesian_constraint())
            (res, st), sec = timed(lambda: D.cartesian_testing_batch(ids[:m], be, N_start=100))
            line(case, "host-rounds", m, res, st, sec)
        elif case == "ur5":              # configs[4]'s per-GPU share: 12 500 testing_test problems
            ids = np.arange(10**6, 10**6 + 12500)
            s = lib.Solver(4, 400)            # a few arm problems keep extending past 100 stages
            D.ur5_testing_device(ids[:256], s, N_start=100)
            (res, st), sec = timed(lambda: D.ur5_testing_device(ids, s, N_start=100))
            line(case, "device", len(ids), res, st, sec)
            m = min(len(ids), a.host_max)
            (res, st), sec = timed(lambda: D.ur5_testing_batch(ids[:m], D.GpuBackend(4, nmax=400), N_start=100))
            line(case, "host-rounds", m, res, st, sec)


if __name__ == "__main__":
    main()
