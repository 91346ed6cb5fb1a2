"""Time the NN fit step of the VBOC loop (vboc_amd.learn.DirTrainer) on one GPU: a first fit or a refit of
--steps steps over --rows synthetic feature rows, HIP-graph replay (default) or eager.  Prints one JSON line with
the per-step time; run under `rocprofv3 --kernel-trace --stats` for the per-kernel split of a step.
usage: python tools/fit_probe.py --nq 3 --rows 500000 --steps 4096 [--refit] [--eager] [--torch]
(default: the native device trainer learn.HipTrainer; --torch: the PyTorch DirTrainer)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from vboc_amd.learn import DirTrainer, HipTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=3)
    ap.add_argument("--rows", type=int, default=500000)
    ap.add_argument("--steps", type=int, default=4096)
    ap.add_argument("--refit", action="store_true")
    ap.add_argument("--eager", action="store_true")
    ap.add_argument("--torch", action="store_true")
    a = ap.parse_args()
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    F = torch.rand((a.rows, 2 * a.nq + 1), device="cuda", generator=g)
    F[:, 2 * a.nq] += 1.0                                  # |qdot| targets away from the stop threshold
    cls = DirTrainer if a.torch else HipTrainer
    tr = cls(a.nq, "cuda", seed=0, graphs=not a.eager)
    n_new = a.rows // 2 if a.refit else 0
    tr.fit(F, n_new=n_new, it_max=257)                     # warm-up: allocations, graph capture path
    torch.cuda.synchronize()
    t = time.time()
    r = tr.fit(F, n_new=n_new, it_max=a.steps + 1)
    torch.cuda.synchronize()
    dt = time.time() - t
    print(json.dumps(dict(trainer=cls.__name__, nq=a.nq, rows=a.rows, refit=a.refit, graphs=not a.eager,
                          steps=r["iterations"],
                          launched=r["launched"], seconds=round(dt, 4),
                          ms_per_step=round(1e3 * dt / r["launched"], 5))), flush=True)


if __name__ == "__main__":
    main()
