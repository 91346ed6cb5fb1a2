"""Scratch: per-problem durations of one device data-generation launch and how well the first solve
predicts the slow problems.  usage: python tools/scratch/dg_tail.py B out.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402

B = int(sys.argv[1])
s = lib.Solver(3, 120, slots=256)
out = s.data_generation_device(torch.arange(B, dtype=torch.int64, device="cuda:0"))
st = out["stats"].cpu().numpy()
np.savez(sys.argv[2], stats=st)
dur = (st[:, 6] - st[:, 5]) / 1e5
order = np.argsort(-dur)
print(f"launch {s.last_kernel_ms()[0]:.0f} ms; mean problem {dur.mean():.1f} ms; p99 {np.percentile(dur, 99):.0f} ms")
for k in (10, 100, 1000):
    top = order[:k]
    print(f"top {k}: min dur {dur[top].min():.0f} ms, first solve failed {np.mean(st[top, 7] != 0):.2f}, "
          f"first solve >= 300 it {np.mean(st[top, 8] >= 300):.2f}, solves mean {st[top, 0].mean():.1f}")
print("all: first solve failed", np.mean(st[:, 7] != 0), "first it>=300", np.mean(st[:, 8] >= 300))
