"""Scratch: outputs of one library build for a bit-exactness A/B (first solves in wave mode + the device
data-generation loop).  usage: VBOC_LIB=<lib> python tools/scratch/ab_bitexact.py out.npz"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from vboc_amd import lib  # noqa: E402
from vboc_amd.ics import data_generation_ics  # noqa: E402

res = {}
for nq in (2, 3):
    b = data_generation_ics(nq, np.arange(1024))
    s = lib.Solver(nq, 100, slots=256)
    g = s.solve_host(b)
    for k in ("x", "u", "cost", "status", "sqp_iter", "qp_iter"):
        res[f"fs{nq}_{k}"] = g[k]
    s = lib.Solver(nq, 120, slots=256)
    o = s.data_generation_device(torch.arange(2048, dtype=torch.int64, device="cuda:0"))
    cnt, off, rows = o["row_cnt"].cpu().numpy(), o["row_off"].cpu().numpy(), o["rows"].cpu().numpy()
    res[f"dg{nq}_cnt"] = cnt
    res[f"dg{nq}_rows"] = np.concatenate([rows[off[i]:off[i] + cnt[i]] for i in range(len(cnt)) if cnt[i] > 0])
    res[f"dg{nq}_stats"] = o["stats"].cpu().numpy()[:, [0, 1, 2, 3, 4, 7, 8]]
np.savez(sys.argv[1], **res)
print("saved", sys.argv[1])
