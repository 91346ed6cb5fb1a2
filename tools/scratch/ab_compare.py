"""Scratch: compare two ab_bitexact.py outputs.  usage: python tools/scratch/ab_compare.py a.npz b.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
for k in a.files:
    x, y = a[k], b[k]
    same = x.shape == y.shape and np.array_equal(x, y)
    d = float(np.nanmax(np.abs(x - y))) if x.shape == y.shape and x.dtype.kind == "f" else None
    print(f"{k}: {'identical' if same else 'DIFFERS'} {x.shape} {y.shape} max|d| {d}")
