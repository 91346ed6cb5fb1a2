"""Diagnostics: the solvers' linearisation (ERK4 + forward sensitivities) standalone on the GPU vs the oracle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from vboc_amd import lib  # noqa: E402
import oracle  # noqa: E402

for nq in [int(a) for a in sys.argv[1:]] or [3, 4]:
    rng = np.random.default_rng(nq)
    X = rng.uniform(-2, 2, (512, 2 * nq))
    U = rng.uniform(-5, 5, (512, nq))
    t = time.time()
    x1, A, B = lib.rk4_sens_host(nq, 1e-2, X, U)
    dt = time.time() - t
    err = 0.0
    for i in range(0, 512, 16):
        r1, rA, rB = oracle.rk4_sens(nq, 1e-2, X[i], U[i])
        err = max(err, np.abs(r1 - x1[i]).max(), np.abs(rA - A[i]).max(), np.abs(rB - B[i]).max())
    print(f"nq={nq}: {dt:.3f} s, max |gpu - oracle| {err:.3e}", flush=True)
