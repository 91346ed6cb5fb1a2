"""One first-solve launch of the wave solver (k_wave) on a fixed batch, for per-pass measurements.

Run once per library variant (VBOC_LIB=<variant .so>, see tools/pass_split.sh): prints one JSON line with the
launch's kernel time (HIP events), the IPM / SQP iteration totals (stage-IPM-iterations = sum N * qp_iter,
the unit per-pass bytes are normalised by) and a digest of the outputs (pass-repeat variants must reproduce
the product build's results exactly).
usage: python tools/pass_probe.py [nq] [B]
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import make_batch
    from vboc_amd import lib
    nq = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    s = lib.Solver(nq, 100, device=0)
    if os.environ.get("VBOC_GROUPS"):   # resident problems (default: the MALL budget)
        s.set_option("wave_groups", int(os.environ["VBOC_GROUPS"]))
    tb = make_batch(nq, np.arange(B), "cuda:0")
    out = s.solve_device(tb)
    torch.cuda.synchronize()
    ms, _ = s.last_kernel_ms()
    qp = out["qp_iter"].cpu().numpy().astype(np.int64)
    sqp = out["sqp_iter"].cpu().numpy().astype(np.int64)
    N = tb["N"].cpu().numpy().astype(np.int64)
    h = hashlib.sha1()
    for k in ("status", "sqp_iter", "qp_iter", "cost", "x"):
        h.update(out[k].cpu().numpy().tobytes())
    print(json.dumps({"lib": os.path.basename(os.environ.get("VBOC_LIB") or "libvboc_amd.so"), "nq": nq, "B": B,
                      "groups": s.get_option("wave_groups"),
                      "kernel_ms": ms, "qp_iter": int(qp.sum()), "sqp_iter": int(sqp.sum()),
                      "stage_ipm_iters": int((N * qp).sum()), "stage_sqp_iters": int((N * sqp).sum()),
                      "digest": h.hexdigest()}), flush=True)


if __name__ == "__main__":
    main()
