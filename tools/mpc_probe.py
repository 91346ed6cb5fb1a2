"""Dump the GPU Safe-MPC results of tests/test_safempc.py's GPU cases (inputs are re-made on the CPU from the same
seeds) for analysis against the oracle on the CPU: python tools/mpc_probe.py <out.npz>"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, ".."))

import test_safempc as T  # noqa: E402


def main():
    out = {}
    P = T._net()
    for name, B, seed, rti, row, mi in (("rti0", 128, 5, True, False, None), ("rti1", 128, 5, True, True, None),
                                        ("sqp0", 96, 7, False, False, 200), ("sqp1", 96, 7, False, True, 200)):
        sp, x0, xg, ug = T._states(B, seed=seed)
        g = T._gpu(sp, P if row else None, x0, xg, ug, rti=rti, max_iter=mi)
        for k, v in g.items():
            out[f"{name}_{k}"] = v
        print(name, "status", np.bincount(g["status"].clip(0)), flush=True)
    np.savez(sys.argv[1], **out)


if __name__ == "__main__":
    main()
