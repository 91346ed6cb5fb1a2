"""Probe: does a handle that ran constrained solves give the same unconstrained results as a fresh one?"""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from vboc_amd import lib
from vboc_amd.ics import cartesian_ics
from vboc_amd.systems import cartesian_constraint
b = cartesian_ics(np.arange(2048))
dev = torch.device("cuda:0")
tb = {k: torch.as_tensor(np.ascontiguousarray(v), device=dev) for k, v in b.items()}
def run(s):
    r = s.solve_device(tb); torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in r.items()}
fresh = lib.Solver(2, 100, slots=65536)
a = run(fresh)
a2 = run(fresh)
print("fresh", np.bincount(a["status"], minlength=6), "rerun identical", np.array_equal(a["x"], a2["x"]), flush=True)
used = lib.Solver(2, 100, slots=65536)
used.set_path_constraint(cartesian_constraint())
c = run(used)
print("circle", np.bincount(c["status"], minlength=6), flush=True)
used.set_path_constraint(None)
d = run(used)
print("after circle", np.bincount(d["status"], minlength=6), "equal to fresh", np.array_equal(a["x"], d["x"]),
      "status diff ids", np.where(a["status"] != d["status"])[0][:20], flush=True)
for mf in (0, 1):
    f2 = lib.Solver(2, 100, slots=65536, factor_mfma=mf)
    e = run(f2)
    print("fresh factor_mfma", mf, np.bincount(e["status"], minlength=6), flush=True)
# discriminate: constrained solves on handle A, then unconstrained on a fresh handle B (other regions)
A = lib.Solver(2, 100, slots=65536)
A.set_path_constraint(cartesian_constraint())
run(A)
B = lib.Solver(2, 100, slots=65536)
f = run(B)
print("fresh handle after another handle's constrained run", np.bincount(f["status"], minlength=6),
      "equal to fresh", np.array_equal(a["x"], f["x"]), flush=True)
A.set_path_constraint(None)
A.set_option("factor_mfma", 0)
g = run(A)
print("A unconstrained VALU factor", np.bincount(g["status"], minlength=6), flush=True)
