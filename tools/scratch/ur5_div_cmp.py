import numpy as np
a = np.load("gpurun_out/ur5div_prod.npz"); b = np.load("gpurun_out/ur5div_dbg.npz")
for k in a.files:
    if k.startswith("x_") or k.startswith("u_"):
        d = np.abs(a[k] - b[k]); bad = (d > 0).reshape(d.shape[0], -1).any(1)
        print(k, "max|d|", float(np.nanmax(d)), "problems differing", int(bad.sum()), "qp_iter", a["q" + k[1:]][:4], b["q" + k[1:]][:4])
