"""C_f of the UR5 arm for the SURVEY 8(d) FLOP convention: sympy CSE op count of the urdf2casadi-style ABA
restatement (oracle/ur5_rbd.py) evaluated on symbols (build container only; -> tests/golden/flops.json "4")."""
import sys, time
import numpy as np, sympy as sp
sys.path.insert(0, __import__('os').path.join(__import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))), 'oracle'))
import ur5_rbd
m = ur5_rbd.UR5()
q = sp.symbols('q0:4'); qd = sp.symbols('v0:4'); u = sp.symbols('u0:4')
# symbolic ABA with object arrays (sin/cos via sympy)
ur5_rbd.np_sin, ur5_rbd.np_cos = np.sin, np.cos
def axis_rotation(axis, qq):
    a = np.asarray(axis, float); K = ur5_rbd.skew(a)
    return np.eye(3) + sp.sin(qq) * K + (1 - sp.cos(qq)) * (K @ K)
ur5_rbd.axis_rotation = axis_rotation
t = time.time()
import types
def spatial_transform(E, r):
    X = np.zeros((6, 6), dtype=object)
    X[:3, :3] = E
    X[3:, :3] = -E @ ur5_rbd.skew(r)
    X[3:, 3:] = E
    return X
ur5_rbd.spatial_transform = spatial_transform
acc = m.aba(np.array(q, dtype=object), np.array(qd, dtype=object), np.array(u, dtype=object))
acc = [sp.nsimplify(0) + a for a in acc]
f = list(qd) + acc
rep, red = sp.cse(f)
cf = sum(sp.count_ops(e) for _, e in rep) + sum(sp.count_ops(e) for e in red)
print('C_f', cf, time.time() - t, flush=True)
X = list(q) + list(qd) + list(u)
J = [sp.diff(a, x) for a in acc for x in X]
rep2, red2 = sp.cse(f + J)
cfj = sum(sp.count_ops(e) for _, e in rep2) + sum(sp.count_ops(e) for e in red2)
print('C_fJ', cfj, time.time() - t, flush=True)
