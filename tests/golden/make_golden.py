"""Generate golden dynamics vectors from the reference's OWN model expressions.

Runs only in the build container (it reads /root/reference at run time); the
outputs (`dynamics_*.npz`, `flops.json`) are small committed fixtures that the
CPU/GPU tests load on any machine.  Nothing of the reference travels: only
numbers computed from its expressions.

How: the reference class files are parsed as TEXT with `ast`.  From
`OCP<sys>.__init__` we take the constant assignments (`self.m1 = 0.4` ...),
the state / control symbol lists (`self.x = vertcat(...)`, `u = vertcat(...)`)
and the `f_expl = ...` expression; from `SYM<sys>INIT.__init__` the unscaled
twin-integrator expression.  Each expression is rebuilt in sympy (exact
derivatives) and evaluated at seeded points:

    VBOC/pendulum_class_vboc.py:14-39          (1 link, damped, dt-scaled)
    VBOC/doublependulum_class_vboc.py:14-91    (2 links, dt-scaled) / :228-293 twin
    VBOC/triplependulum_class_vboc.py:15-58    (3 links, dt-scaled) / :201-228 twin

The twin RK4 step follows AcadosSim ERK with num_stages=4, one step, T=1e-2
(VBOC/triplependulum_class_vboc.py:235-239) - the published classical RK4.

Also recorded: sympy CSE operation counts of f and f+df/d(x,u) (the FLOP
convention of SURVEY.md section 8(d)).
"""
import ast
import json
import os
import sys

import numpy as np
import sympy as sp

REF = "/root/reference/VBOC"
HERE = os.path.dirname(os.path.abspath(__file__))

SYSTEMS = {
    1: ("pendulum_class_vboc.py", "OCPpendulum", None),
    2: ("doublependulum_class_vboc.py", "OCPdoublependulum", "SYMdoublependulumINIT"),
    3: ("triplependulum_class_vboc.py", "OCPtriplependulum", "SYMtriplependulumINIT"),
}


def _init_body(tree, cls_name):
    for node in tree.body:
        if isinstance(node, ast.ClassDef) and node.name == cls_name:
            for fn in node.body:
                if isinstance(fn, ast.FunctionDef) and fn.name == "__init__":
                    return fn.body
    raise KeyError(cls_name)


class _Sym(ast.NodeTransformer):
    """self.<const> -> numeric constant (as sympy Float via the namespace)."""

    def visit_Attribute(self, node):
        self.generic_visit(node)
        if isinstance(node.value, ast.Name) and node.value.id == "self":
            return ast.copy_location(ast.Name(id="SELF_" + node.attr, ctx=ast.Load()), node)
        return node


def _vertcat_names(expr):
    assert isinstance(expr, ast.Call) and expr.func.id == "vertcat"
    return [a.id for a in expr.args]


def extract(nq):
    fname, ocp_cls, sym_cls = SYSTEMS[nq]
    src = open(os.path.join(REF, fname)).read()
    tree = ast.parse(src)
    body = _init_body(tree, ocp_cls)
    consts, xs, us, f_ast = {}, None, None, None
    for st in body:
        if not isinstance(st, ast.Assign) or len(st.targets) != 1:
            continue
        t = st.targets[0]
        if isinstance(t, ast.Attribute) and isinstance(t.value, ast.Name) and t.value.id == "self":
            if isinstance(st.value, ast.Constant) and isinstance(st.value.value, (int, float)):
                consts[t.attr] = float(st.value.value)
            if t.attr == "x" and isinstance(st.value, ast.Call):
                xs = _vertcat_names(st.value)
        if isinstance(t, ast.Name) and t.id == "u":
            us = _vertcat_names(st.value)
        if isinstance(t, ast.Name) and t.id == "f_expl" and f_ast is None:
            f_ast = st.value
    twin_ast, twin_xs = None, None
    if sym_cls is not None:
        for st in _init_body(tree, sym_cls):
            if isinstance(st, ast.Assign) and len(st.targets) == 1:
                t = st.targets[0]
                if isinstance(t, ast.Name) and t.id == "f_expl":
                    twin_ast = st.value
                if isinstance(t, ast.Attribute) and t.attr == "x" and isinstance(st.value, ast.Call):
                    twin_xs = _vertcat_names(st.value)
    syms = {name: sp.Symbol(name, real=True) for name in xs + us}
    ns = {"sin": sp.sin, "cos": sp.cos, "vertcat": lambda *a: sp.Matrix([sp.sympify(v) for v in a])}
    ns.update({"SELF_" + k: sp.Float(v, 30) for k, v in consts.items()})
    ns.update(syms)

    def build(node):
        e = ast.Expression(body=_Sym().visit(node))
        ast.fix_missing_locations(e)
        return eval(compile(e, "<ref-expr>", "eval"), {"__builtins__": {}}, ns)

    f = build(f_ast)
    twin = build(twin_ast) if twin_ast is not None else None
    return dict(consts=consts, xs=[syms[n] for n in xs], us=[syms[n] for n in us], f=f,
                twin=twin, twin_xs=[syms[n] for n in twin_xs] if twin_xs else None)


def cse_ops(exprs):
    rep, red = sp.cse(exprs)
    return int(sum(sp.count_ops(r[1]) for r in rep) + sum(sp.count_ops(e) for e in red))


def rk4(fun, x, u, h):
    k1 = fun(x, u)
    k2 = fun(x + 0.5 * h * k1, u)
    k3 = fun(x + 0.5 * h * k2, u)
    k4 = fun(x + h * k3, u)
    return x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)


def rk4_jac(fun, jac, x, u, h):
    """d RK4(x, u) / d(x, u) by forward sensitivities through the reference's own Jacobian `jac`."""
    nx, nu = len(x), len(u)
    E = np.vstack([np.hstack([np.zeros((nu, nx)), np.eye(nu)])])
    I = np.hstack([np.eye(nx), np.zeros((nx, nu))])
    Jf = lambda xx: np.asarray(jac(list(xx), list(u)), dtype=float)
    dk = lambda xx, dX: Jf(xx) @ np.vstack([dX, E])
    k1 = fun(x, u)
    d1 = dk(x, I)
    X2 = x + 0.5 * h * k1
    k2 = fun(X2, u)
    d2 = dk(X2, I + 0.5 * h * d1)
    X3 = x + 0.5 * h * k2
    k3 = fun(X3, u)
    d3 = dk(X3, I + 0.5 * h * d2)
    X4 = x + h * k3
    d4 = dk(X4, I + h * d3)
    return I + h / 6.0 * (d1 + 2 * d2 + 2 * d3 + d4)


def main():
    rng = np.random.default_rng(20250124)
    flops = {}
    for nq in (1, 2, 3):
        m = extract(nq)
        xs, us, f = m["xs"], m["us"], m["f"]
        nx, nu = len(xs), len(us)
        z = sp.Matrix(xs + us)
        J = f.jacobian(z)
        f_num = sp.lambdify([xs, us], f, "numpy")
        J_num = sp.lambdify([xs, us], J, "numpy")
        npts = 64
        theta = rng.uniform(np.pi * 0.75 - 0.3, np.pi * 1.25 + 0.3, (npts, nq))
        omega = rng.uniform(-10, 10, (npts, nq))
        umax = 3.0 if nq == 1 else 10.0
        ctrl = rng.uniform(-umax, umax, (npts, nu))
        dt = np.full((npts, 1), 1e-2)
        X = np.concatenate([theta, omega, dt], axis=1)
        F = np.array([np.asarray(f_num(list(X[i]), list(ctrl[i])), dtype=float).ravel() for i in range(npts)])
        JJ = np.array([np.asarray(J_num(list(X[i]), list(ctrl[i])), dtype=float) for i in range(npts)])
        out = dict(x=X, u=ctrl, f=F, jac=JJ)
        # physics (un-scaled) rhs = f / dt; twin RK4 of the physics model, T = 1e-2
        phys = lambda x6, uu: np.asarray(
            f_num(list(np.append(x6, 1.0)), list(uu)), dtype=float).ravel()[: 2 * nq]
        if m["twin"] is not None:
            tw = sp.lambdify([m["twin_xs"], us], m["twin"], "numpy")
            twin = lambda x6, uu: np.asarray(tw(list(x6), list(uu)), dtype=float).ravel()
            T = np.array([twin(X[i, : 2 * nq], ctrl[i]) for i in range(npts)])
            out["twin_f"] = T
        else:
            twin = phys
        out["rk4_T"] = np.array(1e-2)
        out["rk4_x1"] = np.array([rk4(twin, X[i, : 2 * nq], ctrl[i], 1e-2) for i in range(npts)])
        # one shooting interval of the OCP model (dt state, tf/N = 1): RK4 with h = 1 on f
        fx = lambda x7, uu: np.asarray(f_num(list(x7), list(uu)), dtype=float).ravel()
        out["shoot_x1"] = np.array([rk4(fx, X[i], ctrl[i], 1.0) for i in range(npts)])
        # its Jacobian w.r.t. (x incl. the dt state, u): the free-time OCP's A_k | B_k
        out["shoot_jac"] = np.array([rk4_jac(fx, J_num, X[i], ctrl[i], 1.0) for i in range(npts)])
        out["consts"] = np.array(json.dumps(m["consts"]))
        np.savez(os.path.join(HERE, f"dynamics_{nq}.npz"), **out)
        flops[str(nq)] = {"C_f": cse_ops(list(f)), "C_fJ": cse_ops(list(f) + list(J)),
                          "nx": nx, "nu": nu, "consts": m["consts"]}
        print(nq, flops[str(nq)])
    with open(os.path.join(HERE, "flops.json"), "w") as fh:
        json.dump(flops, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    sys.exit(main())
