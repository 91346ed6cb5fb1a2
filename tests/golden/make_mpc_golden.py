"""Golden closed loops of the reference's Safe-MPC drivers (run HERE only, needs /root/reference).

`simulate(p)` is taken by AST (the function alone, parsed from the text) from
  VBOC/Safe MPC/hard_terminal_constraints/3dof_sym.py   (OCPtriplependulumHardTerm, SQP_RTI)
  VBOC/Safe MPC/soft_traj_constraints/3dof_sym.py       (OCPtriplependulumSoftTraj, Zl = 1e6 at N only)
  VBOC/Safe MPC/receiding_hard_constraints/3dof_sym.py  (OCPtriplependulumSoftTraj, receding weights per step)
and executed with injected globals:
  * `ocp`: an object with the OCP<...> surface those functions use - OCP_solve(x0, x_sol_guess, u_sol_guess),
    ocp.dims (nx, nu, N), ocp_solver.get(i, 'x' | 'u'), ocp_solver.cost_set(i, 'W' | 'Zl', ...) and
    nn_decisionfunction_conservative - whose OCP_solve solves on the CPU oracle (oracle/vboc_oracle_ft.c
    vboc_oracle_mpc_solve(_soft), test infrastructure) with the weights the driver set;
  * `sim`: SYMtriplependulum's integrator as one oracle RK4 step of time_step (records every applied (x, u));
  * `data`: the drivers' Halton initial positions (vboc_amd.safempc.halton_states); `x_sol_guess_vec` /
    `u_sol_guess_vec`: the reference loads ../x_sol_guess.npy, which is not in the repository - synthetic guesses
    (each problem's initial state held constant, zero torques) stand in;
  * `model`: the reference's trained model_3dof_vboc is not in the repository either - the tests' seeded
    NeuralNetDIR(6, 500, 1) with its output bias raised so the rows bind (tests/test_safempc.py _net), mean pi,
    std 0.5; safety_margin 2.0, time_step 4e-3, tot_time 0.148 (N = 37), as the drivers.
The fixture records, per problem, simulate's returned step and the applied plant inputs.  tests/test_safempc.py
runs vboc_amd.safempc.simulate_batch (the batched restatement of the three simulate functions) on the same oracle and
must reproduce it exactly; the GPU run is checked against it problem by problem.

Usage: python tests/golden/make_mpc_golden.py  ->  tests/golden/mpc_drivers.npz
"""
import ast
import json
import os
import sys
import time

import numpy as np
import scipy.linalg as lin

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
REF = "/root/reference/VBOC/Safe MPC"
DRIVERS = {"hard": "hard_terminal_constraints/3dof_sym.py", "soft": "soft_traj_constraints/3dof_sym.py",
           "receding": "receiding_hard_constraints/3dof_sym.py"}
TEST_NUM, TOT_STEPS, MARGIN = 24, 100, 2.0


def extract(path, name="simulate"):
    tree = ast.parse(open(path).read())
    fn = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name == name][0]
    return compile(ast.Module(body=[fn], type_ignores=[]), path, "exec")


class _Dims:
    def __init__(self, N):
        self.nx, self.nu, self.N = 6, 3, N


class _Ocp:
    def __init__(self, N):
        self.dims = _Dims(N)


class FakeSolver:
    def __init__(self, owner):
        self.o = owner
        self.x = self.u = None

    def get(self, i, field):
        return np.copy(self.x[i] if field == "x" else self.u[i])

    def cost_set(self, i, field, value):
        v = np.asarray(value, dtype=np.float64)
        if field == "Zl":
            self.o.Zl[i] = float(v.reshape(-1)[0])
        elif field == "W":
            assert np.abs(v - np.diag(np.diag(v))).max() == 0.0
            if i < self.o.N:
                self.o.W[i] = np.diag(v)
            else:
                self.o.We[:] = np.diag(v)
        else:
            raise NotImplementedError(field)


class FakeMpc:
    """The driver-facing surface of OCPtriplependulumHardTerm / SoftTraj on the oracle."""

    def __init__(self, spec, params, mean, std, soft):
        self.spec, self.params, self.mean, self.std, self.soft = spec, params, mean, std, soft
        self.N = spec.N
        self.ocp = _Ocp(spec.N)
        self.Zl = np.zeros(self.N + 1)
        self.W = np.tile(spec.W, (self.N, 1))
        self.We = spec.W_e.copy()
        self.ocp_solver = FakeSolver(self)

    def OCP_solve(self, x0, x_sol_guess, u_sol_guess):
        import oracle
        x0 = np.asarray(x0, float)[None]
        xg, ug = np.asarray(x_sol_guess, float)[None], np.asarray(u_sol_guess, float)[None]
        if self.soft:
            assert np.abs(self.W - self.W[0]).max() == 0.0
            x, u, r, _ = oracle.mpc_soft_solve_batch(self.spec, x0, xg, ug, self.params, self.mean, self.std, MARGIN,
                                                     self.Zl[None], W=self.W[0][None], We=self.We[None], rti=True,
                                                     nthreads=1)
        else:
            x, u, r, _ = oracle.mpc_solve_batch(self.spec, x0, xg, ug, self.params, mean=self.mean, std=self.std,
                                                rti=True, nthreads=1)
        self.ocp_solver.x, self.ocp_solver.u = x[0], u[0]
        return int(r["status"][0])

    def nn_decisionfunction_conservative(self, params, mean, std, safety_margin, x):
        import oracle
        return float(oracle.mpc_row(np.asarray(x, float), self.params, self.mean, self.std, safety_margin)[0])


class FakeIntegrator:
    def __init__(self, h, log):
        self.h, self.log, self.x, self.u = h, log, None, None

    def set(self, field, v):
        setattr(self, field, np.array(v, dtype=np.float64))

    def solve(self):
        import oracle
        self.log.append(np.r_[self.x, self.u].tolist())
        self.out = oracle.rk4(3, self.h, self.x, self.u)
        return 0

    def get(self, field):
        return np.copy(self.out)


class FakeSim:
    def __init__(self, h, log):
        self.acados_integrator = FakeIntegrator(h, log)


def run(kind, ps):
    from test_safempc import MEAN, STD, _net
    from vboc_amd.safempc import MpcSpec, halton_states
    spec = MpcSpec(4e-3, 0.148)
    P = _net()
    data = halton_states(spec, TEST_NUM)[:, :3]
    xg = np.repeat(halton_states(spec, TEST_NUM)[:, None, :], spec.N + 1, 1)
    ug = np.zeros((TEST_NUM, spec.N, 3))
    out = []
    for p in ps:
        log = []
        ocp = FakeMpc(spec, P, MEAN, STD, kind != "hard")
        if kind == "soft":   # the soft_traj driver's main block, before the fan-out (:102-105)
            for i in range(1, spec.N):
                ocp.ocp_solver.cost_set(i, "Zl", 0 * np.ones((1,)))
            ocp.ocp_solver.cost_set(spec.N, "Zl", 1e6 * np.ones((1,)))
        g = dict(np=np, time=time, lin=lin, ocp=ocp,
                 sim=FakeSim(spec.time_step, log), data=data, x_sol_guess_vec=xg.copy(), u_sol_guess_vec=ug.copy(),
                 tot_steps=TOT_STEPS, N=spec.N, params=P, mean=MEAN, std=STD, safety_margin=MARGIN)
        exec(extract(os.path.join(REF, DRIVERS[kind])), g)
        f, _ = g["simulate"](p)
        out.append(dict(p=int(p), res=int(f), applied=log))
    return out


def main():
    from multiprocessing import Pool
    res = {}
    for kind in DRIVERS:
        chunks = [list(range(i, TEST_NUM, 8)) for i in range(8)]
        with Pool(8) as pool:
            parts = pool.starmap(run, [(kind, c) for c in chunks])
        res[kind] = sorted([r for part in parts for r in part], key=lambda r: r["p"])
        print(kind, [r["res"] for r in res[kind]], flush=True)
    arrays = {}
    for kind, rs in res.items():
        arrays[f"{kind}_res"] = np.array([r["res"] for r in rs])
        A = np.full((TEST_NUM, TOT_STEPS, 9), np.nan)
        for j, r in enumerate(rs):
            A[j, :len(r["applied"])] = r["applied"]
        arrays[f"{kind}_applied"] = A   # [p, step, (x (6), u (3))] fed to the plant; NaN after the stop
    np.savez_compressed(os.path.join(HERE, "mpc_drivers.npz"), test_num=TEST_NUM, tot_steps=TOT_STEPS,
                        margin=MARGIN, **arrays)


if __name__ == "__main__":
    main()
