"""Test-only backends that put the CPU oracle (oracle/, test infrastructure) behind the product's two
solver interfaces, so the reference's own driver code and the batched drivers can be checked on the
same solver results:
  * OracleBackend     - the vboc_amd.drivers backend interface (solve(batch), rk4(x, u, T));
  * OracleOcpBackend  - the vboc_amd.ocp.use_backend interface (solve_host(batch), rk4(nq, T, x, u)),
                        i.e. the drop-in OCP<sys>INIT classes solving on the oracle.
Never imported by the product path."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))


def forced_failure(q0, fail_mod):
    """Deterministic failure injection (exercises the drivers' restart branches, which the oracle
    rarely reaches on its own): a solve whose initial position has int(|q_0| 1e6) divisible by
    `fail_mod` reports status 4 (ACADOS 'QP failure').  A restart perturbs q_0, so it can succeed."""
    return fail_mod > 0 and int(abs(float(q0)) * 1e6) % fail_mod == 0


def _oracle_solve(nq, b, fail_mod=0, free_time=False, hc=None):
    import oracle
    o = None
    if hc is not None:
        o = oracle.default_opts(hc=1, hc_xc=hc.x_c, hc_yc=hc.y_c, hc_lh=hc.lh, hc_uh=hc.uh)
    xo, uo, r = oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"],
                                   b["lbu"], b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"],
                                   opts=o, free_time=free_time)
    st = np.array(r["status"], copy=True)
    for i in range(st.shape[0]):
        if forced_failure(b["lbx0"][i, 0], fail_mod):
            st[i] = 4
    return dict(status=st, x=xo, u=uo, cost=r["cost"], sqp_iter=r["sqp_iter"], qp_iter=r["qp_iter"])


class OracleBackend:
    """Batched drivers' backend on the oracle."""
    nmax = 512

    def __init__(self, nq, fail_mod=0, path_constraint=None):
        self.nq, self.fail_mod, self.hc = nq, fail_mod, path_constraint

    def solve(self, b, free_time=False):
        return _oracle_solve(self.nq, b, self.fail_mod, free_time, self.hc)

    def rk4(self, x, u, T):
        import oracle
        return np.stack([oracle.rk4(self.nq, T, x[i], u[i]) for i in range(x.shape[0])])


class OracleOcpBackend:
    """Drop-in classes' backend on the oracle (vboc_amd.ocp.use_backend)."""

    def __init__(self, fail_mod=0, path_constraint=None):
        self.fail_mod, self.hc = fail_mod, path_constraint

    def with_path_constraint(self, c):
        return OracleOcpBackend(self.fail_mod, c)

    def solve_host(self, b, free_time=False):
        nq = b["u_guess"].shape[2]
        return _oracle_solve(nq, b, self.fail_mod, free_time, self.hc)

    def rk4(self, nq, T, x, u):
        import oracle
        return oracle.rk4(nq, T, x, u)
