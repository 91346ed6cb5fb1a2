"""GPU parity tests: the HIP solver (through the C ABI) against the CPU oracle on the same seeded
inputs, plus size-independent properties at larger sizes.  All marked `gpu`.

Tolerances (FP64 everywhere): identical algorithm, different operation order / FMA contraction /
libm, so results agree to rounding except where a rounding-level difference flips an SQP decision
(line-search acceptance); then both runs still converge to a KKT point within the solver
tolerance.  Stated bars:
  * status agreement >= 98% of problems, SQP-iteration agreement >= 95%;
  * problems converged on both: |cost_gpu - cost_cpu| median <= 1e-9, max <= 2e-3 (nlp tol_stat
    1e-3); boundary state x0 the same bar;
  * twin RK4 step vs the golden vectors from the reference expressions: 1e-13.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(nq, b, **opts):
    import oracle
    o = oracle.default_opts(**opts)
    return oracle.solve_batch(nq, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                              b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], opts=o)


def _gpu(nq, b, **opts):
    from vboc_amd import lib
    s = lib.Solver(nq, int(np.max(b["N"])), slots=opts.pop("slots", 1024))
    for k, v in opts.items():
        s.set_option(k, v)
    try:
        return s.solve_host(b)
    finally:
        s.close()


def _compare(nq, b, max_iter, coop=8192, wave=0, **opts):
    g = _gpu(nq, b, nlp_solver_max_iter=max_iter, coop_threshold=coop, wave_all=wave, **opts)
    xo, uo, r = _oracle(nq, b, max_iter=max_iter)
    assert np.mean(g["status"] == r["status"]) >= 0.98, (g["status"], r["status"])
    assert np.mean(g["sqp_iter"] == r["sqp_iter"]) >= 0.95
    both = (g["status"] == 0) & (r["status"] == 0)
    assert both.sum() >= 0.5 * len(both)
    dc = np.abs(g["cost"] - r["cost"])[both]
    dx = np.abs(g["x"][:, 0, :2 * nq] - xo[:, 0, :2 * nq]).max(axis=1)[both]
    assert np.median(dc) <= 1e-9 and dc.max() <= 2e-3, (np.median(dc), dc.max())
    assert np.median(dx) <= 1e-9 and dx.max() <= 2e-3
    # dt column and untouched rows follow the reference layout
    for i in np.where(both)[0][:8]:
        N = b["N"][i]
        np.testing.assert_array_equal(g["x"][i, :N + 1, 2 * nq], b["lbx"][i, 2 * nq])
    return g, r


# mode "lane": every SQP iteration in the lane-per-problem kernels (coop_threshold 0);
# mode "coop": 4 lane-mode rounds, then the wave solver (coop.h) takes over every problem still
# iterating (the queue of these small batches is drained at once);
# mode "wave": every problem solved start-to-end by the wave solver (wave_all).
@pytest.mark.parametrize("mode", ["lane", "coop", "wave"])
@pytest.mark.parametrize("nq,law,B", [(1, "heldout", 256), (2, "dg", 128), (3, "heldout", 96), (3, "dg", 96)])
def test_parity_with_oracle(nq, law, B, mode):
    from vboc_amd.ics import data_generation_ics, heldout_ics
    b = (data_generation_ics if law == "dg" else heldout_ics)(nq, np.arange(B))
    _compare(nq, b, max_iter=200 if nq == 3 else 1000, coop=0 if mode == "lane" else 1e9,
             wave=1 if mode == "wave" else 0)


def test_coop_tail_is_used():
    from vboc_amd import lib
    from vboc_amd.ics import heldout_ics
    b = heldout_ics(3, np.arange(64))
    s = lib.Solver(3, 100, slots=256)
    assert s.get_option("coop_available") == 1.0
    assert s.get_option("wave_all") == 1.0          # default: every problem on the wave solver
    s.set_option("wave_all", 0)
    s.set_option("coop_threshold", 1e9)
    s.solve_host(b)
    assert s.get_option("coop_problems") > 0
    s.set_option("coop_threshold", 0)
    s.solve_host(b)
    assert s.get_option("coop_problems") == 0
    s.set_option("wave_all", 1)
    s.solve_host(b)
    assert s.get_option("coop_problems") == 64
    s.close()


def test_parity_ragged_horizons():
    """Per-problem horizons inside one batch (the drivers' N+1 extensions / verification OCPs)."""
    from vboc_amd.ics import data_generation_ics
    parts = []
    for j, N in enumerate((37, 100, 103, 64)):
        parts.append(data_generation_ics(3, np.arange(16 * j, 16 * j + 16), N=N))
    Nmax = 103
    b = {}
    for k in parts[0]:
        if k in ("joint_sel", "vel_sel"):
            continue
        arrs = []
        for p in parts:
            a = p[k]
            if k == "x_guess":
                a = np.concatenate([a, np.repeat(a[:, -1:], Nmax + 1 - a.shape[1], 1)], 1)
            if k == "u_guess":
                a = np.concatenate([a, np.zeros((a.shape[0], Nmax - a.shape[1], a.shape[2]))], 1)
            arrs.append(a)
        b[k] = np.concatenate(arrs)
    _compare(3, b, max_iter=150, coop=0)
    _compare(3, b, max_iter=150, coop=1e9)
    _compare(3, b, max_iter=150, wave=1)


def test_twin_integrator_matches_golden():
    import os
    from vboc_amd import lib
    for nq in (1, 2, 3):
        g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"dynamics_{nq}.npz"))
        x1 = lib.rk4_host(nq, float(g["rk4_T"]), g["x"][:, :2 * nq], g["u"])
        np.testing.assert_allclose(x1, g["rk4_x1"], rtol=1e-13, atol=1e-13)


def test_device_path_equals_host_path():
    import torch
    from vboc_amd import lib
    from vboc_amd.ics import heldout_ics
    b = heldout_ics(2, np.arange(64))
    s = lib.Solver(2, 100, slots=256)
    host = s.solve_host(b)
    dev = {k: torch.as_tensor(np.ascontiguousarray(b[k]), device="cuda") for k in lib.FIELDS_IN + ("N",)}
    out = s.solve_device(dev)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), host["status"])
    np.testing.assert_array_equal(out["x"].cpu().numpy(), host["x"])
    s.close()


def test_unsupported_structure_is_reported_per_problem():
    from vboc_amd import lib
    from vboc_amd.ics import heldout_ics
    b = heldout_ics(3, np.arange(8))
    b["ubx"] = b["ubx"].copy()
    b["ubx"][3, 6] = 2e-2           # free time: dt not pinned
    b["ubx0"] = b["ubx0"].copy()
    b["ubx0"][5, 1] += 0.1          # stage-0 position not fixed
    g = _gpu(3, b, nlp_solver_max_iter=100)
    assert g["status"][3] == 5 and g["status"][5] == 5
    assert np.all(np.isin(g["status"][[0, 1, 2, 4, 6, 7]], [0, 2]))


def test_error_codes():
    import ctypes
    from vboc_amd import lib
    so = lib.load()
    h = ctypes.c_void_p()
    assert so.vboc_create(3, 100, 256, 0, ctypes.byref(h)) == 0
    assert so.vboc_set_option(h, b"no_such_option", ctypes.c_double(1.0)) == -1
    assert b"no_such_option" in so.vboc_last_error()
    assert so.vboc_solve_batch(h, None, None) == -1
    so.vboc_destroy(h)


def test_dropin_ocp_class_matches_oracle():
    """OCPtriplependulumINIT.OCP_solve with the reference driver's first-solve arrays."""
    from vboc_amd.ics import data_generation_ics
    from vboc_amd.ocp import OCPtriplependulumINIT
    b = data_generation_ics(3, np.arange(3))
    ocp = OCPtriplependulumINIT()
    xo, uo, r = _oracle(3, b)
    for i in range(3):
        N = ocp.N
        st = ocp.OCP_solve(b["x_guess"][i, :N], b["u_guess"][i, :N], b["p"][i], b["lbx"][i], b["ubx"][i],
                           b["lbu"][i], b["ubu"][i], b["lbx0"][i], b["ubx0"][i], b["lbxe"][i], b["ubxe"][i])
        assert st == r["status"][i]
        if st == 0:
            assert abs(ocp.ocp_solver.get_cost() - r["cost"][i]) < 2e-3
            np.testing.assert_allclose(ocp.ocp_solver.get(0, "x"), xo[i, 0], atol=2e-3)


def test_full_batch_properties():
    """Size-independent properties on a 16k-problem batch (beyond what the oracle can check in
    seconds): every converged solution is dynamically feasible (re-simulated with the GPU twin
    RK4), inside the boxes, ends at rest, starts along the cost direction, and the cost is the
    boundary velocity along -p."""
    from vboc_amd import lib
    from vboc_amd.ics import data_generation_ics
    nq, B = 3, 16384
    b = data_generation_ics(nq, np.arange(10**6, 10**6 + B))
    g = _gpu(nq, b, nlp_solver_max_iter=60)
    ok = g["status"] == 0
    assert ok.mean() > 0.5
    X = g["x"][ok, :, :2 * nq]
    U = g["u"][ok]
    N = 100
    x1 = lib.rk4_host(nq, 1e-2, X[:, :N].reshape(-1, 2 * nq), U[:, :N].reshape(-1, nq)).reshape(-1, N, 2 * nq)
    assert np.abs(x1 - X[:, 1:N + 1]).max() < 1e-6
    assert np.abs(X[:, N, nq:]).max() < 1e-6
    assert np.all(np.abs(U) <= 10 + 1e-6) and np.all(np.abs(X[:, 1:N, nq:]) <= 10 + 1e-6)
    assert np.all(X[:, 1:N, :nq] >= b["lbx"][0, 0] - 1e-6) and np.all(X[:, 1:N, :nq] <= b["ubx"][0, 0] + 1e-6)
    d = b["p"][ok, :nq] / np.linalg.norm(b["p"][ok, :nq], axis=1, keepdims=True)
    v0 = X[:, 0, nq:]
    assert np.abs(v0 - d * np.sum(d * v0, 1, keepdims=True)).max() < 1e-9
    np.testing.assert_allclose(g["cost"][ok], np.sum(b["p"][ok, :nq] * v0, 1), atol=1e-9)


# ---- free-time OCP (OCPpendulum.OCP_solve, vboc_solve_batch_ft) --------------------------------------
def _ft_batch(B, N_range=(20, 60)):
    from vboc_amd.ics import pendulum_free_time_ics
    return pendulum_free_time_ics(np.arange(B), N_range)


def test_free_time_parity_with_oracle():
    """Same bars as the boundary solver (module docstring), on free-time pendulum OCPs."""
    import oracle
    from vboc_amd import lib
    b = _ft_batch(256)
    s = lib.Solver(1, int(b["N"].max()))
    g = s.solve_host(b, free_time=True)
    s.close()
    xo, uo, r = oracle.solve_batch(1, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], free_time=True)
    assert np.mean(g["status"] == r["status"]) >= 0.98, (g["status"], r["status"])
    assert np.mean(g["sqp_iter"] == r["sqp_iter"]) >= 0.95
    both = (g["status"] == 0) & (r["status"] == 0)
    assert both.mean() >= 0.9
    dc = np.abs(g["cost"] - r["cost"])[both]
    dx = np.abs(g["x"][:, 0] - xo[:, 0]).max(axis=1)[both]
    assert np.median(dc) <= 1e-9 and dc.max() <= 2e-3, (np.median(dc), dc.max())
    assert np.median(dx) <= 1e-9 and dx.max() <= 2e-3
    # one dt along every solution, rest at q_fin
    for i in np.where(both)[0][:16]:
        N = b["N"][i]
        assert np.ptp(g["x"][i, :N + 1, 2]) < 1e-9
        assert abs(g["x"][i, N, 0] - b["lbxe"][i, 0]) < 1e-6 and abs(g["x"][i, N, 1]) < 1e-6


def test_free_time_infinite_bounds_are_a_free_component():
    """A path component with both bounds infinite is free (no barrier terms, not counted in the centring target) on
    the GPU as in the oracle's fcomp (the non-MP instantiation once treated it as boxed)."""
    import oracle
    from vboc_amd import lib
    b = _ft_batch(64)
    b["lbx"][:, 1], b["ubx"][:, 1] = -np.inf, np.inf       # the velocity unbounded on the path
    s = lib.Solver(1, int(b["N"].max()))
    g = s.solve_host(b, free_time=True)
    s.close()
    xo, uo, r = oracle.solve_batch(1, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], free_time=True)
    assert np.mean(g["status"] == r["status"]) >= 0.98
    assert np.mean(g["sqp_iter"] == r["sqp_iter"]) >= 0.95
    both = (g["status"] == 0) & (r["status"] == 0)
    assert both.mean() >= 0.8
    dc = np.abs(g["cost"] - r["cost"])[both]
    assert np.median(dc) <= 1e-9 and dc.max() <= 2e-3, (np.median(dc), dc.max())


def test_free_time_device_path_and_unsupported():
    import torch
    from vboc_amd import lib
    b = _ft_batch(64)
    b["lbx"][3, 1] = b["ubx"][3, 1]            # a pinned path component: outside the free-time structure
    s = lib.Solver(1, int(b["N"].max()))
    h = s.solve_host(b, free_time=True)
    dev = {k: torch.as_tensor(np.ascontiguousarray(v), device="cuda:0") for k, v in b.items()}
    d = s.solve_device(dev, free_time=True)
    torch.cuda.synchronize()
    s.close()
    assert h["status"][3] == 5 and d["status"][3].item() == 5
    np.testing.assert_array_equal(h["status"], d["status"].cpu().numpy())
    np.testing.assert_array_equal(h["x"], d["x"].cpu().numpy())
    np.testing.assert_array_equal(h["cost"], d["cost"].cpu().numpy())


def test_dropin_pendulum_ocp_solve_on_gpu():
    import oracle
    from vboc_amd import ocp
    b = _ft_batch(4, (50, 50))
    xo, uo, r = oracle.solve_batch(1, b["N"], b["x_guess"], b["u_guess"], b["p"], b["lbx"], b["ubx"], b["lbu"],
                                   b["ubu"], b["lbx0"], b["ubx0"], b["lbxe"], b["ubxe"], free_time=True)
    o = ocp.OCPpendulum()
    for i in range(4):
        st = o.OCP_solve(b["x_guess"][i], b["u_guess"][i], b["p"][i, 0], b["lbx"][i], b["ubx"][i],
                         b["lbx0"][i, 0], b["lbxe"][i, 0])
        assert st == r["status"][i]
        if st == 0:
            assert abs(o.ocp_solver.get_cost() - r["cost"][i]) < 1e-6
            np.testing.assert_allclose(o.ocp_solver.get(0, "x"), xo[i, 0], atol=1e-6)


def test_pendulum_data_generation_on_gpu_matches_reference_loop():
    """VBOC/pendulum_vboc.py:52-205 through the batched driver on the GPU against the fixture of the
    reference's own loop (oracle-backed): same samples to 1e-6."""
    import json
    import os
    from vboc_amd.drivers import GpuBackend, pendulum_data_generation
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "driver_1.json")))
    X, stats = pendulum_data_generation(GpuBackend(1, nmax=200), fx["N_start"], fx["eps"])
    G = np.array(fx["X_save"])
    assert X.shape == G.shape
    np.testing.assert_allclose(X, G, atol=1e-6)


def test_pendulum_vboc_run_on_gpu(tmp_path):
    """VBOC/pendulum_vboc.py's main block on one MI355X: free-time data generation on the HIP solver,
    the 2-100-1 fit replayed from a HIP graph with the reference's stop rule, RMSE, artefacts."""
    from vboc_amd.pipeline import pendulum_vboc_run
    r = pendulum_vboc_run(str(tmp_path), device="cuda")
    assert r["X"].shape[0] > 50
    assert r["fit"]["val"] <= 1e-4 or r["fit"]["iterations"] >= 100 * int(r["X"].shape[0] * 100 / 64)
    assert r["rmse"] < 1.0
    assert (tmp_path / "model_1dof_vboc_10").exists()


# problems of the data_generation first-solve law whose oracle SQP runs the longest (found with
# oracle.solve_batch over ids 0..1535, max_iter 1000): 988 and 358 stop at max_iter (status 2), 832 / 1464 /
# 703 / 125 / 73 converge after 701 / 664 / 632 / 556 / 519 iterations
LONG_TAIL = (988, 358, 832, 1464, 703, 125, 73)


@pytest.mark.parametrize("factor", ["mfma", "valu"])
def test_parity_triple_full_iteration_budget_with_long_tail(factor):
    """The triple at the reference's nlp_solver_max_iter = 1000 (VBOC/triplependulum_class_vboc.py:136) on
    a batch holding the long-tail problems the bench hits, on the default wave solver (both Riccati
    factorisations)."""
    from vboc_amd.ics import data_generation_ics
    ids = np.concatenate([np.arange(40), LONG_TAIL])
    b = data_generation_ics(3, ids)
    g, r = _compare(3, b, max_iter=1000, wave=1, factor_mfma=1 if factor == "mfma" else 0)
    tail = np.arange(40, len(ids))
    assert (g["status"][tail] == r["status"][tail]).all(), (g["status"][tail], r["status"][tail])
    assert (r["sqp_iter"][tail] >= 500).all()
    ok = tail[r["status"][tail] == 0]
    assert np.abs(g["cost"][ok] - r["cost"][ok]).max() <= 2e-3


@pytest.mark.parametrize("nq", [1, 2, 3])
def test_shooting_sensitivities_match_golden(nq):
    """The solvers' linearisation (ERK4 + forward sensitivities, vboc_rk4_sens_batch_host) against the
    golden shooting Jacobians from the reference's own f_expl (tests/golden/make_golden.py: RK4 with
    h = 1 on the dt-scaled model, tf / N = 1): A = d x1 / d x, B = d x1 / d u without the dt row/column."""
    import os
    from vboc_amd import lib
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", f"dynamics_{nq}.npz"))
    nx = 2 * nq
    for i in range(g["x"].shape[0]):
        x, u = g["x"][i], g["u"][i]
        x1, A, B = lib.rk4_sens_host(nq, float(x[nx]), x[None, :nx], u[None])
        np.testing.assert_allclose(x1[0], g["shoot_x1"][i, :nx], rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(A[0], g["shoot_jac"][i][:nx, :nx], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(B[0], g["shoot_jac"][i][:nx, nx + 1:], rtol=1e-10, atol=1e-12)
