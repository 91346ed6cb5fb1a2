"""Deterministic, GPU-count-independent initial conditions for the boundary OCPs.

The reference draws ICs with Python's global `random` inside each forked worker (unseeded,
VBOC/triplependulum_vboc.py:33-73, triplependulum_testdata.py:19-28).  Here every problem id
gets its own Philox4x32-10 stream keyed by (seed, problem id), so the union of the ICs solved
on 1, 2, 4 or 8 GPUs is identical and any shard can be regenerated.

Laws implemented (each returns the arrays OCP_solve / the ocp_solver API would receive):
  * `data_generation_ics(nq, ids)`: the first solve of `data_generation`
    (VBOC/triplependulum_vboc.py:32-103, VBOC/doublependulum_vboc.py:33-96) - reference joint at
    q_min+eps / q_max-eps, other joints ~U clamped by eps, random unit cost direction with the
    reference component's sign fixed by vel_sel, straight-line guess over N rows.
  * `heldout_ics(nq, ids)`: `testing` (triplependulum_testdata.py:19-38,
    doublependulum_testdata.py, pendulum_testdata.py:14-27) - uniform interior IC, random unit
    direction, constant guess.
"""
import numpy as np

from .systems import system

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)

SEED = 20250124


def philox4x32(counter, key):
    """Philox4x32-10.  counter: (..., 4) uint32-valued uint64 array, key: (2,) ints.
    Returns (..., 4) uint64 array of 32-bit outputs."""
    c = [counter[..., i].astype(np.uint64) & _MASK for i in range(4)]
    k0, k1 = np.uint64(key[0]) & _MASK, np.uint64(key[1]) & _MASK
    for _ in range(10):
        p0 = _M0 * c[0]
        p1 = _M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c = [(hi1 ^ c[1] ^ k0) & _MASK, lo1, (hi0 ^ c[3] ^ k1) & _MASK, lo0]
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return np.stack(c, axis=-1)


def uniforms(ids, n, seed=SEED, stream=0):
    """n independent U[0,1) doubles (53-bit) per problem id -> (len(ids), n)."""
    ids = np.asarray(ids, dtype=np.uint64)
    nblk = (n + 1) // 2
    ctr = np.zeros((ids.shape[0], nblk, 4), dtype=np.uint64)
    ctr[..., 0] = (ids & _MASK)[:, None]
    ctr[..., 1] = (ids >> np.uint64(32))[:, None]
    ctr[..., 2] = np.arange(nblk, dtype=np.uint64)[None, :]
    ctr[..., 3] = np.uint64(stream)
    r = philox4x32(ctr, (seed & 0xFFFFFFFF, (seed >> 32) ^ 0x5BD1E995))
    a = (r[..., 0::2] >> np.uint64(5)).astype(np.float64)   # 27 bits
    b = (r[..., 1::2] >> np.uint64(6)).astype(np.float64)   # 26 bits
    u = (a * 67108864.0 + b) / 9007199254740992.0
    return u.reshape(ids.shape[0], -1)[:, :n]


def _row_norms(r):
    """Per-row 2-norms computed as the reference does, numpy.linalg.norm of each 1-D vector
    (triplependulum_vboc.py:48): the axis=1 reduction rounds differently in the last bit."""
    return np.array([[np.linalg.norm(row)] for row in r]).reshape(r.shape[0], 1)


def _choice(u, options):
    options = np.asarray(options)
    return options[np.minimum((u * len(options)).astype(np.int64), len(options) - 1)]


class Batch(dict):
    """Arrays of one batched solve in the reference layout (problem-major)."""


def data_generation_ics(nq, ids, N=None, seed=SEED):
    """First OCP of `data_generation` for each id (VBOC/triplependulum_vboc.py:32-103)."""
    sysd = system(nq)
    N = N or sysd.N
    ids = np.asarray(ids)
    B = ids.shape[0]
    q_min, q_max, v_max, tau, dt, eps = sysd.q_min, sysd.q_max, sysd.v_max, sysd.u_max, sysd.dt, sysd.eps
    U = uniforms(ids, 3 * nq + 1, seed)
    joint_sel = _choice(U[:, 0], list(range(nq))) if nq > 1 else np.zeros(B, dtype=np.int64)
    vel_sel = _choice(U[:, 1], [-1.0, 1.0])
    q_init_sel = np.where(vel_sel == -1, q_min, q_max)
    q_fin_sel = np.where(vel_sel == -1, q_max, q_min)
    # cost direction: ran1 carries vel_sel; the others random sign (:45-54)
    rans = [vel_sel * U[:, 2]]
    for j in range(1, nq):
        rans.append(_choice(U[:, 2 + 2 * j - 1], [-1.0, 1.0]) * U[:, 2 + 2 * j])
    rans = np.stack(rans, axis=1)
    rans /= _row_norms(rans)
    p = np.zeros((B, nq + 1))
    # joint_sel == j: p = [others..., ran1 at position j] following :49-54 / double :45-50
    for j in range(nq):
        m = joint_sel == j
        order = list(range(1, nq))  # ran2, ran3 fill the non-selected joints in order
        cols = [c for c in range(nq) if c != j]
        p[m, j] = rans[m, 0]
        for c, o in zip(cols, order):
            p[m, c] = rans[m, o]
    # positions of the other joints ~U, clamped by eps (:57-73): the triple draws one per joint
    # (draws 8-10), the double one for the other joint (its 6th draw, VBOC/doublependulum_vboc.py:56)
    qi = np.zeros((B, nq))
    for j in range(nq):
        col = 2 * nq + 1 + j if nq != 2 else 2 * nq + 1
        v = q_min + U[:, col] * (q_max - q_min)
        v = np.where(v > q_max - eps, v - eps, v)
        v = np.where(v < q_min + eps, v + eps, v)
        qi[:, j] = v
    nxr = 2 * nq + 1
    lbx0 = np.concatenate([qi, np.full((B, nq), -v_max), np.full((B, 1), dt)], axis=1)
    ubx0 = np.concatenate([qi, np.full((B, nq), v_max), np.full((B, 1), dt)], axis=1)
    rows = np.arange(B)
    lbx0[rows, joint_sel] = np.where(q_init_sel == q_min, q_min + eps, q_max - eps)
    ubx0[rows, joint_sel] = lbx0[rows, joint_sel]
    # straight-line guess over N rows (:85-93); the stage-N guess is row N-1 (class :185)
    tau_grid = np.linspace(0.0, 1.0, N)
    xg = np.zeros((B, N + 1, nxr))
    xg[:, :N, :nq] = qi[:, None, :]
    xg[:, :N, 2 * nq] = dt
    xg[rows[:, None], np.arange(N)[None, :], joint_sel[:, None]] = \
        (1 - tau_grid)[None, :] * q_init_sel[:, None] + tau_grid[None, :] * q_fin_sel[:, None]
    xg[rows[:, None], np.arange(N)[None, :], (joint_sel + nq)[:, None]] = \
        2 * (1 - tau_grid)[None, :] * (q_fin_sel - q_init_sel)[:, None]
    xg[:, N] = xg[:, N - 1]
    ug = np.zeros((B, N, nq))
    if sysd.gravity_guess:
        # double pendulum guess u = gravity compensation (VBOC/doublependulum_vboc.py:84)
        ug[:, :, 0] = sysd.g * sysd.l[0] * (sysd.m[0] + sysd.m[1]) * np.sin(xg[:, :N, 0])
        ug[:, :, 1] = sysd.g * sysd.l[1] * sysd.m[1] * np.sin(xg[:, :N, 1])
    return _bounds(sysd, B, N, xg, ug, p, lbx0, ubx0, extra=dict(joint_sel=joint_sel, vel_sel=vel_sel))


def heldout_ics(nq, ids, N=None, seed=SEED):
    """`testing` (triplependulum_testdata.py:19-38): uniform interior IC, unit direction."""
    sysd = system(nq)
    N = N or sysd.N
    ids = np.asarray(ids)
    B = ids.shape[0]
    U = uniforms(ids, 3 * nq + 1, seed, stream=1)
    if nq == 1:
        p = np.zeros((B, 2))
        p[:, 0] = _choice(U[:, 0], [-1.0, 1.0])
    else:
        r = np.stack([_choice(U[:, 2 * j], [-1.0, 1.0]) * U[:, 2 * j + 1] for j in range(nq)], axis=1)
        p = np.zeros((B, nq + 1))
        p[:, :nq] = r / _row_norms(r)
    # draw order of the reference: (choice, random) per joint, then one position per joint; the
    # pendulum draws choice, then its position (pendulum_testdata.py:14-18)
    qi = sysd.q_min + (U[:, 1:2] if nq == 1 else U[:, 2 * nq: 3 * nq]) * (sysd.q_max - sysd.q_min)
    dt = sysd.dt
    lbx0 = np.concatenate([qi, np.full((B, nq), -sysd.v_max), np.full((B, 1), dt)], axis=1)
    ubx0 = np.concatenate([qi, np.full((B, nq), sysd.v_max), np.full((B, 1), dt)], axis=1)
    xg = np.zeros((B, N + 1, 2 * nq + 1))
    xg[:, :, :nq] = qi[:, None, :]
    xg[:, :, 2 * nq] = dt
    ug = np.zeros((B, N, nq))
    if sysd.gravity_guess:
        # double pendulum: constant gravity-compensation guess (doublependulum_testdata.py:37), with
        # the reference's scalar math.sin
        import math
        ug[:, :, 0] = (sysd.g * sysd.l[0] * (sysd.m[0] + sysd.m[1]) * np.array([math.sin(q) for q in qi[:, 0]]))[:, None]
        ug[:, :, 1] = (sysd.g * sysd.l[1] * sysd.m[1] * np.array([math.sin(q) for q in qi[:, 1]]))[:, None]
    return _bounds(sysd, B, N, xg, ug, p, lbx0, ubx0)


def _bounds(sysd, B, N, xg, ug, p, lbx0, ubx0, extra=None):
    nq = sysd.nq
    dt = sysd.dt
    lbx = np.tile(np.r_[[sysd.q_min] * nq, [-sysd.v_max] * nq, [dt]], (B, 1))
    ubx = np.tile(np.r_[[sysd.q_max] * nq, [sysd.v_max] * nq, [dt]], (B, 1))
    lbu = np.full((B, nq), -sysd.u_max)
    ubu = np.full((B, nq), sysd.u_max)
    lbxe = np.tile(np.r_[[sysd.q_min] * nq, [0.0] * nq, [dt]], (B, 1))
    ubxe = np.tile(np.r_[[sysd.q_max] * nq, [0.0] * nq, [dt]], (B, 1))
    b = Batch(N=np.full(B, N, dtype=np.int32), x_guess=xg, u_guess=ug, p=p, lbx=lbx, ubx=ubx,
              lbu=lbu, ubu=ubu, lbx0=lbx0, ubx0=ubx0, lbxe=lbxe, ubxe=ubxe)
    if extra:
        b.update(extra)
    return b


UR5_DRAWS = 12   # testing_test: (random, choice) per joint for p, one random per joint for q_init
UR5_STREAM = 5


def ur5_ics(ids, N=100, seed=SEED):
    """First OCP of the UR5's `testing_test` (VBOC/UR5/vboc_multiprocessing_ur5.py:369-426), what its main
    block fans out for the test and training sets (:487-511): p[l] = random() * choice([-1, 1]),
    normalised; q_init ~ U(x_min, x_max) per joint (x_max[1] = 0); constant guess [q_init, 0]; u = 0.
    9-column C-ABI layout (the UR5 time step 1e-2 pinned in the dt column, p padded with 0)."""
    from .ur5 import DT, NQ, U_LIMITS, XMAX, XMIN
    ids = np.asarray(ids)
    B = ids.shape[0]
    U = uniforms(ids, UR5_DRAWS, seed, stream=UR5_STREAM)
    r = np.stack([U[:, 2 * j] * _choice(U[:, 2 * j + 1], [-1.0, 1.0]) for j in range(NQ)], axis=1)
    p = np.zeros((B, NQ + 1))
    p[:, :NQ] = r / _row_norms(r)
    qi = XMIN[:NQ] + U[:, 2 * NQ:3 * NQ] * (XMAX[:NQ] - XMIN[:NQ])
    col = lambda a: np.concatenate([a, np.full(a.shape[:-1] + (1,), DT)], axis=-1)
    xg = np.zeros((B, N + 1, 2 * NQ + 1))
    xg[:, :, :NQ] = qi[:, None, :]
    xg[:, :, 2 * NQ] = DT
    return Batch(N=np.full(B, N, dtype=np.int32), x_guess=xg, u_guess=np.zeros((B, N, NQ)), p=p,
                 lbx=np.tile(col(XMIN), (B, 1)), ubx=np.tile(col(XMAX), (B, 1)),
                 lbu=np.tile(-U_LIMITS, (B, 1)), ubu=np.tile(U_LIMITS, (B, 1)),
                 lbx0=col(np.concatenate([qi, np.tile(XMIN[NQ:], (B, 1))], axis=1)),
                 ubx0=col(np.concatenate([qi, np.tile(XMAX[NQ:], (B, 1))], axis=1)),
                 lbxe=np.tile(col(np.r_[XMIN[:NQ], np.zeros(NQ)]), (B, 1)),
                 ubxe=np.tile(col(np.r_[XMAX[:NQ], np.zeros(NQ)]), (B, 1)))


CART_DRAWS = 6   # testing_test of the Cartesian driver: (random, choice) per joint for p, one random per joint
CART_STREAM = 6


def cartesian_ics(ids, N=100, seed=SEED):
    """First OCP of the Cartesian double pendulum's `testing_test`
    (VBOC/Cartesian constraints/vboc_multiprocessing.py:19-92), what its main block fans out for the test
    and training sets (:557-572): p[l] = random() * choice([-1, 1]), normalised; q_init ~ U(q_min, q_max)
    per joint; velocities free in [-v_max, v_max]; constant guess [q_init, 0, 0, dt]; u = 0.  Philox
    stream 6.  The keep-out circle is an OCP-level constraint (systems.cartesian_constraint)."""
    sysd = system(2)
    ids = np.asarray(ids)
    B = ids.shape[0]
    U = uniforms(ids, CART_DRAWS, seed, stream=CART_STREAM)
    r = np.stack([U[:, 2 * j] * _choice(U[:, 2 * j + 1], [-1.0, 1.0]) for j in range(2)], axis=1)
    p = np.zeros((B, 3))
    p[:, :2] = r / _row_norms(r)
    qi = sysd.q_min + U[:, 4:6] * (sysd.q_max - sysd.q_min)
    dt = sysd.dt
    lbx0 = np.concatenate([qi, np.full((B, 2), -sysd.v_max), np.full((B, 1), dt)], axis=1)
    ubx0 = np.concatenate([qi, np.full((B, 2), sysd.v_max), np.full((B, 1), dt)], axis=1)
    xg = np.zeros((B, N + 1, 5))
    xg[:, :, :2] = qi[:, None, :]
    xg[:, :, 4] = dt
    b = _bounds(sysd, B, N, xg, np.zeros((B, N, 2)), p, lbx0, ubx0)
    return b


def pendulum_free_time_ics(ids, N_range=(20, 60), seed=SEED):
    """Free-time pendulum OCPs shaped like VBOC/pendulum_vboc.py's solves (OCPpendulum.OCP_solve,
    VBOC/pendulum_class_vboc.py:107-130): sweep direction v_sel = +-v_max (:55-77), a fixed initial
    position q_init (the sweep's first solve starts at the box edge, :61/:70; its verification solves
    anywhere along the trajectory, :181 - here uniform in the box, kept 0.05 rad away from q_fin),
    terminal rest at q_fin, dt free in [0, 1e-2], straight-line guess (:79-84), horizon uniform in
    N_range.  Philox stream 4.  For parity tests and benchmarks of the free-time solver."""
    sysd = system(1)
    ids = np.asarray(ids)
    B = ids.shape[0]
    U = uniforms(ids, 4, seed, stream=4)
    q_min, q_max, v_max = sysd.q_min, sysd.q_max, sysd.v_max
    vsel = np.where(U[:, 0] < 0.5, -v_max, v_max)
    N = (N_range[0] + np.floor(U[:, 2] * (N_range[1] - N_range[0] + 1))).astype(np.int32)
    N = np.minimum(N, N_range[1])
    Nm = int(N.max())
    span = q_max - q_min - 0.05
    q_init = np.where(vsel < 0, q_min + 0.05 + U[:, 1] * span, q_max - 0.05 - U[:, 1] * span)
    q_fin = np.where(vsel < 0, q_min, q_max)
    lbx = np.stack([np.full(B, q_min), np.where(vsel < 0, -v_max, 0.0), np.zeros(B)], axis=1)
    ubx = np.stack([np.full(B, q_max), np.where(vsel < 0, 0.0, v_max), np.full(B, 1e-2)], axis=1)
    xg = np.zeros((B, Nm + 1, 3))
    for b in range(B):
        n = int(N[b])
        xg[b, :n + 1, 0] = np.linspace(q_init[b], q_fin[b], n + 1)
        xg[b, :n + 1, 1] = vsel[b]
        xg[b, :n + 1, 2] = 1e-2
        xg[b, n + 1:] = xg[b, n]
    p = np.stack([np.where(vsel < 0, 1.0, -1.0), np.ones(B)], axis=1)
    return Batch(N=N, x_guess=xg, u_guess=np.zeros((B, Nm, 1)), p=p, lbx=lbx, ubx=ubx,
                 lbu=np.full((B, 1), -sysd.u_max), ubu=np.full((B, 1), sysd.u_max),
                 lbx0=np.stack([q_init, np.full(B, -v_max), np.zeros(B)], axis=1),
                 ubx0=np.stack([q_init, np.full(B, v_max), np.full(B, 1e-2)], axis=1),
                 lbxe=np.stack([q_fin, np.zeros(B), np.zeros(B)], axis=1),
                 ubxe=np.stack([q_fin, np.zeros(B), np.full(B, 1e-2)], axis=1))
