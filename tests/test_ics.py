"""Counter-based IC generation: determinism, shard invariance, and the reference's IC laws
(VBOC/triplependulum_vboc.py:32-103, triplependulum_testdata.py:19-38)."""
import numpy as np
import pytest

from vboc_amd.ics import data_generation_ics, heldout_ics, philox4x32, uniforms
from vboc_amd.systems import system


def test_philox_known_answer():
    # Random123 Philox4x32-10 known-answer vectors (counter 0 / key 0, and pi digits)
    out = philox4x32(np.zeros((1, 4), np.uint64), (0, 0))[0]
    assert [int(v) for v in out] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    ctr = np.array([[0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344]], np.uint64)
    out = philox4x32(ctr, (0xA4093822, 0x299F31D0))[0]
    assert [int(v) for v in out] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_uniforms_shard_invariant():
    full = uniforms(np.arange(1000), 7)
    parts = np.concatenate([uniforms(np.arange(r, 1000, 4), 7) for r in range(4)])
    order = np.concatenate([np.arange(r, 1000, 4) for r in range(4)])
    np.testing.assert_array_equal(full[order], parts)
    assert full.min() >= 0 and full.max() < 1
    assert abs(full.mean() - 0.5) < 0.02


@pytest.mark.parametrize("nq", [2, 3])
def test_data_generation_law(nq):
    sysd = system(nq)
    b = data_generation_ics(nq, np.arange(512))
    B, N = 512, sysd.N
    p = b["p"]
    np.testing.assert_allclose(np.linalg.norm(p[:, :nq], axis=1), 1.0, rtol=1e-14)
    assert np.all(p[:, nq] == 0.0)
    js, vs = b["joint_sel"], b["vel_sel"]
    # the reference joint's cost weight carries vel_sel's sign (:45-54)
    assert np.all(np.sign(p[np.arange(B), js]) == vs)
    # reference joint starts eps inside the limit it starts from; others clamped by eps
    q0 = b["lbx0"][:, :nq]
    np.testing.assert_array_equal(b["lbx0"][:, :nq], b["ubx0"][:, :nq])
    sel = q0[np.arange(B), js]
    exp = np.where(vs == -1, sysd.q_min + sysd.eps, sysd.q_max - sysd.eps)
    np.testing.assert_allclose(sel, exp)
    assert np.all(q0 >= sysd.q_min + sysd.eps - 1e-12) and np.all(q0 <= sysd.q_max - sysd.eps + 1e-12)
    # straight-line guess from the start limit to the opposite limit (:85-93); stage N = row N-1
    xg = b["x_guess"]
    np.testing.assert_allclose(xg[np.arange(B), 0, js], np.where(vs == -1, sysd.q_min, sysd.q_max))
    np.testing.assert_allclose(xg[np.arange(B), N - 1, js], np.where(vs == -1, sysd.q_max, sysd.q_min))
    np.testing.assert_array_equal(xg[:, N], xg[:, N - 1])
    np.testing.assert_allclose(xg[np.arange(B), 0, js + nq], 2 * (np.where(vs == -1, 1, -1) * np.pi / 2))
    assert np.all(xg[:, :, 2 * nq] == sysd.dt)
    assert set(np.unique(js)) == set(range(nq)) and set(np.unique(vs)) == {-1.0, 1.0}
    # bounds as the driver sets them (:98-103)
    assert np.all(b["lbxe"][:, nq:2 * nq] == 0) and np.all(b["ubxe"][:, nq:2 * nq] == 0)
    assert np.all(b["lbx"][:, 2 * nq] == sysd.dt) and np.all(b["ubx"][:, 2 * nq] == sysd.dt)


@pytest.mark.parametrize("nq", [1, 2, 3])
def test_heldout_law(nq):
    sysd = system(nq)
    b = heldout_ics(nq, np.arange(256))
    q0 = b["lbx0"][:, :nq]
    assert np.all(q0 >= sysd.q_min) and np.all(q0 <= sysd.q_max)
    if nq == 1:
        assert set(np.unique(b["p"][:, 0])) == {-1.0, 1.0}
    else:
        np.testing.assert_allclose(np.linalg.norm(b["p"][:, :nq], axis=1), 1.0, rtol=1e-14)
    # constant guess at the initial position, at rest (:37-38)
    np.testing.assert_array_equal(b["x_guess"][:, :, :nq], np.repeat(q0[:, None, :], sysd.N + 1, 1))
    assert np.all(b["x_guess"][:, :, nq:2 * nq] == 0)
    if nq == 2:   # gravity compensation at q0 (doublependulum_testdata.py:37)
        np.testing.assert_allclose(b["u_guess"][:, 0, 1], sysd.g * sysd.l[1] * sysd.m[1] * np.sin(q0[:, 1]),
                                   rtol=1e-15)
        assert np.all(b["u_guess"] == b["u_guess"][:, :1])
    else:
        assert np.all(b["u_guess"] == 0)
