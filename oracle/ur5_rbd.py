"""ORACLE - TEST INFRASTRUCTURE ONLY (tests/ import it; the product path never does).

Independent numpy restatement of the UR5 forward dynamics the reference gets from urdf2casadi
(`VBOC/UR5/ur5reduced_class_fixedveldir.py:20-45`: `get_forward_dynamics_aba(root='base_link',
tip='tool0', gravity=[0, 0, -9.81])`).  urdf2casadi is an un-vendored, un-pinned dependency absent
from this image; this module restates its published model builder and articulated-body algorithm
(`urdfparser.URDFparser._model_calculation` / `get_forward_dynamics_aba`, `geometry.plucker`) in 6x6
spatial algebra (Featherstone's order: angular first), straight from the RAW chain data of
`tests/golden/ur5_urdf.json` - not from the generated compact parameters the C oracle and the HIP
kernels use - so it cross-checks `tools/gen_ur5_model.py`'s fixed-joint merging as well:

  XT(xyz, rpy)        = spatial_transform(R(rpy)^T, xyz)
  XJT_revolute(...)   = XJ(axis, q) @ XT(xyz, rpy), composed with the preceding fixed joints' XT
  inertia             = spatial_inertia_matrix_IO(I, m, inertial.origin.xyz)   (inertial rpy unused)
  fixed-joint merge   = I_prev + XT^T I XT ;  base-side inertias dropped
  ABA                 = Featherstone RBDA Table 7.1 with a_0 = -a_g.

Parity of this restatement with urdf2casadi itself is UNPINNED (no urdf2casadi output is stored in
the reference); tests pin its physics instead: energy conservation of the unforced, gravity-only
motion against independently computed forward kinematics, and M(q) symmetric positive definite.
"""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
RAW = os.path.join(os.path.dirname(HERE), "tests", "golden", "ur5_urdf.json")


def skew(r):
    return np.array([[0.0, -r[2], r[1]], [r[2], 0.0, -r[0]], [-r[1], r[0], 0.0]])


def rpy_matrix(rpy):
    r, p, y = rpy
    Rx = np.array([[1, 0, 0], [0, np.cos(r), -np.sin(r)], [0, np.sin(r), np.cos(r)]])
    Ry = np.array([[np.cos(p), 0, np.sin(p)], [0, 1, 0], [-np.sin(p), 0, np.cos(p)]])
    Rz = np.array([[np.cos(y), -np.sin(y), 0], [np.sin(y), np.cos(y), 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def axis_rotation(axis, q):
    a = np.asarray(axis, float) / np.linalg.norm(axis)
    K = skew(a)
    return np.eye(3) + np.sin(q) * K + (1 - np.cos(q)) * K @ K


def spatial_transform(E, r):
    X = np.zeros((6, 6))
    X[:3, :3] = E
    X[3:, :3] = -E @ skew(r)
    X[3:, 3:] = E
    return X


def XT(xyz, rpy):
    return spatial_transform(rpy_matrix(rpy).T, np.asarray(xyz, float))


def inertia_IO(ine):
    ixx, ixy, ixz, iyy, iyz, izz = ine["inertia"]
    c = np.asarray(ine["xyz"], float)
    m = ine["mass"]
    cx = skew(c)
    I = np.zeros((6, 6))
    I[:3, :3] = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]]) + m * cx @ cx.T
    I[:3, 3:] = m * cx
    I[3:, :3] = m * cx.T
    I[3:, 3:] = m * np.eye(3)
    return I


class UR5:
    def __init__(self, path=RAW):
        with open(path) as f:
            d = json.load(f)
        self.chain = d["chain"]
        self.gravity = np.asarray(d["gravity"], float)
        self.nq = sum(1 for it in self.chain if it["kind"] == "joint" and it["type"] in ("revolute", "continuous"))

    def model(self, q):
        """i_X_p, S, I per actuated joint (urdf2casadi _model_calculation, restated)."""
        Xs, Ss, Is = [], [], []
        prev_joint, XT_prev, prev_inertia, n_act, i = None, None, None, 0, 0
        inertia_transform, spatial_inertia = None, np.zeros((6, 6))
        for it in self.chain:
            if it["kind"] == "joint":
                if it["type"] == "fixed":
                    X = XT(it["xyz"], it["rpy"])
                    XT_prev = X @ XT_prev if prev_joint == "fixed" else X
                    inertia_transform = XT_prev
                    prev_inertia = spatial_inertia
                else:
                    if n_act != 0:
                        Is.append(spatial_inertia)
                    n_act += 1
                    XJ = spatial_transform(axis_rotation(it["axis"], q[i]).T, np.zeros(3))
                    X = XJ @ XT(it["xyz"], it["rpy"])
                    if prev_joint == "fixed":
                        X = X @ XT_prev
                    Xs.append(X)
                    Ss.append(np.concatenate([it["axis"], [0.0, 0.0, 0.0]]))
                    i += 1
                prev_joint = it["type"]
            else:
                spatial_inertia = np.zeros((6, 6)) if it["inertial"] is None else inertia_IO(it["inertial"])
                if prev_joint == "fixed":
                    spatial_inertia = prev_inertia + inertia_transform.T @ spatial_inertia @ inertia_transform
                if it["name"] == "tool0":
                    Is.append(spatial_inertia)
        return Xs, Ss, Is

    def aba(self, q, qd, tau):
        n = self.nq
        Xs, S, Ic = self.model(q)
        crm = lambda v: np.block([[skew(v[:3]), np.zeros((3, 3))], [skew(v[3:]), skew(v[:3])]])
        crf = lambda v: -crm(v).T
        v, c, IA, pA = [], [], [], []
        for i in range(n):
            vJ = S[i] * qd[i]
            vi = vJ if i == 0 else Xs[i] @ v[i - 1] + vJ
            v.append(vi)
            c.append(np.zeros(6) if i == 0 else crm(vi) @ vJ)
            IA.append(Ic[i].copy())
            pA.append(crf(vi) @ Ic[i] @ vi)
        U, d, u = [None] * n, [None] * n, [None] * n
        for i in range(n - 1, -1, -1):
            U[i] = IA[i] @ S[i]
            d[i] = S[i] @ U[i]
            u[i] = tau[i] - S[i] @ pA[i]
            if i > 0:
                Ia = IA[i] - np.outer(U[i], U[i]) / d[i]
                pa = pA[i] + Ia @ c[i] + U[i] * u[i] / d[i]
                IA[i - 1] = IA[i - 1] + Xs[i].T @ Ia @ Xs[i]
                pA[i - 1] = pA[i - 1] + Xs[i].T @ pa
        ag = np.concatenate([np.zeros(3), self.gravity])
        qdd, a = [0.0] * n, []
        for i in range(n):
            ap = -ag if i == 0 else a[i - 1]
            ai = Xs[i] @ ap + c[i]
            qdd[i] = (u[i] - U[i] @ ai) / d[i]
            a.append(ai + S[i] * qdd[i])
        return np.array(qdd)

    # --- independent physics for the checks: poses of every massive link, energies -----------
    def link_frames(self, q):
        """World (base_link) pose of every link with an inertial, following the raw chain."""
        T, i, out = np.eye(4), 0, []
        for it in self.chain:
            if it["kind"] == "joint":
                J = np.eye(4)
                J[:3, :3] = rpy_matrix(it["rpy"])
                J[:3, 3] = it["xyz"]
                T = T @ J
                if it["type"] != "fixed":
                    R = np.eye(4)
                    R[:3, :3] = axis_rotation(it["axis"], q[i])
                    T = T @ R
                    i += 1
            elif it["inertial"] is not None and i > 0:
                out.append((it["inertial"], T.copy()))
        return out

    def energy(self, q, qd, h=1e-7):
        """Kinetic + potential energy (potential from -gravity . COM), velocities of the COMs and
        angular velocities by central differences of the link poses along qd."""
        E = 0.0
        f0, fp, fm = self.link_frames(q), self.link_frames(q + h * qd), self.link_frames(q - h * qd)
        for (ine, T), (_, Tp), (_, Tm) in zip(f0, fp, fm):
            c = np.asarray(ine["xyz"], float)
            com = T[:3, :3] @ c + T[:3, 3]
            vc = ((Tp[:3, :3] @ c + Tp[:3, 3]) - (Tm[:3, :3] @ c + Tm[:3, 3])) / (2 * h)
            dR = (Tp[:3, :3] - Tm[:3, :3]) / (2 * h)
            W = dR @ T[:3, :3].T
            w = np.array([W[2, 1], W[0, 2], W[1, 0]])
            ixx, ixy, ixz, iyy, iyz, izz = ine["inertia"]
            Ic = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])   # link frame (rpy unused)
            Iw = T[:3, :3] @ Ic @ T[:3, :3].T
            E += 0.5 * ine["mass"] * vc @ vc + 0.5 * w @ Iw @ w - ine["mass"] * self.gravity @ com
        return E
