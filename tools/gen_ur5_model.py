"""Generate the UR5 rigid-body parameters from the reference's URDF (build container only).

The reference builds the UR5 dynamics with urdf2casadi (`VBOC/UR5/ur5reduced_class_fixedveldir.py:20-45`:
`URDFparser().from_file('ur5.urdf')`, chain root 'base_link' -> tip 'tool0', gravity [0, 0, -9.81],
`get_forward_dynamics_aba`).  urdf2casadi is an un-vendored, un-pinned third-party dependency that is
not installed here, so this script restates how its model builder (`urdfparser.URDFparser.
_model_calculation`, github.com/mahaarbo/urdf2casadi) turns the URDF chain into a rigid-body model:

  * the chain is the path root -> tip; links hanging off it (the gripper fingers) are not in the model;
  * a link's spatial inertia is `spatial_inertia_matrix_IO(ixx..izz, mass, inertial.origin.xyz)`: the
    inertia tensor is taken in the LINK frame about the COM at `inertial.origin.xyz` - the inertial
    origin's rpy is NOT applied (quirk, kept: it matters for upper_arm_link and forearm_link);
  * fixed joints are merged: the transforms of consecutive fixed joints are composed, folded into the
    next actuated joint's transform, and the inertias of links behind a fixed joint are added to the
    preceding body's inertia through that transform (`prev + XT^T I XT`);
  * inertias before the first actuated joint belong to the fixed base and are dropped;
  * revolute joints rotate about `axis` of the joint frame `origin xyz/rpy` (URDF rpy = Rz(y)Ry(p)Rx(r)).

Outputs (committed; nothing of the reference travels but these numbers):
  tests/golden/ur5_urdf.json      the raw chain data (joint types/origins/axes, link inertials) - used by
                                  the independent 6x6 spatial-algebra ABA check in tests/test_ur5.py
  vboc_amd/csrc/ur5_params.h      per actuated joint: tree rotation R_i and offset p_i of the joint frame
                                  in the parent body frame; per body: mass, COM and inertia about the body
                                  origin (merged over fixed joints), in C syntax for the HIP solver and
                                  the C oracle
  vboc_amd/ur5_params.json        the same numbers for the Python drop-in class and the numpy checks
"""
import json
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

URDF = "/root/reference/VBOC/UR5/ur5.urdf"
ROOT, TIP = "base_link", "tool0"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _vec(s, n=3):
    v = [float(t) for t in s.split()] if s else [0.0] * n
    return v


def rpy_matrix(rpy):
    r, p, y = rpy
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def parse_chain(path=URDF):
    """Ordered chain root -> tip: [('link', {...}) | ('joint', {...}), ...]."""
    tree = ET.parse(path).getroot()
    links, joints_by_child = {}, {}
    for ln in tree.findall("link"):
        inert = ln.find("inertial")
        d = {"name": ln.get("name"), "inertial": None}
        if inert is not None:
            o = inert.find("origin")
            I = inert.find("inertia")
            d["inertial"] = {
                "mass": float(inert.find("mass").get("value")),
                "xyz": _vec(o.get("xyz") if o is not None else None),
                "rpy": _vec(o.get("rpy") if o is not None else None),
                "inertia": [float(I.get(k)) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")],
            }
        links[d["name"]] = d
    for jt in tree.findall("joint"):
        o = jt.find("origin")
        ax = jt.find("axis")
        joints_by_child[jt.find("child").get("link")] = {
            "name": jt.get("name"), "type": jt.get("type"),
            "parent": jt.find("parent").get("link"), "child": jt.find("child").get("link"),
            "xyz": _vec(o.get("xyz") if o is not None else None),
            "rpy": _vec(o.get("rpy") if o is not None else None),
            "axis": _vec(ax.get("xyz")) if ax is not None else [1.0, 0.0, 0.0],
        }
    chain = []
    cur = TIP
    while cur != ROOT:
        chain.append(("link", links[cur]))
        j = joints_by_child[cur]
        chain.append(("joint", j))
        cur = j["parent"]
    chain.append(("link", links[ROOT]))
    return chain[::-1]


def pose(xyz, rpy):
    T = np.eye(4)
    T[:3, :3] = rpy_matrix(rpy)
    T[:3, 3] = xyz
    return T


def build_model(chain):
    """Bodies after each actuated joint, fixed joints merged (urdf2casadi rules, module docstring).

    Returns joints [{R, p, axis}] (joint frame relative to the parent BODY frame, before the joint
    rotation) and bodies [{m, com, Io}] (inertia about the body origin, body frame)."""
    joints, bodies = [], []
    T_fixed = np.eye(4)      # pose of the current link frame in the current body frame
    body = None              # accumulator of the current body: list of (m, com_body, Icom_body)
    for kind, d in chain:
        if kind == "joint":
            if d["type"] == "fixed":
                T_fixed = T_fixed @ pose(d["xyz"], d["rpy"])
            elif d["type"] in ("revolute", "continuous"):
                T = T_fixed @ pose(d["xyz"], d["rpy"])
                ax = np.asarray(d["axis"], float)
                joints.append({"name": d["name"], "R": T[:3, :3], "p": T[:3, 3], "axis": ax / np.linalg.norm(ax)})
                if body is not None:
                    bodies.append(body)
                body = []
                T_fixed = np.eye(4)
            else:
                raise ValueError("unsupported joint type " + d["type"])
        else:
            ine = d["inertial"]
            if ine is None or body is None:
                continue       # massless link, or part of the fixed base (dropped)
            R, p = T_fixed[:3, :3], T_fixed[:3, 3]
            ixx, ixy, ixz, iyy, iyz, izz = ine["inertia"]
            Ic = np.array([[ixx, ixy, ixz], [ixy, iyy, iyz], [ixz, iyz, izz]])  # rpy NOT applied (quirk)
            body.append((ine["mass"], R @ np.asarray(ine["xyz"]) + p, R @ Ic @ R.T))
    bodies.append(body)
    out = []
    for parts in bodies:
        m = sum(pm for pm, _, _ in parts)
        com = sum(pm * c for pm, c, _ in parts) / m
        Io = np.zeros((3, 3))
        for pm, c, Ic in parts:       # about the body origin (parallel axis from each part's COM)
            Io += Ic + pm * (np.dot(c, c) * np.eye(3) - np.outer(c, c))
        out.append({"m": m, "com": com, "Io": Io})
    return joints, out


def main():
    chain = parse_chain()
    raw = [{"kind": k, **d} for k, d in chain]
    with open(os.path.join(REPO, "tests", "golden", "ur5_urdf.json"), "w") as f:
        json.dump({"source": "VBOC/UR5/ur5.urdf chain base_link -> tool0 (data only)",
                   "gravity": [0.0, 0.0, -9.81], "chain": raw}, f, indent=1)
    joints, bodies = build_model(chain)
    assert len(joints) == 4, len(joints)
    for j in joints:
        assert np.allclose(j["axis"], [0, 0, 1]), j   # the kernels assume z-axis revolute joints
    params = {
        "source": "tools/gen_ur5_model.py from VBOC/UR5/ur5.urdf (urdf2casadi model rules)",
        "gravity": [0.0, 0.0, -9.81],
        "joints": [{"name": j["name"], "R": j["R"].tolist(), "p": j["p"].tolist()} for j in joints],
        "bodies": [{"m": b["m"], "com": b["com"].tolist(), "Io": b["Io"].tolist()} for b in bodies],
    }
    with open(os.path.join(REPO, "vboc_amd", "ur5_params.json"), "w") as f:
        json.dump(params, f, indent=1)

    def arr(name, vals):
        init = "{%s}" % ", ".join("%.17g" % v for v in vals)
        return "#define %s_INIT %s\nUR5_CONST double %s[%d] = %s_INIT;\n" % (name, init, name, len(vals), name)

    h = ["/* ur5_params.h - GENERATED by tools/gen_ur5_model.py from the reference's VBOC/UR5/ur5.urdf",
         " * (chain base_link -> tool0, urdf2casadi model rules: fixed joints merged, inertial rpy not applied).",
         " * Plain C, shared by the HIP solver (model.h) and the C oracle.  Do not edit.",
         " *   UR5_R[i]   rotation (row-major 3x3) of joint frame i in its parent body frame, before the",
         " *              joint rotation Rz(q_i); UR5_P[i] its origin in the parent body frame",
         " *   UR5_M[i]   body mass; UR5_MC[i] = mass * COM (body frame); UR5_IO[i] inertia about the body",
         " *              origin (row-major 3x3, body frame); gravity (0, 0, -9.81) in the base_link frame */",
         "#ifndef VBOC_UR5_PARAMS_H", "#define VBOC_UR5_PARAMS_H", "#define UR5_NQ 4",
         "#ifndef UR5_CONST", "#define UR5_CONST static const", "#endif", ""]
    h.append(arr("UR5_R", [v for j in joints for v in j["R"].ravel()]))
    h.append(arr("UR5_P", [v for j in joints for v in j["p"]]))
    h.append(arr("UR5_M", [b["m"] for b in bodies]))
    h.append(arr("UR5_MC", [v for b in bodies for v in b["m"] * b["com"]]))
    h.append(arr("UR5_IO", [v for b in bodies for v in b["Io"].ravel()]))
    h.append("#endif")
    with open(os.path.join(REPO, "vboc_amd", "csrc", "ur5_params.h"), "w") as f:
        f.write("\n".join(h) + "\n")
    for j in joints:
        print(j["name"], np.round(j["R"], 6).tolist(), np.round(j["p"], 6).tolist())
    for b in bodies:
        print("m %.4f com %s" % (b["m"], np.round(b["com"], 5).tolist()))


if __name__ == "__main__":
    sys.exit(main())
