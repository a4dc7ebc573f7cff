"""URDF -> lgx_model (the rigid-body model the HIP solver and the oracle consume).

Replaces what Isaac Gym's closed asset importer does for the reference
(gym.load_asset, legged_robot.py:834, with collapse_fixed_joints=True,
replace_cylinder_with_capsule=True, legged_robot_config.py:95,99):

* rigid bodies kept in the reference's body list = the URDF links that are not merged
  away: links reached through revolute joints and fixed joints marked
  dont_collapse="true" (Go2: Head_upper, Head_lower, feet). Order = depth-first in
  joint declaration order -> `body_names`, `dof_names`.
* dynamic links (what the solver integrates) = the base + one link per revolute joint;
  every fixed child is merged into its dynamic ancestor (mass, COM, inertia), since a
  fixed child moves rigidly with it.
* contact candidates = collision shapes reduced to sphere centres in the dynamic link
  frame: sphere -> 1, cylinder (capsule) -> 2 end spheres, box -> 8 corners (thigh
  boxes -> a 2-sphere capsule along the long axis to stay within the 64-lane budget).

The built model is cached as JSON under resources/robots/ so the GPU box (where the
reference URDFs are absent) loads the same numbers.
"""
import json
import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from . import _abi

RES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "resources", "robots")


def _rpy_to_R(rpy):
    r, p, y = rpy
    cr, sr, cp, sp, cy, sy = math.cos(r), math.sin(r), math.cos(p), math.sin(p), math.cos(y), math.sin(y)
    return np.array([[cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
                     [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def _vec(s, default="0 0 0"):
    return np.array([float(x) for x in (s if s is not None else default).split()])


def _origin(el):
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.zeros(3), np.eye(3)
    return _vec(o.get("xyz")), _rpy_to_R(_vec(o.get("rpy")))


class _Link:
    def __init__(self, el):
        self.name = el.get("name")
        self.mass = 0.0
        self.com = np.zeros(3)
        self.I = np.zeros((3, 3))
        inert = el.find("inertial")
        if inert is not None:
            self.mass = float(inert.find("mass").get("value"))
            c, R = _origin(inert)
            i = inert.find("inertia")
            g = lambda k: float(i.get(k, "0"))
            Il = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")], [g("ixz"), g("iyz"), g("izz")]])
            self.com = c
            self.I = R @ Il @ R.T
        self.shapes = []  # (kind, params, pos, R)
        for col in el.findall("collision"):
            p, R = _origin(col)
            geo = col.find("geometry")[0]
            if geo.tag == "box":
                self.shapes.append(("box", _vec(geo.get("size")), p, R))
            elif geo.tag == "cylinder":
                self.shapes.append(("cylinder", (float(geo.get("radius")), float(geo.get("length"))), p, R))
            elif geo.tag == "sphere":
                self.shapes.append(("sphere", float(geo.get("radius")), p, R))


def _merge_inertia(parts):
    """parts: list of (m, com[3], I_com[3,3]) in a common frame -> (m, com, I about com)."""
    m = sum(p[0] for p in parts)
    if m <= 0:
        return 0.0, np.zeros(3), np.zeros((3, 3))
    c = sum(p[0] * p[1] for p in parts) / m
    I = np.zeros((3, 3))
    for mi, ci, Ii in parts:
        d = ci - c
        I += Ii + mi * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
    return m, c, I


def build_from_urdf(path, foot_name="foot", thigh_capsule=True):
    root = ET.parse(path).getroot()
    links = {l.get("name"): _Link(l) for l in root.findall("link")}
    joints = root.findall("joint")
    children = {}
    parent_of = set()
    for j in joints:
        p, c = j.find("parent").get("link"), j.find("child").get("link")
        children.setdefault(p, []).append(j)
        parent_of.add(c)
    base = [n for n in links if n not in parent_of][0]

    bodies = []        # (name, dyn_link_idx, offset p in dyn link frame, R offset)
    dyn = [{"name": base, "parent": -1, "origin": np.zeros(3), "rot": np.eye(3), "axis": np.zeros(3), "lower": 0.0,
            "upper": 0.0, "limited": 0, "effort": 0.0, "velocity": 0.0, "parts": [], "shapes": []}]
    dof_names = []

    def attach(link_name, dyn_idx, p, R, kept_body):
        L = links[link_name]
        if L.mass > 0:
            dyn[dyn_idx]["parts"].append((L.mass, p + R @ L.com, R @ L.I @ R.T))
        for kind, prm, sp, sR in L.shapes:
            dyn[dyn_idx]["shapes"].append((kind, prm, p + R @ sp, R @ sR, kept_body))

    def visit(link_name, dyn_idx, p, R):
        body_idx = len(bodies)
        bodies.append((link_name, dyn_idx, p.copy(), R.copy()))
        attach(link_name, dyn_idx, p, R, body_idx)
        walk_children(link_name, dyn_idx, p, R, body_idx)

    def walk_children(link_name, dyn_idx, p, R, body_idx):
        for j in children.get(link_name, []):
            child = j.find("child").get("link")
            jp, jR = _origin(j)
            cp, cR = p + R @ jp, R @ jR
            jt = j.get("type")
            if jt in ("revolute", "continuous"):
                axis = _vec(j.find("axis").get("xyz"))
                lim = j.find("limit")
                lo = float(lim.get("lower", 0)) if lim is not None else 0.0
                hi = float(lim.get("upper", 0)) if lim is not None else 0.0
                effort = float(lim.get("effort", 0)) if lim is not None else 0.0
                velocity = float(lim.get("velocity", 0)) if lim is not None else 0.0
                dyn.append({"name": child, "parent": dyn_idx, "origin": cp, "rot": cR, "axis": axis / np.linalg.norm(axis),
                            "lower": lo, "upper": hi, "limited": int(jt == "revolute" and hi > lo),
                            "effort": effort, "velocity": velocity, "parts": [], "shapes": []})
                dof_names.append(j.get("name"))
                visit(child, len(dyn) - 1, np.zeros(3), np.eye(3))
            elif jt == "fixed":
                if j.get("dont_collapse") == "true":
                    visit(child, dyn_idx, cp, cR)
                else:
                    attach(child, dyn_idx, cp, cR, body_idx)
                    walk_children(child, dyn_idx, cp, cR, body_idx)
            else:
                raise ValueError(f"unsupported joint type {jt}")

    visit(base, 0, np.zeros(3), np.eye(3))
    body_names = [b[0] for b in bodies]
    feet = [i for i, n in enumerate(body_names) if foot_name in n]

    # candidates: feet spheres first (keeps the common case in the first wave lanes)
    cands = []
    for li, d in enumerate(dyn):
        for kind, prm, p, R, body in d["shapes"]:
            if kind == "sphere":
                cands.append((li, body, p, prm))
            elif kind == "cylinder":
                r, length = prm
                for s in (-0.5, 0.5):
                    cands.append((li, body, p + R @ np.array([0, 0, s * length]), r))
            elif kind == "box":
                sx, sy, sz = prm
                if thigh_capsule and "thigh" in body_names[body]:
                    ext = R @ np.diag([sx, sy, sz])
                    ax = int(np.argmax(np.abs(ext).sum(0) * 0 + np.array([sx, sy, sz])))
                    half = np.array([sx, sy, sz]) / 2
                    r = float(sorted(half)[1])
                    e = np.zeros(3); e[ax] = half[ax] - r
                    for s in (-1, 1):
                        cands.append((li, body, p + R @ (s * e), r))
                else:
                    for cx in (-0.5, 0.5):
                        for cy in (-0.5, 0.5):
                            for cz in (-0.5, 0.5):
                                cands.append((li, body, p + R @ np.array([cx * sx, cy * sy, cz * sz]), 0.0))
    cands.sort(key=lambda c: (0 if c[1] in feet else 1))
    if len(cands) > _abi.MAX_CANDIDATES:
        raise ValueError(f"{len(cands)} contact candidates > {_abi.MAX_CANDIDATES}")

    out = {"body_names": body_names, "dof_names": dof_names, "links": [], "bodies": [], "candidates": []}
    for d in dyn:
        m, c, I = _merge_inertia(d["parts"])
        out["links"].append({"name": d["name"], "parent": d["parent"], "origin": d["origin"].tolist(),
                             "rot": d["rot"].reshape(9).tolist(),
                             "axis": d["axis"].tolist(), "lower": d["lower"], "upper": d["upper"],
                             "limited": d["limited"], "effort": d["effort"], "velocity": d["velocity"], "mass": m, "com": c.tolist(),
                             "inertia": [I[0, 0], I[1, 1], I[2, 2], I[0, 1], I[0, 2], I[1, 2]]})
    for name, li, p, R in bodies:
        out["bodies"].append({"name": name, "link": li, "offset": p.tolist(), "rot": R.reshape(9).tolist()})
    for li, body, p, r in cands:
        out["candidates"].append({"link": li, "body": body, "pos": list(map(float, p)), "radius": float(r)})
    return out


def save_json(model, name):
    os.makedirs(RES_DIR, exist_ok=True)
    with open(os.path.join(RES_DIR, name + ".json"), "w") as f:
        json.dump(model, f, indent=1)


def load_model(asset_file, foot_name="foot", root_dir=None):
    """Model for the cfg.asset.file path: parse the URDF when it exists, else the
    bundled JSON with the same robot name."""
    path = asset_file.format(LEGGED_GYM_ROOT_DIR=root_dir or "")
    if os.path.exists(path):
        return build_from_urdf(path, foot_name)
    name = os.path.splitext(os.path.basename(path))[0]
    js = os.path.join(RES_DIR, name + ".json")
    if not os.path.exists(js):
        raise FileNotFoundError(f"robot model {path} not found and no bundled {js}")
    with open(js) as f:
        return json.load(f)


def to_struct(model):
    M = _abi.Model()
    M.num_links = len(model["links"])
    M.num_bodies = len(model["bodies"])
    M.num_candidates = len(model["candidates"])
    for i, l in enumerate(model["links"]):
        M.link_parent[i] = l["parent"]
        for k in range(3):
            M.joint_origin[i][k] = l["origin"][k]
            M.joint_axis[i][k] = l["axis"][k]
            M.link_com[i][k] = l["com"][k]
        for k in range(9):
            M.joint_rot[i][k] = l["rot"][k]
        M.joint_lower[i] = l["lower"]
        M.joint_upper[i] = l["upper"]
        M.joint_has_limits[i] = l["limited"]
        M.link_mass[i] = l["mass"]
        for k in range(6):
            M.link_inertia[i][k] = l["inertia"][k]
    for i, b in enumerate(model["bodies"]):
        M.body_link[i] = b["link"]
        for k in range(3):
            M.body_offset[i][k] = b["offset"][k]
        for k in range(9):
            M.body_rot[i][k] = b["rot"][k]
    for i, c in enumerate(model["candidates"]):
        M.cand_link[i] = c["link"]
        M.cand_body[i] = c["body"]
        for k in range(3):
            M.cand_pos[i][k] = c["pos"][k]
        M.cand_radius[i] = c["radius"]
    return M
