"""MJCF <-> kinematic-tree helpers of the kinematics front end.

The reference builds its controller from the robot's MJCF file (OperationalSpaceController(
xml_path), unitree_go2/operational_space_controller.h:108-152); the native reader is
osc_kin_desc_from_mjcf (csrc/osc_mjcf.cpp).  This module writes the <robot>_kinematics.json
trees (and any tree in that schema) out as MJCF, so the same model can be fed through either
door, and loads MJCF through the native reader into the JSON-schema dict the oracle takes.
"""
from __future__ import annotations

from . import _lib


def _fmt(v) -> str:
    return " ".join(repr(float(x)) for x in v)


def tree_to_mjcf(tree: dict, body_names=None, site_names=None, extra_bodies=(),
                 model_name: str = "osc_tree") -> str:
    """MJCF text of a tree in the <robot>_kinematics.json schema.  body_names / site_names
    rename bodies / sites (default: the tree's "name" fields, else b<i> / s<k>); extra_bodies =
    [(name, parent_index, pos)] adds massless welded bodies (frames) after the tree's own.
    Angles are written as quaternions, so the compiler's angle unit does not matter."""
    bodies = tree["bodies"]
    bn = list(body_names) if body_names else [b.get("name", f"b{i}") for i, b in enumerate(bodies)]
    sn = list(site_names) if site_names else [s.get("name", f"s{k}") for k, s in enumerate(tree["sites"])]
    children = {i: [] for i in range(-1, len(bodies) + len(extra_bodies))}
    for i, b in enumerate(bodies):
        children[b["parent"]].append(i)
    extra = []
    for j, (name, parent, pos) in enumerate(extra_bodies):
        idx = len(bodies) + j
        children[parent].append(idx)
        extra.append(dict(name=name, pos=pos))
    sites_of = {}
    for k, s in enumerate(tree["sites"]):
        sites_of.setdefault(s["body"], []).append(k)
    out = [f'<mujoco model="{model_name}">', '  <compiler angle="radian"/>',
           f'  <option gravity="{_fmt(tree["gravity"])}"/>', "  <worldbody>"]

    def emit(i, ind):
        sp = "  " * ind
        if i >= len(bodies):
            e = extra[i - len(bodies)]
            out.append(f'{sp}<body name="{e["name"]}" pos="{_fmt(e["pos"])}">')
        else:
            b = bodies[i]
            out.append(f'{sp}<body name="{bn[i]}" pos="{_fmt(b["pos"])}" quat="{_fmt(b["quat"])}">')
            out.append(f'{sp}  <inertial pos="{_fmt(b["ipos"])}" quat="{_fmt(b["iquat"])}" '
                       f'mass="{float(b["mass"])!r}" diaginertia="{_fmt(b["diaginertia"])}"/>')
            joints = b["joints"] if "joints" in b else (
                [] if b["joint"] == "none" else
                [dict(type=b["joint"], axis=b.get("axis", [0, 0, 1]),
                      pos=b.get("jnt_pos", [0, 0, 0]), armature=b.get("armature", 0.0))])
            for n, j in enumerate(joints):
                jn = f"{bn[i]}_joint" if n == 0 else f"{bn[i]}_joint{n}"
                arm = float(j.get("armature", 0.0))
                if j["type"] == "free":
                    out.append(f'{sp}  <freejoint name="{bn[i]}_root"/>' if not arm else
                               f'{sp}  <joint name="{bn[i]}_root" type="free" armature="{arm!r}"/>')
                    continue
                ax = f' axis="{_fmt(j.get("axis", [0, 0, 1]))}"' if j["type"] != "ball" else ""
                out.append(f'{sp}  <joint name="{jn}" type="{j["type"]}"{ax} '
                           f'pos="{_fmt(j.get("pos", [0, 0, 0]))}" armature="{arm!r}"/>')
        for k in sites_of.get(i, []):
            out.append(f'{sp}  <site name="{sn[k]}" pos="{_fmt(tree["sites"][k]["pos"])}"/>')
        for c in children[i]:
            emit(c, ind + 1)
        out.append(f"{sp}</body>")

    for r in children[-1]:
        emit(r, 2)
    out += ["  </worldbody>", "</mujoco>", ""]
    return "\n".join(out)


def load_mjcf(xml_path: str, body_names, site_names, model_order: bool = False) -> dict:
    """osc_kin_desc_from_mjcf -> the JSON-schema dict (with per-site "jac_body")."""
    d = _lib.kin_desc_from_mjcf(xml_path, body_names, site_names, model_order)
    return _lib.kin_desc_to_dict(d, name=xml_path)


def load_mjcf_robot(robot: str, xml_path: str, yaml_path: str | None = None) -> dict:
    """osc_kin_desc_from_mjcf_robot: the robot's config lists and site convention."""
    d = _lib.kin_desc_from_mjcf_robot(robot, xml_path, yaml_path)
    return _lib.kin_desc_to_dict(d, name=xml_path)
