"""MJCF front door of the kinematics front end (include/osc_kinematics.h: osc_kin_desc_from_mjcf,
csrc/osc_mjcf.cpp): the reference builds its controller from the robot's MJCF path and resolves
task sites and bodies by name (unitree_go2/operational_space_controller.h:108-152).

CPU only (the reader is host code):
  * every JSON tree (illustrative Go2 / WaLTER, random trees, pendulum, free body) written out as
    MJCF reads back to the same descriptor -- bitwise where the tree has no welded bodies;
    welded bodies are fused into their parents and the oracle's M, C, J, b are unchanged;
  * MuJoCo conventions a hand-written file uses: degrees by default, euler / axisangle /
    xyaxes / zaxis frames, nested default classes with childclass / class, <freejoint>,
    fullinertia, fromto sites, gravity;
  * the two site conventions: WaLTER points by site name (W/osc.h:417), Go2 points by model
    order (G/osc.h:373) with Jacobian bodies from body_list -- pinned by finite differences of
    a point moving with the Jacobian body (mj_jac's semantics);
  * malformed or unsupported files are errors, not guesses.
"""
import json
import os

import numpy as np
import pytest

from osc_amd import _lib
from osc_amd.mjcf import load_mjcf, load_mjcf_robot, tree_to_mjcf

import kinematics as kin   # oracle (checker only)
from kin_trees import chain_tree, free_body, pendulum, random_tree

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = os.path.join(REPO, "operational-space-control_amd", "config")


def _json(robot):
    with open(os.path.join(CFG, f"{robot}_kinematics.json")) as fh:
        return json.load(fh)


def _names(tree):
    bn = [tree["bodies"][s["body"]].get("name", f"b{s['body']}") for s in tree["sites"]]
    sn = [s.get("name", f"s{k}") for k, s in enumerate(tree["sites"])]
    return bn, sn


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def _desc_equal(a, b, exact=True):
    for k in ("parent", "joint"):
        assert [x[k] for x in a["bodies"]] == [x[k] for x in b["bodies"]], k
    for k in ("pos", "quat", "ipos", "iquat", "diaginertia", "mass", "armature"):
        x = np.array([np.asarray(v[k], dtype=float) for v in a["bodies"]])
        y = np.array([np.asarray(v[k], dtype=float) for v in b["bodies"]])
        if exact:
            assert np.array_equal(x, y), k
        else:
            if k in ("quat", "iquat"):                 # MuJoCo normalises quaternions
                y = y / np.linalg.norm(y, axis=1, keepdims=True)
            assert np.allclose(x, y, rtol=0, atol=1e-15), k
    hinge = [i for i, v in enumerate(a["bodies"]) if v["joint"] == "hinge"]
    for k in ("axis", "jnt_pos"):
        x = np.array([a["bodies"][i][k] for i in hinge], dtype=float)
        y = np.array([b["bodies"][i][k] for i in hinge], dtype=float)
        assert np.array_equal(x, y), k
    assert [s["body"] for s in a["sites"]] == [s["body"] for s in b["sites"]]
    assert np.array_equal(np.array([s["pos"] for s in a["sites"]], dtype=float),
                          np.array([s["pos"] for s in b["sites"]], dtype=float))
    assert list(a["gravity"]) == list(map(float, b["gravity"]))


def _dfs(tree):
    """The tree renumbered in MuJoCo's body order (depth-first, document order), which is the
    order an MJCF file defines; the random trees are only parents-first."""
    kids = {i: [] for i in range(-1, len(tree["bodies"]))}
    for i, b in enumerate(tree["bodies"]):
        kids[b["parent"]].append(i)
    order = []

    def visit(i):
        order.append(i)
        for c in kids[i]:
            visit(c)
    for r in kids[-1]:
        visit(r)
    new = {o: k for k, o in enumerate(order)}
    bodies = [dict(tree["bodies"][o], parent=(-1 if tree["bodies"][o]["parent"] < 0 else
                                              new[tree["bodies"][o]["parent"]])) for o in order]
    sites = [dict(s, body=new[s["body"]]) for s in tree["sites"]]
    return dict(tree, bodies=bodies, sites=sites)


def _kin_close(ta, tb, seed=3, n=3, tol=1e-11):
    ma, mb = kin.KinModel(ta), kin.KinModel(tb)
    assert (ma.nq, ma.nv, ma.ns) == (mb.nq, mb.nv, mb.ns)
    rng = np.random.default_rng(seed)
    for _ in range(n):
        q, v = kin.random_state(ma, rng)
        for x, y in zip(kin.kinematics(ma, q, v), kin.kinematics(mb, q, v)):
            assert np.abs(x - y).max() <= tol * (1 + np.abs(y).max())


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_json_trees_roundtrip_bitwise(tmp_path, robot):
    tree = _json(robot)
    path = _write(tmp_path, "m.xml", tree_to_mjcf(tree))
    bn, sn = _names(tree)
    got = load_mjcf(path, bn, sn)
    _desc_equal(got, tree)
    assert all(s["jac_body"] == s["body"] for s in got["sites"])


@pytest.mark.parametrize("tree", [pendulum(), free_body(iquat=(0.9, 0.1, -0.3, 0.2)),
                                  chain_tree(5)], ids=["pendulum", "free_body", "chain16"])
def test_known_trees_roundtrip(tmp_path, tree):
    path = _write(tmp_path, "m.xml", tree_to_mjcf(tree))
    bn, sn = _names(tree)
    got = load_mjcf(path, bn, sn)
    _desc_equal(got, tree, exact=False)   # quaternions re-normalised by the reader
    _kin_close(got, tree)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_welded_bodies_fused_kinematics_unchanged(tmp_path, seed):
    """Random trees with massive welded bodies: fused into their parents (fewer bodies), sites
    and Jacobian bodies follow, and M, C, J, b of the oracle are unchanged."""
    tree = _dfs(random_tree(100 + seed, nbody=12, weld_p=0.3))
    nweld = sum(b["joint"] == "none" for b in tree["bodies"][1:])
    path = _write(tmp_path, "m.xml", tree_to_mjcf(tree))
    bn, sn = _names(tree)
    got = load_mjcf(path, bn, sn)
    assert len(got["bodies"]) == len(tree["bodies"]) - nweld
    assert all(b["joint"] != "none" for b in got["bodies"][1:])
    _kin_close(got, tree)


def test_robot_files_and_site_conventions():
    """config/<robot>.xml (tools/make_mjcf_models.py), read with the robot's config lists."""
    # WaLTER: points by name; the wheel bodies (massless frames) fuse into the shins -> the
    # descriptor is the JSON tree's, bitwise
    w = load_mjcf_robot("walter_sr", os.path.join(CFG, "walter_sr.xml"))
    jw = _json("walter_sr")
    _desc_equal(w, jw)
    assert [s["jac_body"] for s in w["sites"]] == [s["body"] for s in jw["sites"]]
    # Go2: body_list resolves by name, points are the model's sites 0..4 in model order: the
    # file declares the legs FL, FR, RL, RR, so task site "front_right_foot" (k = 1) takes the
    # FL foot's point and the FR calf's Jacobian -- G/osc.h:373 with such a file
    g = load_mjcf_robot("unitree_go2", os.path.join(CFG, "unitree_go2.xml"))
    jg = _json("unitree_go2")
    names = [b["name"] for b in jg["bodies"]]
    calf = {k: names.index(f"{k}_calf") for k in ("FL", "FR", "RL", "RR")}
    assert [s["jac_body"] for s in g["sites"]] == [0, calf["FR"], calf["FL"], calf["RR"], calf["RL"]]
    assert [s["body"] for s in g["sites"]] == [0, calf["FL"], calf["FR"], calf["RL"], calf["RR"]]
    _desc_equal(dict(g, sites=jg["sites"]), jg)


def test_jacobian_body_is_mj_jac_of_a_point_moving_with_that_body():
    """Oracle semantics of a site whose Jacobian body differs from its point's body: the columns
    are the derivative of the point carried rigidly by the Jacobian body."""
    tree = _json("unitree_go2")
    g = load_mjcf_robot("unitree_go2", os.path.join(CFG, "unitree_go2.xml"))
    m = kin.KinModel(g)
    rng = np.random.default_rng(11)
    q, v = kin.random_state(m, rng)
    M, C, J, b = kin.kinematics(m, q, v)
    xpos, xmat, _, _ = kin.forward(m, q)
    k = 1
    jb = g["sites"][k]["jac_body"]
    p = kin.site_positions(m, q)[k]
    local = xmat[jb].T @ (p - xpos[jb])          # the point in the Jacobian body's frame
    eps = 1e-7
    for c in range(m.nv):
        dv = np.zeros(m.nv)
        dv[c] = 1.0
        qp = kin.integrate(m, q, dv, eps)
        qm = kin.integrate(m, q, dv, -eps)
        xp, Rp, _, _ = kin.forward(m, qp)
        xm, Rm, _, _ = kin.forward(m, qm)
        fd = ((xp[jb] + Rp[jb] @ local) - (xm[jb] + Rm[jb] @ local)) / (2 * eps)
        assert np.abs(fd - J[3 * k:3 * k + 3, c]).max() < 1e-6
    assert tree["sites"][k]["body"] != g["sites"][k]["body"]


MJCF_FEATURES = """<?xml version="1.0"?>
<!-- hand-written: MuJoCo defaults and conventions -->
<mujoco model="features">
  <option gravity="0 0 -9.5" timestep="0.002"/>
  <default>
    <joint armature="0.01" damping="1"/>
    <site size="0.01"/>
    <default class="leg">
      <joint axis="0 1 0"/>
      <default class="knee">
        <joint armature="0.03" pos="0 0 0.01"/>
      </default>
    </default>
  </default>
  <asset><mesh name="m" file="x.stl"/></asset>
  <worldbody>
    <light pos="0 0 3"/>
    <geom type="plane" size="5 5 0.1"/>
    <body name="base" pos="0 0 0.4" euler="0 0 90">
      <freejoint/>
      <inertial pos="0 0 0" mass="4" fullinertia="0.1 0.2 0.3 0.01 0 0.02"/>
      <geom type="box" size="0.1 0.1 0.1"/>
      <site name="imu" pos="0.01 0 0.02"/>
      <body name="thigh" pos="0.1 0 0" axisangle="1 0 0 30" childclass="leg">
        <joint name="hip"/>
        <inertial pos="0 0 -0.1" mass="1" diaginertia="0.01 0.01 0.001"/>
        <body name="shin" pos="0 0 -0.2" xyaxes="0 1 0 -1 0 0">
          <joint name="knee" class="knee"/>
          <inertial pos="0 0 -0.1" quat="1 0 0 0" mass="0.5" diaginertia="0.005 0.005 0.0005"/>
          <site name="foot" fromto="0 0 -0.2 0 0 -0.22"/>
          <body name="toe" pos="0 0 -0.2" zaxis="1 0 0">
            <site name="toe_tip" pos="0.01 0 0"/>
          </body>
        </body>
      </body>
    </body>
  </worldbody>
  <actuator><motor joint="hip"/></actuator>
</mujoco>
"""


def _quat_axis(axis, ang):
    a = np.asarray(axis, dtype=float) / np.linalg.norm(axis)
    return np.concatenate([[np.cos(ang / 2)], np.sin(ang / 2) * a])


def test_hand_written_mjcf_conventions(tmp_path):
    path = _write(tmp_path, "f.xml", MJCF_FEATURES)
    d = load_mjcf(path, ["base", "shin", "toe"], ["imu", "foot", "toe_tip"])
    assert [b["joint"] for b in d["bodies"]] == ["free", "hinge", "hinge"]   # toe fused into shin
    assert d["gravity"] == [0.0, 0.0, -9.5]
    base, thigh, shin = d["bodies"]
    assert np.allclose(base["quat"], _quat_axis([0, 0, 1], np.pi / 2), atol=1e-15)   # degrees
    assert np.allclose(thigh["quat"], _quat_axis([1, 0, 0], np.pi / 6), atol=1e-15)
    assert np.allclose(shin["quat"], _quat_axis([0, 0, 1], np.pi / 2), atol=1e-15)   # xyaxes
    assert thigh["axis"] == [0.0, 1.0, 0.0] and thigh["armature"] == 0.01      # class leg < main
    assert shin["armature"] == 0.03 and shin["jnt_pos"] == [0.0, 0.0, 0.01]    # class knee
    assert base["armature"] == 0.01                                            # main on freejoint
    # fullinertia: principal moments and axes reproduce the tensor
    R = kin.quat2mat(base["iquat"])
    I = R @ np.diag(base["diaginertia"]) @ R.T
    assert np.allclose(I, [[0.1, 0.01, 0], [0.01, 0.2, 0.02], [0, 0.02, 0.3]], atol=1e-15)
    assert np.linalg.det(R) > 0
    # sites: fromto midpoint; the toe site moved into the shin's frame by the zaxis rotation
    assert np.allclose(d["sites"][1]["pos"], [0.0, 0.0, -0.21], atol=1e-16)
    assert d["sites"][2]["body"] == 2 and d["sites"][2]["jac_body"] == 2
    Rz = kin.quat2mat(_quat_axis([0, 1, 0], np.pi / 2))   # zaxis (1,0,0): +90 deg about y
    assert np.allclose(d["sites"][2]["pos"], np.array([0, 0, -0.2]) + Rz @ [0.01, 0, 0], atol=1e-15)
    # model order: imu, foot, toe_tip (same as the names here)
    d2 = load_mjcf(path, ["base", "shin", "toe"], ["x", "y", "z"], model_order=True)
    assert [s["pos"] for s in d2["sites"]] == [s["pos"] for s in d["sites"]]


def test_radian_and_eulerseq(tmp_path):
    text = """<mujoco><compiler angle="radian" eulerseq="zyx"/><worldbody>
      <body name="a" euler="0.3 -0.2 0.1"><joint type="hinge" axis="1 0 0"/>
      <inertial pos="0 0 0" mass="1" diaginertia="1 1 1"/><site name="s"/></body>
      <body name="b" euler="0.3 -0.2 0.1"><joint type="hinge" axis="1 0 0"/>
      <inertial pos="0 0 0" mass="1" diaginertia="1 1 1"/></body></worldbody></mujoco>"""
    d = load_mjcf(_write(tmp_path, "r.xml", text), ["a"], ["s"])
    # intrinsic z, then y', then x'': q = qz * qy * qx
    def qmul(a, b):
        w1, x1, y1, z1 = a
        w2, x2, y2, z2 = b
        return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                         w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
    q = qmul(qmul(_quat_axis([0, 0, 1], 0.3), _quat_axis([0, 1, 0], -0.2)), _quat_axis([1, 0, 0], 0.1))
    assert np.allclose(d["bodies"][0]["quat"], q, atol=1e-15)
    assert d["bodies"][1]["parent"] == -1


@pytest.mark.parametrize("text,why", [
    ("<mujoco><worldbody><body name='a'><joint/><geom size='1'/></body></worldbody></mujoco>",
     "inertia from geoms"),
    ("<mujoco><worldbody><body name='a'><joint type='slide'/><inertial pos='0 0 0' mass='1' "
     "diaginertia='1 1 1'/></body></worldbody></mujoco>", "slide joint"),
    ("<mujoco><worldbody><body name='a'><joint/><joint/><inertial pos='0 0 0' mass='1' "
     "diaginertia='1 1 1'/></body></worldbody></mujoco>", "two joints"),
    ("<mujoco><worldbody><body name='a' class='nope'><joint class='nope'/><inertial pos='0 0 0' "
     "mass='1' diaginertia='1 1 1'/></body></worldbody></mujoco>", "unknown class"),
    ("<mujoco><worldbody><body name='a'><joint/>", "unterminated"),
    ("<mujoco><include file='x.xml'/><worldbody/></mujoco>", "include"),
    ("<mujoco><worldbody><site name='s'/><body name='a'><joint/><inertial pos='0 0 0' mass='1' "
     "diaginertia='1 1 1'/></body></worldbody></mujoco>", "world site as task site"),
    ("<mujoco><worldbody><body name='a'><joint/><inertial pos='0 0 0' mass='1' "
     "diaginertia='1 1 1'/><site name='t'/></body></worldbody></mujoco>", "unknown site name"),
])
def test_errors(tmp_path, text, why):
    path = _write(tmp_path, "e.xml", text)
    order = why == "world site as task site"
    with pytest.raises(_lib.OSCError) as e:
        load_mjcf(path, ["a"], ["s"], model_order=order)
    assert e.value.code == 3, why   # OSC_ERR_IO


def test_missing_file_and_bad_args(tmp_path):
    with pytest.raises(_lib.OSCError) as e:
        load_mjcf(str(tmp_path / "none.xml"), ["a"], ["s"])
    assert e.value.code == 3
    with pytest.raises(_lib.OSCError) as e:
        load_mjcf_robot("no_such_robot", os.path.join(CFG, "unitree_go2.xml"))
    assert e.value.code == 1
