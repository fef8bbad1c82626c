"""CPU oracle, part 3: rigid-body kinematics of a floating-base tree -- what the reference asks
MuJoCo for each tick (§8(f) row 1 moves it onto the GPU).

TEST INFRASTRUCTURE ONLY (see osc_qp.py): only tests/ and __graft_entry__.smoke() import it.

The reference (paths relative to /root/reference/operational-space-control):
  * update_mj_data: qpos = [0,0,0, quat (w,x,y,z), q_m], qvel = [v, omega, qd_m], then
    mj_fwdPosition / mj_fwdVelocity ................ unitree_go2/operational_space_controller.h:350-374
  * update_osc_data: M = mj_fullM, C = qfrc_bias, per site Jp, Jr = mj_jac(site_xpos, body),
    Jpd, Jrd = mj_jacDot, J = [Jp_0..; Jr_0..], b = [Jpd; Jrd] qvel ... :376-455
MuJoCo 3.2.7 (MODULE.bazel.lock:242-247) is not vendored and not installed, so this restates
its published semantics: mj_kinematics (free joint: xpos = qpos[0:3], xquat = qpos[3:7];
hinge: rotation about the body-frame axis through the body-frame anchor; slide: translation
along the body-frame axis; ball: rotation by the quaternion qpos about the anchor; several
joints on one body act in order), qvel of a free joint = (world-frame linear velocity of the
body origin, body-frame angular velocity), of a ball the body-frame angular velocity, mj_fullM
(including dof armature), qfrc_bias = RNE with zero joint acceleration (Coriolis, centrifugal
and gravity), mj_jac / mj_jacDot of a point fixed to a body, world frame.

The formulation here is deliberately different from the kernel's (spatial-vector CRBA/RNEA in
world coordinates, osc_kinematics.hip): M = sum over bodies of m Jc'Jc + Jw' I Jw (body COM and
angular Jacobians), C by Kane's method from the classical bias accelerations of every body.
PARITY STATUS: unpinned against MuJoCo (no MuJoCo, no robot XMLs here); pinned by physical
identities in tests/test_kinematics_oracle.py: Jacobians against finite differences of the
forward kinematics, J-dot q-dot against finite differences of J q-dot, C(q, 0) against the
gravity potential, and energy conservation of the free (unactuated) motion M qdd + C = 0.
"""
from __future__ import annotations

import json
import os

import numpy as np

CONFIG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                      "operational-space-control_amd", "config")


def quat2mat(q):
    w, x, y, z = np.asarray(q, dtype=np.float64) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def axis_angle(a, t):
    a = np.asarray(a, dtype=np.float64)
    a = a / np.linalg.norm(a)
    K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
    return np.eye(3) + np.sin(t) * K + (1 - np.cos(t)) * K @ K


class KinModel:
    """A tree in the <robot>_kinematics.json schema.  A body carries one joint ("joint": "free" |
    "ball" | "slide" | "hinge" | "none", with "axis", "jnt_pos", "armature") or, as MuJoCo allows,
    a list of them ("joints": [{"type", "axis", "pos", "armature"}, ...], applied in order) --
    the list form is restated directly here, while the kernel's descriptor holds one joint per
    body and the MJCF reader splits such a body into a chain (csrc/osc_mjcf.cpp)."""

    NQ = {"free": 7, "ball": 4, "slide": 1, "hinge": 1}
    NV = {"free": 6, "ball": 3, "slide": 1, "hinge": 1}

    def __init__(self, d):
        self.d = d
        self.bodies = d["bodies"]
        self.sites = d["sites"]
        self.gravity = np.array(d["gravity"], dtype=np.float64)
        self.nbody = len(self.bodies)
        self.joints = []          # flat, in body order: type, body, axis, pos, qadr, dadr
        self.body_joints = []     # per body: indices into self.joints
        self.qadr, self.dadr = [], []   # per body: first qpos / dof of its joints
        nq = nv = 0
        arm = []
        for i, b in enumerate(self.bodies):
            if "joints" in b:
                js = [dict(type=j["type"], axis=j.get("axis", [0.0, 0.0, 1.0]),
                           pos=j.get("pos", [0.0, 0.0, 0.0]), armature=j.get("armature", 0.0))
                      for j in b["joints"]]
            elif b["joint"] == "none":
                js = []
            else:
                js = [dict(type=b["joint"], axis=b.get("axis", [0.0, 0.0, 1.0]),
                           pos=b.get("jnt_pos", [0.0, 0.0, 0.0]), armature=b.get("armature", 0.0))]
            self.qadr.append(nq)
            self.dadr.append(nv)
            self.body_joints.append([])
            for j in js:
                if j["type"] not in self.NQ:
                    raise ValueError(f"joint type {j['type']}")
                ax = np.asarray(j["axis"], dtype=np.float64)
                self.body_joints[i].append(len(self.joints))
                self.joints.append(dict(type=j["type"], body=i, axis=ax / np.linalg.norm(ax),
                                        pos=np.asarray(j["pos"], dtype=np.float64), qadr=nq,
                                        dadr=nv))
                nq += self.NQ[j["type"]]
                nv += self.NV[j["type"]]
                arm += [float(j["armature"])] * self.NV[j["type"]]
        self.nq, self.nv, self.ns = nq, nv, len(self.sites)
        self.njnt = len(self.joints)
        self.armature = np.array(arm, dtype=np.float64)   # dof_armature: every dof of the joint
        # body inertia about the COM, body frame
        self.Ibody = [quat2mat(b["iquat"]) @ np.diag(b["diaginertia"]) @ quat2mat(b["iquat"]).T
                      for b in self.bodies]

    def chain(self, bi):
        out = []
        while bi >= 0:
            out.append(bi)
            bi = self.bodies[bi]["parent"]
        return out[::-1]


def load(robot):
    with open(os.path.join(CONFIG, f"{robot}_kinematics.json")) as f:
        return KinModel(json.load(f))


def forward(m: KinModel, qpos):
    """mj_kinematics: body frames (xpos, xmat) and, per joint (m.joints order), its world anchor
    and world axis (hinge, slide) at the instant the joint is applied -- a body's joints act in
    order, each on the frame the previous ones left (MuJoCo 3.2.7 engine_core_smooth.c)."""
    xpos = np.zeros((m.nbody, 3))
    xmat = np.zeros((m.nbody, 3, 3))
    anchor = np.zeros((m.njnt, 3))
    axis = np.zeros((m.njnt, 3))
    for i, b in enumerate(m.bodies):
        p = b["parent"]
        pp = xpos[p] if p >= 0 else np.zeros(3)
        pR = xmat[p] if p >= 0 else np.eye(3)
        pos = pp + pR @ np.asarray(b["pos"], dtype=np.float64)
        R = pR @ quat2mat(b["quat"])
        for ji in m.body_joints[i]:
            j = m.joints[ji]
            qa = j["qadr"]
            if j["type"] == "free":
                pos = np.array(qpos[qa:qa + 3], dtype=np.float64)
                R = quat2mat(qpos[qa + 3:qa + 7])
                anchor[ji] = pos
                continue
            axis[ji] = R @ j["axis"]
            if j["type"] == "slide":
                pos = pos + axis[ji] * qpos[qa]
                anchor[ji] = pos
                continue
            anchor[ji] = pos + R @ j["pos"]
            if j["type"] == "hinge":
                R = R @ axis_angle(j["axis"], qpos[qa])
            else:   # ball
                R = R @ quat2mat(qpos[qa:qa + 4])
            pos = anchor[ji] - R @ j["pos"]
        xpos[i], xmat[i] = pos, R
    return xpos, xmat, anchor, axis


def point_jacobian(m: KinModel, fk, bi, point):
    """mj_jac: (Jp, Jr), 3 x nv each, of a point fixed to body bi."""
    xpos, xmat, anchor, axis = fk
    Jp = np.zeros((3, m.nv))
    Jr = np.zeros((3, m.nv))
    for c in m.chain(bi):
        for ji in m.body_joints[c]:
            j = m.joints[ji]
            da = j["dadr"]
            if j["type"] == "free":
                Jp[:, da:da + 3] = np.eye(3)
                for k in range(3):
                    a = xmat[c][:, k]
                    Jr[:, da + 3 + k] = a
                    Jp[:, da + 3 + k] = np.cross(a, point - xpos[c])
            elif j["type"] == "ball":
                # MuJoCo's ball dofs rotate about the axes of the body's final frame (mj_comPos);
                # the MJCF reader admits a ball only as its body's last rotating joint, where that
                # frame is the joint's own
                for k in range(3):
                    a = xmat[c][:, k]
                    Jr[:, da + k] = a
                    Jp[:, da + k] = np.cross(a, point - anchor[ji])
            elif j["type"] == "hinge":
                Jr[:, da] = axis[ji]
                Jp[:, da] = np.cross(axis[ji], point - anchor[ji])
            else:   # slide
                Jp[:, da] = axis[ji]
    return Jp, Jr


def bias_motion(m: KinModel, fk, qvel):
    """Per body, with zero joint acceleration: angular velocity w, angular acceleration al, and
    (o, v_o, a_o) = a reference point fixed to the body with its velocity and acceleration.  A
    body's joints are walked in order, each moving the frame the previous ones left."""
    xpos, xmat, anchor, axis = fk
    w = np.zeros((m.nbody, 3))
    al = np.zeros((m.nbody, 3))
    o = np.zeros((m.nbody, 3))
    vo = np.zeros((m.nbody, 3))
    ao = np.zeros((m.nbody, 3))

    def state_at(fr, x):     # velocity / acceleration of the point x fixed to frame fr
        fw, fal, fo, fvo, fao = fr
        r = x - fo
        return fvo + np.cross(fw, r), fao + np.cross(fal, r) + np.cross(fw, np.cross(fw, r))

    for i, b in enumerate(m.bodies):
        p = b["parent"]
        if p >= 0:
            fr = (w[p], al[p], o[p], vo[p], ao[p])
        else:
            z = np.zeros(3)
            fr = (z, z, z, z, z)
        for ji in m.body_joints[i]:
            j = m.joints[ji]
            da = j["dadr"]
            fw, fal = fr[0], fr[1]
            if j["type"] == "free":
                # world-frame linear velocity of the origin and body-frame angular velocity, both
                # constant at zero acceleration (d/dt (R w_local) = w x w = 0)
                fr = (xmat[i] @ qvel[da + 3:da + 6], np.zeros(3), xpos[i].copy(),
                      np.array(qvel[da:da + 3], dtype=np.float64), np.zeros(3))
            elif j["type"] == "hinge":
                v0, a0 = state_at(fr, anchor[ji])
                wj = axis[ji] * qvel[da]
                fr = (fw + wj, fal + np.cross(fw, wj), anchor[ji].copy(), v0, a0)
            elif j["type"] == "ball":
                v0, a0 = state_at(fr, anchor[ji])
                wj = xmat[i] @ qvel[da:da + 3]
                fr = (fw + wj, fal + np.cross(fw, wj), anchor[ji].copy(), v0, a0)
            else:   # slide: the new origin moves along the axis fixed in the previous frame
                v0, a0 = state_at(fr, anchor[ji])
                vr = axis[ji] * qvel[da]
                fr = (fw, fal, anchor[ji].copy(), v0 + vr, a0 + 2.0 * np.cross(fw, vr))
        w[i], al[i] = fr[0], fr[1]
        if m.body_joints[i]:
            o[i], vo[i], ao[i] = fr[2], fr[3], fr[4]
        else:   # welded: the parent's motion, referred to this body's origin
            o[i] = xpos[i]
            vo[i], ao[i] = state_at(fr, xpos[i])

    def accel(bi, x):
        return state_at((w[bi], al[bi], o[bi], vo[bi], ao[bi]), x)
    return w, al, accel


def kinematics(m: KinModel, qpos, qvel):
    """(M, C, J, b) exactly as update_osc_data stores them: M nv x nv, C nv, J (6 ns) x nv with
    rows [Jp_0; ..; Jp_{ns-1}; Jr_0; ..; Jr_{ns-1}], b = [Jpd; Jrd] qvel."""
    qpos = np.asarray(qpos, dtype=np.float64)
    qvel = np.asarray(qvel, dtype=np.float64)
    fk = forward(m, qpos)
    xpos, xmat, _, _ = fk
    w, al, accel = bias_motion(m, fk, qvel)
    M = np.diag(m.armature).astype(np.float64)
    C = np.zeros(m.nv)
    for i, b in enumerate(m.bodies):
        com = xpos[i] + xmat[i] @ np.asarray(b["ipos"])
        Jc, Jw = point_jacobian(m, fk, i, com)
        Iw = xmat[i] @ m.Ibody[i] @ xmat[i].T
        M += b["mass"] * Jc.T @ Jc + Jw.T @ Iw @ Jw
        _, a_com = accel(i, com)
        C += Jc.T @ (b["mass"] * (a_com - m.gravity)) + Jw.T @ (Iw @ al[i] + np.cross(w[i], Iw @ w[i]))
    ns = m.ns
    J = np.zeros((6 * ns, m.nv))
    bb = np.zeros(6 * ns)
    for k, s in enumerate(m.sites):
        bi = s["body"]
        x = xpos[bi] + xmat[bi] @ np.asarray(s["pos"])
        # mj_jac(point, body_ids[k]): the point is the site's, the rigid motion is the Jacobian
        # body's (unitree_go2/operational_space_controller.h:409-412; "jac_body" absent = same)
        jb = s.get("jac_body", bi)
        Jp, Jr = point_jacobian(m, fk, jb, x)
        J[3 * k:3 * k + 3] = Jp
        J[3 * ns + 3 * k:3 * ns + 3 * k + 3] = Jr
        _, a = accel(jb, x)
        bb[3 * k:3 * k + 3] = a
        bb[3 * ns + 3 * k:3 * ns + 3 * k + 3] = al[jb]
    return M, C, J, bb


def site_positions(m: KinModel, qpos):
    xpos, xmat, _, _ = forward(m, np.asarray(qpos, dtype=np.float64))
    return np.array([xpos[s["body"]] + xmat[s["body"]] @ np.asarray(s["pos"]) for s in m.sites])


def _quat_step(q, wl):
    """q * exp(wl / 2): mju_quatIntegrate with a body-frame rotation vector wl."""
    th = np.linalg.norm(wl)
    dq = np.array([1.0, 0, 0, 0]) if th == 0 else np.concatenate(
        [[np.cos(th / 2)], np.sin(th / 2) * wl / th])
    w0, x0, y0, z0 = q
    w1, x1, y1, z1 = dq
    qn = np.array([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1,
                   w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                   w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1,
                   w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1])
    return qn / np.linalg.norm(qn)


def integrate(m: KinModel, qpos, qvel, dt):
    """mj_integratePos: free joint pos += v dt, quat <- quat * exp(w_local dt / 2); ball likewise
    for its quaternion; hinge / slide q += qd dt."""
    q = np.array(qpos, dtype=np.float64)
    for j in m.joints:
        qa, da = j["qadr"], j["dadr"]
        if j["type"] == "free":
            q[qa:qa + 3] += qvel[da:da + 3] * dt
            q[qa + 3:qa + 7] = _quat_step(q[qa + 3:qa + 7], np.asarray(qvel[da + 3:da + 6]) * dt)
        elif j["type"] == "ball":
            q[qa:qa + 4] = _quat_step(q[qa:qa + 4], np.asarray(qvel[da:da + 3]) * dt)
        else:
            q[qa] += qvel[da] * dt
    return q


def potential(m: KinModel, qpos):
    xpos, xmat, _, _ = forward(m, np.asarray(qpos, dtype=np.float64))
    e = 0.0
    for i, b in enumerate(m.bodies):
        com = xpos[i] + xmat[i] @ np.asarray(b["ipos"])
        e -= b["mass"] * m.gravity @ com
    return e


def random_state(m: KinModel, rng, base_pos_zero=True):
    """A random (qpos, qvel): unit base / ball quaternions, joint angles in +-1 rad, slides in
    +-0.3, velocities ~N(0,1) (base position 0 as update_mj_data sets it, unless base_pos_zero
    is False)."""
    qpos = np.zeros(m.nq)
    qvel = rng.normal(size=m.nv)
    for j in m.joints:
        qa = j["qadr"]
        if j["type"] == "free":
            qpos[qa:qa + 3] = 0.0 if base_pos_zero else rng.normal(size=3) * 0.3
            qq = rng.normal(size=4)
            qpos[qa + 3:qa + 7] = qq / np.linalg.norm(qq)
        elif j["type"] == "ball":
            qq = rng.normal(size=4)
            qpos[qa:qa + 4] = qq / np.linalg.norm(qq)
        elif j["type"] == "hinge":
            qpos[qa] = rng.uniform(-1.0, 1.0)
        else:
            qpos[qa] = rng.uniform(-0.3, 0.3)
    return qpos, qvel
