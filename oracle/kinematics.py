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
hinge: rotation about the body-frame axis through the body-frame anchor), qvel of a free joint
= (world-frame linear velocity of the body origin, body-frame angular velocity), mj_fullM
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
    def __init__(self, d):
        self.d = d
        self.bodies = d["bodies"]
        self.sites = d["sites"]
        self.gravity = np.array(d["gravity"], dtype=np.float64)
        self.nbody = len(self.bodies)
        self.qadr, self.dadr = [], []
        nq = nv = 0
        for b in self.bodies:
            self.qadr.append(nq)
            self.dadr.append(nv)
            if b["joint"] == "free":
                nq += 7
                nv += 6
            elif b["joint"] == "hinge":
                nq += 1
                nv += 1
        self.nq, self.nv, self.ns = nq, nv, len(self.sites)
        self.armature = np.zeros(nv)
        for b, da in zip(self.bodies, self.dadr):   # dof_armature: every dof of the joint
            ndof = {"free": 6, "hinge": 1}.get(b["joint"], 0)
            self.armature[da:da + ndof] = b.get("armature", 0.0)
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
    """Body frames (xpos, xmat) and, per hinge, its world anchor and axis."""
    xpos = np.zeros((m.nbody, 3))
    xmat = np.zeros((m.nbody, 3, 3))
    anchor = np.zeros((m.nbody, 3))
    axis = np.zeros((m.nbody, 3))
    for i, b in enumerate(m.bodies):
        p = b["parent"]
        pp = xpos[p] if p >= 0 else np.zeros(3)
        pR = xmat[p] if p >= 0 else np.eye(3)
        if b["joint"] == "free":
            qa = m.qadr[i]
            xpos[i] = qpos[qa:qa + 3]
            xmat[i] = quat2mat(qpos[qa + 3:qa + 7])
            continue
        pos = pp + pR @ np.asarray(b["pos"])
        R = pR @ quat2mat(b["quat"])
        if b["joint"] == "hinge":
            jp = np.asarray(b["jnt_pos"])
            anchor[i] = pos + R @ jp
            axis[i] = R @ (np.asarray(b["axis"]) / np.linalg.norm(b["axis"]))
            R = R @ axis_angle(b["axis"], qpos[m.qadr[i]])
            pos = anchor[i] - R @ jp
        xpos[i], xmat[i] = pos, R
    return xpos, xmat, anchor, axis


def point_jacobian(m: KinModel, fk, bi, point):
    """mj_jac: (Jp, Jr), 3 x nv each, of a point fixed to body bi."""
    xpos, xmat, anchor, axis = fk
    Jp = np.zeros((3, m.nv))
    Jr = np.zeros((3, m.nv))
    for c in m.chain(bi):
        b = m.bodies[c]
        da = m.dadr[c]
        if b["joint"] == "free":
            Jp[:, da:da + 3] = np.eye(3)
            for k in range(3):
                a = xmat[c][:, k]
                Jr[:, da + 3 + k] = a
                Jp[:, da + 3 + k] = np.cross(a, point - xpos[c])
        elif b["joint"] == "hinge":
            Jr[:, da] = axis[c]
            Jp[:, da] = np.cross(axis[c], point - anchor[c])
    return Jp, Jr


def bias_motion(m: KinModel, fk, qvel):
    """Per body, with zero joint acceleration: angular velocity w, angular acceleration al, and
    (o, v_o, a_o) = a reference point fixed to the body with its velocity and acceleration."""
    xpos, xmat, anchor, axis = fk
    w = np.zeros((m.nbody, 3))
    al = np.zeros((m.nbody, 3))
    o = np.zeros((m.nbody, 3))
    vo = np.zeros((m.nbody, 3))
    ao = np.zeros((m.nbody, 3))

    def point_state(p, x):     # velocity / acceleration of the point x fixed to body p
        r = x - o[p]
        v = vo[p] + np.cross(w[p], r)
        a = ao[p] + np.cross(al[p], r) + np.cross(w[p], np.cross(w[p], r))
        return v, a

    for i, b in enumerate(m.bodies):
        p = b["parent"]
        da = m.dadr[i]
        if b["joint"] == "free":
            o[i] = xpos[i]
            vo[i] = qvel[da:da + 3]               # world-frame linear velocity, constant
            w[i] = xmat[i] @ qvel[da + 3:da + 6]  # body-frame angular velocity, constant:
            al[i] = 0.0                           # d/dt (R w_local) = w x w = 0
            ao[i] = 0.0
            continue
        if b["joint"] == "hinge":
            o[i] = anchor[i]
        else:
            o[i] = xpos[i]
        if p >= 0:
            vo[i], ao[i] = point_state(p, o[i])
            wp, alp = w[p], al[p]
        else:
            vo[i] = ao[i] = 0.0
            wp = alp = np.zeros(3)
        if b["joint"] == "hinge":
            qd = qvel[da]
            w[i] = wp + axis[i] * qd
            al[i] = alp + np.cross(wp, axis[i] * qd)
        else:
            w[i], al[i] = wp, alp

    def accel(bi, x):
        return point_state(bi, x)
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


def integrate(m: KinModel, qpos, qvel, dt):
    """mj_integratePos: free joint pos += v dt, quat <- quat * exp(w_local dt / 2); hinge q += qd dt."""
    q = np.array(qpos, dtype=np.float64)
    for i, b in enumerate(m.bodies):
        qa, da = m.qadr[i], m.dadr[i]
        if b["joint"] == "free":
            q[qa:qa + 3] += qvel[da:da + 3] * dt
            wl = np.asarray(qvel[da + 3:da + 6]) * dt
            th = np.linalg.norm(wl)
            dq = np.array([1.0, 0, 0, 0]) if th == 0 else np.concatenate(
                [[np.cos(th / 2)], np.sin(th / 2) * wl / th])
            w0, x0, y0, z0 = q[qa + 3:qa + 7]
            w1, x1, y1, z1 = dq
            qn = np.array([w0 * w1 - x0 * x1 - y0 * y1 - z0 * z1,
                           w0 * x1 + x0 * w1 + y0 * z1 - z0 * y1,
                           w0 * y1 - x0 * z1 + y0 * w1 + z0 * x1,
                           w0 * z1 + x0 * y1 - y0 * x1 + z0 * w1])
            q[qa + 3:qa + 7] = qn / np.linalg.norm(qn)
        elif b["joint"] == "hinge":
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
    """A random (qpos, qvel): unit base quaternion, joint angles in +-1 rad, velocities ~N(0,1)
    (base position 0 as update_mj_data sets it, unless base_pos_zero is False)."""
    qpos = np.zeros(m.nq)
    qvel = rng.normal(size=m.nv)
    for i, b in enumerate(m.bodies):
        qa = m.qadr[i]
        if b["joint"] == "free":
            qpos[qa:qa + 3] = 0.0 if base_pos_zero else rng.normal(size=3) * 0.3
            qq = rng.normal(size=4)
            qpos[qa + 3:qa + 7] = qq / np.linalg.norm(qq)
        elif b["joint"] == "hinge":
            qpos[qa] = rng.uniform(-1.0, 1.0)
    return qpos, qvel
