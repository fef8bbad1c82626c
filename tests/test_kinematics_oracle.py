"""CPU checks of the kinematics oracle (oracle/kinematics.py) against physical identities -- the
pins that stand in for MuJoCo, which is absent here (parity against it stays unpinned):
  * Jp qvel / Jr qvel = finite-difference velocity of each site / body orientation,
  * b = d/dt (J) qvel = finite difference of J qvel along the motion,
  * 1/2 qvel' M qvel = kinetic energy from finite-difference body velocities,
  * C(q, 0) = gradient of the gravity potential,
  * qvel' (C(q, qvel) - C(q, 0)) = 1/2 qvel' Mdot qvel  (energy balance of the velocity terms),
  * M symmetric positive definite, armature on the diagonal."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "oracle"))
import kinematics as kin  # noqa: E402
from kin_trees import (chain_tree, free_body, mixed_tree, multi_joint_tree, pendulum,  # noqa: E402
                       random_tree, slider, spherical_pendulum, two_joint_body)

ROBOTS = ["unitree_go2", "walter_sr", "random_free", "random_fixed", "chain", "mixed",
          "mixed_fixed", "multi_joint"]
EPS = 1e-6


def _load(name):
    if name == "random_free":
        return kin.KinModel(random_tree(5))
    if name == "random_fixed":
        return kin.KinModel(random_tree(6, free_root=False))
    if name == "chain":
        return kin.KinModel(chain_tree(7))
    if name == "mixed":
        return kin.KinModel(mixed_tree(8))
    if name == "mixed_fixed":
        return kin.KinModel(mixed_tree(9, free_root=False))
    if name == "multi_joint":
        return kin.KinModel(multi_joint_tree(10))
    return kin.load(name)


def _rot_vee(Rd):
    """Angle-axis vector of a small rotation matrix."""
    A = 0.5 * (Rd - Rd.T)
    return np.array([A[2, 1], A[0, 2], A[1, 0]])


@pytest.mark.parametrize("robot", ROBOTS[:2])
def test_sizes_match_the_qp_models(robot):
    m = kin.load(robot)
    nv, ns = {"unitree_go2": (18, 5), "walter_sr": (14, 17)}[robot]
    assert (m.nv, m.ns, m.nq) == (nv, ns, nv + 1)


@pytest.mark.parametrize("robot", ROBOTS)
def test_jacobians_match_finite_differences(robot):
    m = _load(robot)
    rng = np.random.default_rng(11)
    for _ in range(3):
        q, v = kin.random_state(m, rng, base_pos_zero=False)
        M, C, J, b = kin.kinematics(m, q, v)
        qp, qm = kin.integrate(m, q, v, EPS), kin.integrate(m, q, v, -EPS)
        vel = (kin.site_positions(m, qp) - kin.site_positions(m, qm)) / (2 * EPS)
        np.testing.assert_allclose(J[:3 * m.ns].reshape(m.ns, 3, -1) @ v, vel, rtol=0, atol=1e-7)
        _, Rp, _, _ = kin.forward(m, qp)
        _, Rm, _, _ = kin.forward(m, qm)
        for k, s in enumerate(m.sites):
            w = _rot_vee(Rp[s["body"]] @ Rm[s["body"]].T) / (2 * EPS)
            np.testing.assert_allclose(J[3 * m.ns + 3 * k:3 * m.ns + 3 * k + 3] @ v, w,
                                       rtol=0, atol=1e-7)


@pytest.mark.parametrize("robot", ROBOTS)
def test_jdot_qdot_matches_finite_differences(robot):
    m = _load(robot)
    rng = np.random.default_rng(12)
    for _ in range(3):
        q, v = kin.random_state(m, rng)
        _, _, _, b = kin.kinematics(m, q, v)
        Jp = kin.kinematics(m, kin.integrate(m, q, v, EPS), v)[2]
        Jm = kin.kinematics(m, kin.integrate(m, q, v, -EPS), v)[2]
        np.testing.assert_allclose((Jp - Jm) @ v / (2 * EPS), b, rtol=0,
                                   atol=1e-6 * (1 + np.abs(b).max()))


@pytest.mark.parametrize("robot", ROBOTS)
def test_mass_matrix_is_the_kinetic_energy(robot):
    m = _load(robot)
    rng = np.random.default_rng(13)
    for _ in range(3):
        q, v = kin.random_state(m, rng)
        M = kin.kinematics(m, q, v)[0]
        assert np.allclose(M, M.T, atol=1e-14)
        assert np.linalg.eigvalsh(M).min() > 0
        qp, qm = kin.integrate(m, q, v, EPS), kin.integrate(m, q, v, -EPS)
        xp, Rp, _, _ = kin.forward(m, qp)
        xm, Rm, _, _ = kin.forward(m, qm)
        _, R0, _, _ = kin.forward(m, q)
        ke = 0.5 * float(np.sum(m.armature * v * v))
        for i, bd in enumerate(m.bodies):
            ip = np.asarray(bd["ipos"])
            vc = ((xp[i] + Rp[i] @ ip) - (xm[i] + Rm[i] @ ip)) / (2 * EPS)
            w = _rot_vee(Rp[i] @ Rm[i].T) / (2 * EPS)
            Iw = R0[i] @ m.Ibody[i] @ R0[i].T
            ke += 0.5 * (bd["mass"] * vc @ vc + w @ Iw @ w)
        assert abs(0.5 * v @ M @ v - ke) <= 1e-7 * (1 + ke)


@pytest.mark.parametrize("robot", ROBOTS)
def test_bias_gravity_and_energy_balance(robot):
    m = _load(robot)
    rng = np.random.default_rng(14)
    for _ in range(3):
        q, v = kin.random_state(m, rng)
        M, C, _, _ = kin.kinematics(m, q, v)
        g = kin.kinematics(m, q, np.zeros(m.nv))[1]
        # C(q, 0) = dV/dq along every dof direction (integrate = the dof's own motion)
        grad = np.zeros(m.nv)
        for i in range(m.nv):
            e = np.zeros(m.nv)
            e[i] = 1.0
            grad[i] = (kin.potential(m, kin.integrate(m, q, e, EPS)) -
                       kin.potential(m, kin.integrate(m, q, e, -EPS))) / (2 * EPS)
        np.testing.assert_allclose(g, grad, rtol=0, atol=1e-6 * (1 + np.abs(g).max()))
        # qvel' c(q, qvel) = 1/2 qvel' Mdot qvel
        Mp = kin.kinematics(m, kin.integrate(m, q, v, EPS), v)[0]
        Mm = kin.kinematics(m, kin.integrate(m, q, v, -EPS), v)[0]
        lhs = v @ (C - g)
        rhs = 0.5 * v @ ((Mp - Mm) / (2 * EPS)) @ v
        assert abs(lhs - rhs) <= 1e-6 * (1 + abs(lhs))


def pendulum_known_answer(th, thd, mass=1.5, length=0.7, izz=1e-3, armature=0.05, g=9.81):
    """Closed forms (MuJoCo conventions): hinge about +y, bob at -L z rotated by th about y:
    p = (-L sin th, 0, -L cos th).  M = m L^2 + I + armature; qfrc_bias = m g L sin th (gravity
    only, no velocity terms for one dof); Jp = dp/dth; Jpdot thd = d^2p/dt^2 at thdd = 0."""
    L = length
    M = mass * L * L + izz + armature
    C = mass * g * L * np.sin(th)
    Jp = np.array([-L * np.cos(th), 0.0, L * np.sin(th)])
    bp = np.array([L * np.sin(th), 0.0, L * np.cos(th)]) * thd * thd
    return M, C, Jp, bp


def test_pendulum_known_answer():
    m = kin.KinModel(pendulum())
    for th, thd in ((0.3, 1.2), (-1.1, -0.4), (2.5, 3.0)):
        M, C, J, b = kin.kinematics(m, np.array([th]), np.array([thd]))
        Mk, Ck, Jp, bp = pendulum_known_answer(th, thd)
        np.testing.assert_allclose(M[0, 0], Mk, rtol=1e-14)
        np.testing.assert_allclose(C[0], Ck, rtol=1e-13, atol=1e-13)
        np.testing.assert_allclose(J[:3, 0], Jp, atol=1e-15)
        np.testing.assert_allclose(J[3:, 0], [0.0, 1.0, 0.0], atol=1e-15)   # Jr = hinge axis
        np.testing.assert_allclose(b[:3], bp, atol=1e-13)
        np.testing.assert_allclose(b[3:], 0.0, atol=1e-15)


def free_body_known_answer(quat, v, w_body, mass=2.0, diag=(0.1, 0.2, 0.3), g=9.81):
    """Free body, COM at the origin: MuJoCo's rotational dofs are body axes, so
    M = blockdiag(m I3, I_body) and qfrc_bias = (m g e_z, w x (I_body w)) in those coordinates."""
    Ib = np.diag(diag)
    M = np.zeros((6, 6))
    M[:3, :3] = mass * np.eye(3)
    M[3:, 3:] = Ib
    C = np.concatenate([[0.0, 0.0, mass * g], np.cross(w_body, Ib @ w_body)])
    return M, C


def test_free_body_known_answer():
    m = kin.KinModel(free_body())
    rng = np.random.default_rng(3)
    for _ in range(3):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        v, w = rng.normal(size=3), rng.normal(size=3)
        qpos = np.concatenate([rng.normal(size=3), q])
        M, C, J, b = kin.kinematics(m, qpos, np.concatenate([v, w]))
        Mk, Ck = free_body_known_answer(q, v, w)
        np.testing.assert_allclose(M, Mk, atol=1e-14)
        np.testing.assert_allclose(C, Ck, atol=1e-13)
        R = kin.quat2mat(q)
        np.testing.assert_allclose(J[:3], np.hstack([np.eye(3), np.zeros((3, 3))]), atol=1e-15)
        np.testing.assert_allclose(J[3:], np.hstack([np.zeros((3, 3)), R]), atol=1e-15)
        np.testing.assert_allclose(b, 0.0, atol=1e-14)   # origin = COM: no bias acceleration


def test_slide_known_answer():
    """A mass on a slide along the unit axis a: x = x0 + a q, M = m + armature, qfrc_bias =
    -m g.a, Jp = a, Jr = 0, no bias acceleration."""
    t = slider()
    m = kin.KinModel(t)
    a = np.asarray(t["bodies"][0]["axis"]) / np.linalg.norm(t["bodies"][0]["axis"])
    for q, qd in ((0.2, -1.0), (-0.4, 2.5)):
        M, C, J, b = kin.kinematics(m, np.array([q]), np.array([qd]))
        np.testing.assert_allclose(kin.site_positions(m, [q])[0], np.array([0.1, 0.2, 0.3]) + a * q,
                                   atol=1e-15)
        np.testing.assert_allclose(M[0, 0], 1.3 + 0.02, rtol=1e-14)
        np.testing.assert_allclose(C[0], 1.3 * 9.81 * a[2], rtol=1e-14)
        np.testing.assert_allclose(J[:3, 0], a, atol=1e-15)
        np.testing.assert_allclose(J[3:, 0], 0.0, atol=0)
        np.testing.assert_allclose(b, 0.0, atol=1e-15)


def spherical_known_answer(quat, wb, mass=0.8, length=0.5, i_small=1e-4, g=9.81):
    """Ball joint at the origin, point-like mass at l = (0, 0, -L) in the body frame; dofs = the
    body-frame angular velocity.  M = I_O (inertia about the anchor, body frame); qfrc_bias =
    w x I_O w - l x (R' m g); Jp = -R [l]x, Jr = R; tip acceleration w x (w x p)."""
    R = kin.quat2mat(quat)
    lv = np.array([0.0, 0.0, -length])
    IO = np.diag([mass * length ** 2 + i_small, mass * length ** 2 + i_small, i_small])
    gv = np.array([0.0, 0.0, -g])
    C = np.cross(wb, IO @ wb) - np.cross(lv, R.T @ (mass * gv))
    lx = np.array([[0, -lv[2], lv[1]], [lv[2], 0, -lv[0]], [-lv[1], lv[0], 0]])
    Jp = -R @ lx
    w = R @ wb
    p = R @ lv
    return IO, C, Jp, R, np.cross(w, np.cross(w, p))


def test_ball_known_answer():
    m = kin.KinModel(spherical_pendulum())
    rng = np.random.default_rng(21)
    for _ in range(3):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        wb = rng.normal(size=3)
        M, C, J, b = kin.kinematics(m, q, wb)
        Mk, Ck, Jp, Jr, bp = spherical_known_answer(q, wb)
        np.testing.assert_allclose(M, Mk, atol=1e-15)
        np.testing.assert_allclose(C, Ck, atol=1e-14)
        np.testing.assert_allclose(J[:3], Jp, atol=1e-15)
        np.testing.assert_allclose(J[3:], Jr, atol=1e-15)
        np.testing.assert_allclose(b[:3], bp, atol=1e-14)
        np.testing.assert_allclose(b[3:], 0.0, atol=1e-15)


def two_joint_known_answer(t1, t2, d1, d2, mass=1.1, length=0.6, i_small=1e-4, arm=(0.01, 0.03),
                           g=9.81):
    """Hinge about x (t1) then about the rotated y (t2) on ONE body, point mass at -L z:
    p = (-L s2, L c2 s1, -L c2 c1), M = diag(m L^2 c2^2 + i + a1, m L^2 + i + a2),
    qfrc_bias = m g L (c2 s1, s2 c1) + m L^2 c2 s2 (-2 d1 d2, d1^2)."""
    L = length
    s1, c1, s2, c2 = np.sin(t1), np.cos(t1), np.sin(t2), np.cos(t2)
    M = np.diag([mass * L * L * c2 * c2 + i_small + arm[0], mass * L * L + i_small + arm[1]])
    C = mass * g * L * np.array([c2 * s1, s2 * c1]) + \
        mass * L * L * c2 * s2 * np.array([-2 * d1 * d2, d1 * d1])
    Jp = np.array([[0.0, -L * c2], [L * c2 * c1, -L * s2 * s1], [L * c2 * s1, L * s2 * c1]])
    Jr = np.array([[1.0, 0.0], [0.0, c1], [0.0, s1]])
    ss = d1 * d1 + d2 * d2
    bp = np.array([L * s2 * d2 * d2, -L * (c2 * s1 * ss + 2 * s2 * c1 * d1 * d2),
                   L * (c2 * c1 * ss - 2 * s2 * s1 * d1 * d2)])
    br = d1 * d2 * np.array([0.0, -s1, c1])
    return M, C, Jp, Jr, bp, br


def test_two_joint_body_known_answer():
    m = kin.KinModel(two_joint_body())
    assert (m.nq, m.nv, m.njnt) == (2, 2, 2)
    for t1, t2, d1, d2 in ((0.3, -0.5, 1.1, -0.7), (1.2, 0.9, -2.0, 0.4), (-2.2, 2.8, 0.3, 1.9)):
        M, C, J, b = kin.kinematics(m, np.array([t1, t2]), np.array([d1, d2]))
        Mk, Ck, Jp, Jr, bp, br = two_joint_known_answer(t1, t2, d1, d2)
        np.testing.assert_allclose(M, Mk, atol=1e-15)
        np.testing.assert_allclose(C, Ck, atol=1e-13)
        np.testing.assert_allclose(J[:3], Jp, atol=1e-15)
        np.testing.assert_allclose(J[3:], Jr, atol=1e-15)
        np.testing.assert_allclose(b[:3], bp, atol=1e-14)
        np.testing.assert_allclose(b[3:], br, atol=1e-15)
