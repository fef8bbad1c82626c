"""GPU parity of the kinematics front end (osc_batch_kinematics, osc_state_to_qpos,
osc_batch_solve_qpos; include/osc_kinematics.h) against the CPU kinematics oracle
(oracle/kinematics.py: COM-Jacobian / Kane formulation, pinned by finite-difference and energy
identities in test_kinematics_oracle.py; parity against MuJoCo itself is unpinned -- no MuJoCo,
no robot XMLs offline).

Tolerance (fp64, two different formulations of the same quantities): per environment and per
output, max |gpu - oracle| <= 1e-12 * (1 + max |oracle|).  M must be exactly symmetric."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import kinematics as kin
from kin_trees import (chain_tree, free_body, mixed_tree, multi_joint_tree, pendulum, random_tree,
                       slider, spherical_pendulum, two_joint_body)
from osc_amd.kinematics import KinematicsBatch, load_tree, random_states

pytestmark = pytest.mark.gpu
TOL = 1e-12


def _mjcf_tree(robot):
    """config/<robot>.xml through the MJCF reader with the robot's site convention: Go2 in
    model order (its task sites' points and Jacobian bodies differ, G/osc.h:373), WaLTER by
    name (W/osc.h:417)."""
    import os
    from osc_amd.mjcf import load_mjcf_robot
    from osc_amd.kinematics import kin_json_path
    return load_mjcf_robot(robot, os.path.join(os.path.dirname(kin_json_path(robot)), f"{robot}.xml"))


def _split(tree):
    """A tree with MuJoCo joint lists through the MJCF reader: one joint per body (chains)."""
    import os
    import tempfile
    from osc_amd.mjcf import load_mjcf, tree_to_mjcf
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "m.xml")
        with open(path, "w") as fh:
            fh.write(tree_to_mjcf(tree))
        bn = [tree["bodies"][s["body"]].get("name", f"b{s['body']}") for s in tree["sites"]]
        sn = [s.get("name", f"s{k}") for k, s in enumerate(tree["sites"])]
        return load_mjcf(path, bn, sn)


def _dfs(tree):
    from test_mjcf import _dfs as dfs
    return dfs(tree)


def _trees():
    return {"unitree_go2": load_tree("unitree_go2"), "walter_sr": load_tree("walter_sr"),
            "random_free": random_tree(5), "random_fixed": random_tree(6, free_root=False),
            "chain16": chain_tree(7), "unitree_go2_mjcf": _mjcf_tree("unitree_go2"),
            "walter_sr_mjcf": _mjcf_tree("walter_sr"),
            "slide_ball_free": mixed_tree(2), "slide_ball_fixed": mixed_tree(3, free_root=False)}


TREES = _trees()


def _check(tree, nenv, seed, base_pos_zero=True, oracle_tree=None):
    """Kernel on `tree` against the oracle on `oracle_tree` (default: the same tree; a tree with
    joint lists for a split descriptor)."""
    kb = KinematicsBatch(tree=tree)
    qpos, qvel = random_states(tree, nenv, seed, base_pos_zero=base_pos_zero)
    out = kb.compute(qpos, qvel)
    torch.cuda.synchronize()
    M, C, J, b, X = (t.cpu().numpy() for t in (out.M, out.C, out.J, out.b, out.site_xpos))
    m = kin.KinModel(oracle_tree or tree)
    for e in range(nenv):
        Mr, Cr, Jr, br = kin.kinematics(m, qpos[e], qvel[e])
        Xr = kin.site_positions(m, qpos[e])
        for name, got, ref in (("M", M[e], Mr), ("C", C[e], Cr), ("J", J[e], Jr), ("b", b[e], br),
                               ("site_xpos", X[e], Xr)):
            err = np.abs(got - ref).max()
            assert err <= TOL * (1 + np.abs(ref).max()), (name, e, err)
        assert np.array_equal(M[e], M[e].T)
    return kb


@pytest.mark.parametrize("name", list(TREES))
def test_kinematics_matches_oracle(gpu, name):
    # 37 envs: 9 full wavefronts + a ragged tail row
    _check(TREES[name], 37, 100 + len(name), base_pos_zero=(name != "random_free"))


def test_single_env_and_empty_batch(gpu):
    kb = _check(TREES["unitree_go2"], 1, 3)
    out = kb.alloc(0)
    empty = torch.empty((0, kb.nq), dtype=torch.float64, device=gpu)
    kb.compute_into(out, empty, torch.empty((0, kb.nv), dtype=torch.float64, device=gpu))


def test_large_batch_properties(gpu):
    """65,536 Go2 envs: M symmetric positive definite, J structure = the tree's (feet rows touch
    base + own leg only), gravity-only bias at zero velocity equals the total weight on base z,
    and a sample of environments matches the oracle."""
    tree = TREES["unitree_go2"]
    kb = KinematicsBatch(tree=tree)
    nenv = 65536
    qpos, qvel = random_states(tree, nenv, 77)
    out = kb.compute(qpos, qvel, want_sites=False)
    M = out.M
    assert torch.equal(M, M.transpose(1, 2))
    assert torch.linalg.eigvalsh(M).min().item() > 0
    J = out.J.cpu().numpy()
    m = kin.KinModel(tree)
    for k, s in enumerate(m.sites):
        chain = set()
        for c in m.chain(s["body"]):
            nd = {"free": 6, "hinge": 1}.get(m.bodies[c]["joint"], 0)
            chain |= set(range(m.dadr[c], m.dadr[c] + nd))
        off = [d for d in range(m.nv) if d not in chain]
        assert np.all(J[:, 3 * k:3 * k + 3, off] == 0.0)
        assert np.all(J[:, 3 * m.ns + 3 * k:3 * m.ns + 3 * k + 3, off] == 0.0)
    g = kb.compute(qpos[:64], np.zeros((64, kb.nv))).C.cpu().numpy()
    total = sum(b["mass"] for b in tree["bodies"])
    np.testing.assert_allclose(g[:, 2], total * 9.81, rtol=1e-13)
    for e in (0, 12345, nenv - 1):
        Mr, Cr, Jr, br = kin.kinematics(m, qpos[e], qvel[e])
        assert np.abs(M[e].cpu().numpy() - Mr).max() <= TOL * (1 + np.abs(Mr).max())
        assert np.abs(out.b[e].cpu().numpy() - br).max() <= TOL * (1 + np.abs(br).max())


def test_state_to_qpos_packing(gpu):
    """update_mj_data (osc.h:357-361): qpos = [0,0,0, quat, q_m], qvel = [v, w, qd_m]."""
    kb = KinematicsBatch("unitree_go2")
    rng = np.random.default_rng(4)
    n, nu = 33, 12
    rot = rng.standard_normal((n, 4))
    lin, ang = rng.standard_normal((n, 3)), rng.standard_normal((n, 3))
    qm, qdm = rng.standard_normal((n, nu)), rng.standard_normal((n, nu))
    qpos, qvel = kb.state_to_qpos(rot, lin, ang, qm, qdm)
    np.testing.assert_array_equal(qpos.cpu().numpy(), np.hstack([np.zeros((n, 3)), rot, qm]))
    np.testing.assert_array_equal(qvel.cpu().numpy(), np.hstack([lin, ang, qdm]))


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_solve_from_joint_states(gpu, robot):
    """osc_batch_solve_qpos == osc_batch_kinematics + osc_batch_solve (bitwise), and its torques
    match the oracle chain (oracle kinematics -> reference QP -> exact optimum) within the solve's
    parity tolerance (test_gpu_parity.py)."""
    from osc_amd.solver import OSCBatchSolver
    from osc_amd.synth import SEED_BASE
    from osc_qp import build_qp, load_model, torque
    from qp_exact import solve_exact
    tree = load_tree(robot)
    kb = KinematicsBatch(tree=tree)
    solver = OSCBatchSolver(robot)
    nenv = 24
    qpos, qvel = random_states(tree, nenv, SEED_BASE + 9, joint_range=0.5)
    rng = np.random.default_rng(9)
    ns, nc = solver.dims["ns"], solver.dims["nc"]
    T = np.zeros((nenv, ns, 6))
    T[:, 0, :] = 10.0 * rng.standard_normal((nenv, 6))
    mask = (rng.uniform(size=(nenv, nc)) < 0.75).astype(np.float64)
    res = kb.solve(solver, qpos, qvel, T, mask, want_x=True)
    k = kb.compute(qpos, qvel, want_sites=False)
    ref = solver.solve(k.M, k.C, k.J, k.b, T, mask, want_x=True)
    torch.cuda.synchronize()
    assert torch.equal(res.tau, ref.tau) and torch.equal(res.x, ref.x)
    assert (res.status.cpu().numpy() == 0).all(), res.status
    model = load_model(robot)
    m = kin.KinModel(tree)
    tau = res.tau.cpu().numpy()
    for e in range(nenv):
        M, C, J, b = kin.kinematics(m, qpos[e], qvel[e])
        args = (M, C, J, b, T[e], mask[e])
        tr = torque(model, solve_exact(model, build_qp(model, *args), M, C, J).x)
        assert np.abs(tau[e] - tr).max() / max(np.abs(tr).max(), 1.0) <= 1e-5, e


def test_warm_solve_from_joint_states(gpu):
    """osc_batch_solve_qpos_warm == osc_batch_kinematics + osc_batch_solve_warm, bitwise, over
    three ticks of a small joint-space walk (warm state carried)."""
    from osc_amd.solver import OSCBatchSolver
    tree = load_tree("unitree_go2")
    kb = KinematicsBatch(tree=tree)
    solver = OSCBatchSolver("unitree_go2")
    nenv = 16
    qpos, qvel = random_states(tree, nenv, 5, joint_range=0.5)
    rng = np.random.default_rng(5)
    T = np.zeros((nenv, 5, 6))
    T[:, 0] = 10.0 * rng.standard_normal((nenv, 6))
    mask = np.ones((nenv, 4))
    wa, wb = solver.alloc_warm_state(nenv), solver.alloc_warm_state(nenv)
    oa, ob = solver.alloc_outputs(nenv), solver.alloc_outputs(nenv)
    ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64, device=gpu)
    Td, md = torch.from_numpy(T).to(gpu), torch.from_numpy(mask).to(gpu)
    for k in range(3):
        qp = torch.from_numpy(qpos + 0.01 * k).to(gpu)
        qv = torch.from_numpy(qvel).to(gpu)
        kb.solve_warm_into(solver, oa, wa, qp, qv, Td, md, ws)
        kk = kb.compute(qp, qv, want_sites=False)
        solver.solve_warm_into(ob, wb, kk.M, kk.C, kk.J, kk.b, Td, md)
        torch.cuda.synchronize()
        assert torch.equal(oa.tau, ob.tau) and torch.equal(wa, wb)
        assert (oa.status.cpu().numpy() == 0).all()


def test_known_answer_trees(gpu):
    """The kernel against closed forms (tests/test_kinematics_oracle.py): a pendulum (M = m L^2 +
    I + armature, qfrc_bias = m g L sin th, Jp, Jdot qdot) and a free body with body-frame
    rotational dofs (M = blockdiag(m I, I_body), qfrc_bias = (m g e_z, w x I w))."""
    from test_kinematics_oracle import free_body_known_answer, pendulum_known_answer
    kb = KinematicsBatch(tree=pendulum())
    th = np.array([0.3, -1.1, 2.5])
    thd = np.array([1.2, -0.4, 3.0])
    out = kb.compute(th[:, None], thd[:, None])
    torch.cuda.synchronize()
    for e in range(3):
        Mk, Ck, Jp, bp = pendulum_known_answer(th[e], thd[e])
        assert abs(out.M[e, 0, 0].item() - Mk) <= 1e-14 * Mk
        assert abs(out.C[e, 0].item() - Ck) <= 1e-13
        np.testing.assert_allclose(out.J[e, :3, 0].cpu().numpy(), Jp, atol=1e-15)
        np.testing.assert_allclose(out.b[e, :3].cpu().numpy(), bp, atol=1e-13)
    kb = KinematicsBatch(tree=free_body())
    rng = np.random.default_rng(3)
    q = rng.normal(size=(5, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    qpos = np.hstack([rng.normal(size=(5, 3)), q])
    qvel = rng.normal(size=(5, 6))
    out = kb.compute(qpos, qvel)
    torch.cuda.synchronize()
    for e in range(5):
        Mk, Ck = free_body_known_answer(q[e], qvel[e, :3], qvel[e, 3:])
        np.testing.assert_allclose(out.M[e].cpu().numpy(), Mk, atol=1e-14)
        np.testing.assert_allclose(out.C[e].cpu().numpy(), Ck, atol=1e-13)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_multi_joint_bodies_match_oracle(gpu, seed):
    """Bodies with MuJoCo joint lists (hinge / slide pairs and triples, hinge-then-ball): the
    MJCF reader's chain descriptor on the GPU against the oracle restating the lists directly."""
    tree = _dfs(multi_joint_tree(seed))
    _check(_split(tree), 37, 300 + seed, oracle_tree=tree)


def test_known_answer_slide_ball_two_joint(gpu):
    """The kernel against closed forms (tests/test_kinematics_oracle.py): a slider (M = m +
    armature, qfrc_bias = -m g.a, Jp = a), a spherical pendulum (ball: M = I_O, qfrc_bias =
    w x I_O w - l x R'm g, Jp = -R[l]x, Jr = R) and a two-hinge body split by the MJCF reader."""
    from test_kinematics_oracle import spherical_known_answer, two_joint_known_answer
    t = slider()
    a = np.asarray(t["bodies"][0]["axis"]) / np.linalg.norm(t["bodies"][0]["axis"])
    kb = KinematicsBatch(tree=t)
    q = np.array([[0.2], [-0.4]])
    out = kb.compute(q, np.array([[-1.0], [2.5]]))
    torch.cuda.synchronize()
    for e in range(2):
        assert abs(out.M[e, 0, 0].item() - 1.32) <= 1e-14
        assert abs(out.C[e, 0].item() - 1.3 * 9.81 * a[2]) <= 1e-13
        np.testing.assert_allclose(out.J[e, :3, 0].cpu().numpy(), a, atol=1e-15)
        np.testing.assert_allclose(out.J[e, 3:, 0].cpu().numpy(), 0.0, atol=0)
        np.testing.assert_allclose(out.b[e].cpu().numpy(), 0.0, atol=1e-15)
        np.testing.assert_allclose(out.site_xpos[e, 0].cpu().numpy(),
                                   np.array([0.1, 0.2, 0.3]) + a * q[e, 0], atol=1e-15)
    kb = KinematicsBatch(tree=spherical_pendulum())
    rng = np.random.default_rng(21)
    qq = rng.normal(size=(5, 4))
    qq /= np.linalg.norm(qq, axis=1, keepdims=True)
    wb = rng.normal(size=(5, 3))
    out = kb.compute(qq, wb)
    torch.cuda.synchronize()
    for e in range(5):
        Mk, Ck, Jp, Jr, bp = spherical_known_answer(qq[e], wb[e])
        np.testing.assert_allclose(out.M[e].cpu().numpy(), Mk, atol=1e-15)
        np.testing.assert_allclose(out.C[e].cpu().numpy(), Ck, atol=1e-14)
        np.testing.assert_allclose(out.J[e, :3].cpu().numpy(), Jp, atol=1e-15)
        np.testing.assert_allclose(out.J[e, 3:].cpu().numpy(), Jr, atol=1e-15)
        np.testing.assert_allclose(out.b[e, :3].cpu().numpy(), bp, atol=1e-14)
    kb = KinematicsBatch(tree=_split(two_joint_body()))
    th = np.array([[0.3, -0.5], [1.2, 0.9], [-2.2, 2.8]])
    thd = np.array([[1.1, -0.7], [-2.0, 0.4], [0.3, 1.9]])
    out = kb.compute(th, thd)
    torch.cuda.synchronize()
    for e in range(3):
        Mk, Ck, Jp, Jr, bp, br = two_joint_known_answer(*th[e], *thd[e])
        np.testing.assert_allclose(out.M[e].cpu().numpy(), Mk, atol=1e-15)
        np.testing.assert_allclose(out.C[e].cpu().numpy(), Ck, atol=1e-13)
        np.testing.assert_allclose(out.J[e, :3].cpu().numpy(), Jp, atol=1e-15)
        np.testing.assert_allclose(out.J[e, 3:].cpu().numpy(), Jr, atol=1e-15)
        np.testing.assert_allclose(out.b[e, :3].cpu().numpy(), bp, atol=1e-14)
        np.testing.assert_allclose(out.b[e, 3:].cpu().numpy(), br, atol=1e-15)
