"""The host-fed batched tick (include/osc_host_feed.h): inputs in pinned host
memory every tick, one H2D copy, the solve, D2H of the torques, pipelined over `depth` slots.
Every tick's results must be BITWISE those of the device-resident solve of the same inputs
(osc_batch_solve / _warm / _qpos): the feed moves bytes, it changes no arithmetic."""
import ctypes

import numpy as np
import pytest
import torch

from osc_amd import _lib
from osc_amd.synth import SEED_BASE, generate

pytestmark = pytest.mark.gpu


def _batches(robot, nenv, n, seed):
    return [generate(robot, nenv, SEED_BASE + seed + k, "standing", "ones") for k in range(n)]


def _fill(feed, k, d):
    v = feed.inputs(k)
    for key in ("M", "C", "J", "b", "T", "mask"):
        v[key][...] = d[key]


@pytest.mark.parametrize("robot,depth", [("unitree_go2", 2), ("walter_sr", 2), ("unitree_go2", 1),
                                         ("unitree_go2", 3)])
def test_qp_form_bitwise_device_resident(gpu, robot, depth):
    from osc_amd.host_feed import HostFeed
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver(robot)
    nenv, nt = 1000, 6
    data = _batches(robot, nenv, nt, 301)
    feed = HostFeed(s, nenv, "qp", depth=depth)
    got = {}
    for k in range(nt + depth - 1):
        if k < nt:
            _fill(feed, k, data[k])
            feed.submit(k)
        j = k - depth + 1
        if j >= 0:
            got[j] = tuple(a.copy() for a in feed.wait(j))
    for k in range(nt):
        r = s.solve(**data[k])
        torch.cuda.synchronize()
        assert np.array_equal(got[k][0], r.tau.cpu().numpy()), k
        assert np.array_equal(got[k][1], r.status.cpu().numpy()), k
        assert np.array_equal(got[k][2], r.iters.cpu().numpy()), k
        assert (got[k][1] == 0).all()
    t = feed.timing(nt - 1)
    assert t["h2d_ms"] > 0 and t["solve_ms"] > 0 and t["latency_ms"] >= t["solve_ms"]
    feed.close()


def test_qp_form_warm_bitwise_device_warm(gpu):
    """Warm-started feed: the warm state carried tick to tick on the device equals
    osc_batch_solve_warm called tick after tick on the same inputs."""
    from osc_amd.host_feed import HostFeed
    from osc_amd.solver import OSCBatchSolver
    from osc_amd.synth import random_walk
    s = OSCBatchSolver("unitree_go2")
    nenv, nt = 777, 6
    d0 = generate("unitree_go2", nenv, SEED_BASE + 311, "standing", "ones")
    data = [d0]
    rng = np.random.default_rng(SEED_BASE + 312)
    for k in range(1, nt):
        data.append(random_walk(data[-1], rng))
    feed = HostFeed(s, nenv, "qp", depth=2, warm=True)
    got = {}
    for k in range(nt + 1):
        if k < nt:
            _fill(feed, k, data[k])
            feed.submit(k)
        if k >= 1:
            got[k - 1] = tuple(a.copy() for a in feed.wait(k - 1))
    warm = s.alloc_warm_state(nenv)
    out = s.alloc_outputs(nenv)
    for k in range(nt):
        s.solve_warm_into(out, warm, *s.prepare(**data[k]))
        torch.cuda.synchronize()
        assert np.array_equal(got[k][0], out.tau.cpu().numpy()), k
        assert np.array_equal(got[k][2], out.iters.cpu().numpy()), k
    assert got[nt - 1][2].mean() < got[0][2].mean()   # warm ticks take fewer iterations


@pytest.mark.parametrize("warm", [False, True])
def test_joint_state_form_bitwise(gpu, warm):
    from osc_amd.host_feed import HostFeed
    from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver("unitree_go2")
    tree = load_tree("unitree_go2")
    kb = KinematicsBatch(tree=tree)
    nenv, nt = 900, 5
    q0, v0 = random_states(tree, nenv, SEED_BASE + 321, joint_range=0.5)
    d = generate("unitree_go2", nenv, SEED_BASE + 322, "standing", "ones")
    rng = np.random.default_rng(5)
    states = []
    for k in range(nt):
        q = q0.copy()
        q[:, 7:] += 0.01 * k * rng.standard_normal(q[:, 7:].shape)
        states.append((q, v0 * (1 + 0.01 * k)))
    feed = HostFeed(s, nenv, "joint_states", depth=2, warm=warm, kin=kb)
    got = {}
    for k in range(nt + 1):
        if k < nt:
            v = feed.inputs(k)
            v["qpos"][...], v["qvel"][...] = states[k]
            v["T"][...], v["mask"][...] = d["T"], d["mask"]
            feed.submit(k)
        if k >= 1:
            got[k - 1] = tuple(a.copy() for a in feed.wait(k - 1))
    out = s.alloc_outputs(nenv)
    ws = torch.empty((kb.workspace_bytes(s, nenv) // 8 + 2,), dtype=torch.float64, device="cuda")
    wst = s.alloc_warm_state(nenv)
    T, mask = torch.from_numpy(d["T"]).cuda(), torch.from_numpy(d["mask"]).cuda()
    for k in range(nt):
        q, v = (torch.from_numpy(a).cuda() for a in states[k])
        if warm:
            kb.solve_warm_into(s, out, wst, q, v, T, mask, ws)
        else:
            kb.solve_into(s, out, q, v, T, mask, ws)
        torch.cuda.synchronize()
        assert np.array_equal(got[k][0], out.tau.cpu().numpy()), k
        assert np.array_equal(got[k][1], out.status.cpu().numpy()), k
        assert (got[k][1] == 0).all()


def test_feed_argument_errors(gpu):
    from osc_amd.host_feed import HostFeed
    from osc_amd.kinematics import KinematicsBatch
    from osc_amd.solver import OSCBatchSolver
    L = _lib.lib()
    s = OSCBatchSolver("unitree_go2")
    h = ctypes.c_void_p()
    assert L.osc_host_feed_create(s._h, None, 16, 0, 0, 0, ctypes.byref(h)) == 1      # depth 0
    assert L.osc_host_feed_create(s._h, None, 16, 0, 0, 9, ctypes.byref(h)) == 1      # > max
    assert L.osc_host_feed_create(s._h, None, 16, 1, 0, 2, ctypes.byref(h)) == 1      # no kin
    assert L.osc_host_feed_create(s._h, None, 16, 0, 4, 2, ctypes.byref(h)) == 1      # flags
    kw = KinematicsBatch("walter_sr")
    assert L.osc_host_feed_create(s._h, kw._h, 16, 1, 0, 2, ctypes.byref(h)) == 1     # other robot
    noslip = OSCBatchSolver("walter_sr_wheels", _noslip_yaml())
    assert L.osc_host_feed_create(noslip._h, None, 16, 0, 0, 2, ctypes.byref(h)) == 1
    feed = HostFeed(s, 16, "qp", depth=2)
    with pytest.raises(_lib.OSCError):
        feed.submit(1)                      # out of order
    feed.inputs(0)
    feed.submit(0)
    with pytest.raises(_lib.OSCError):
        feed.wait(1)                        # not submitted
    feed.wait(0)                            # all-zero inputs: a defined QP (M = 0 -> NUMERICAL)
    for k in (1, 2, 3):
        feed.inputs(k)
        feed.submit(k)
    with pytest.raises(_lib.OSCError):
        feed.wait(1)                        # older than depth
    feed.wait(3)


def _noslip_yaml():
    import os
    from osc_amd.robots import config_path
    return os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                        "walter_sr_wheels_noslip_config.yaml")


@pytest.mark.parametrize("nenv", [1, 3])
def test_tiny_batches(gpu, nenv):
    """A single env (the reference's own case, configs[0]) and a partial wavefront."""
    from osc_amd.host_feed import HostFeed
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver("unitree_go2")
    data = _batches("unitree_go2", nenv, 3, 331)
    feed = HostFeed(s, nenv, "qp", depth=2)
    got = {}
    for k in range(4):
        if k < 3:
            _fill(feed, k, data[k])
            feed.submit(k)
        if k >= 1:
            got[k - 1] = feed.wait(k - 1)[0].copy()
    for k in range(3):
        r = s.solve(**data[k])
        torch.cuda.synchronize()
        assert np.array_equal(got[k], r.tau.cpu().numpy()), k
