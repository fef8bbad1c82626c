"""GPU parity on kinematics-generated QPs: joint states -> GPU kinematics -> reduced QP -> interior
point -> full-space refinement (osc_batch_solve_qpos), at BASELINE sizes.

Why this file exists: on joint-state batches the QP has nearly active rows along
the internal-force directions, whose curvature is only 2 w_reg = 2e-4, so the interior point's
iterate at mu = 1e-9 sits up to ~2e-2 off the optimum there, and the refinement (method of
multipliers on the active set, residual in factored form: DESIGN.md §3) has to move it that far.
Round 3's per-lane move bound rejected those refinements: 26 of 4,096 Go2 envs of this seed ended
OSC_SOLVE_UNREFINED (2e-4 .. 1.6e-2 normwise off).  The synthetic batches of test_gpu_parity.py
never produce such envs.

Checks (stated tolerances):
  * every env of every batch status OK (no UNREFINED, no MAX_ITER);
  * osc_batch_solve_qpos == osc_batch_kinematics + osc_batch_solve (bitwise);
  * the OSQP-form KKT certificate of (x, y) on EVERY env (test_gpu_wheels._kkt: stationarity
    1e-6, primal 1e-9, dual sign 1e-9, complementarity 1e-7, scaled as
    oracle/qp_exact.kkt_certificate);
  * EVERY env against the exact optimum of the reference QP on the same M, C, J, b
    (oracle/parallel.py: the full oracle over a host process pool at 4,096 envs; at 65,536 the
    oracle's exact KKT solve on the working set the GPU's duals mark active, certified, the full
    oracle wherever that set does not certify): normwise <= 1e-9, elementwise <= 1e-7 -- the bars
    of test_gpu_parity.py -- with the worst env printed; and the oracle chain from the oracle's
    own kinematics within the 1e-5 contract;
  * ten consecutive 4,096-env ticks (cold and warm-started) with every status OK.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import kinematics as kin
from osc_amd.dist import shard_seed
from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
from osc_amd.synth import generate
from osc_qp import build_qp, load_model, torque
from parallel import seeded_batch, solve_batch
from qp_exact import solve_exact
from test_gpu_wheels import _batched_qp, _certify, _kkt, _rel_errors

pytestmark = pytest.mark.gpu

NORM_ACH, ELEM_ACH, CONTRACT = 1e-9, 1e-7, 1e-5
SEED = shard_seed(0) + 7
# (round 3's UNREFINED envs of the Go2 0.5 batch -- 0, 42, 124, 158, 286, 610, 669, 893, 902, 1046,
# 2064, 2103, 2125, profiles/r03zr_qpos_refine_diag_widened.jsonl -- are among every env checked.)

_cache = {}


def _setup(robot):
    from osc_amd.solver import OSCBatchSolver
    if robot not in _cache:
        tree = load_tree(robot)
        _cache[robot] = (tree, KinematicsBatch(tree=tree), OSCBatchSolver(robot))
    return _cache[robot]


def _batch(robot, nenv, jr, mask_mode, seed=SEED):
    tree, kb, solver = _setup(robot)
    qpos, qvel = random_states(tree, nenv, seed, joint_range=jr)
    d = generate(robot, nenv, seed, "standing" if mask_mode == "ones" else "tumbling", mask_mode)
    return qpos, qvel, d["T"], d["mask"]


@pytest.mark.parametrize("robot,nenv,jr,mask_mode", [
    ("unitree_go2", 4096, 0.5, "ones"),       # round 3's failing batch
    ("unitree_go2", 4096, 1.0, "bernoulli"),
    ("unitree_go2", 65536, 0.5, "ones"),      # the north-star batch size
    ("walter_sr", 4096, 0.5, "ones"),
    ("walter_sr", 4096, 1.0, "bernoulli"),
    ("walter_sr", 65536, 1.0, "ones"),
])
def test_joint_state_batch(gpu, robot, nenv, jr, mask_mode):
    tree, kb, solver = _setup(robot)
    qpos, qvel, T, mask = _batch(robot, nenv, jr, mask_mode)
    res = kb.solve(solver, qpos, qvel, T, mask, want_x=True)          # osc_batch_solve_qpos
    k = kb.compute(qpos, qvel, want_sites=False)
    args = solver.prepare(k.M, k.C, k.J, k.b, T, mask)
    out = solver.alloc_outputs(nenv, want_y=True)
    solver.solve_into(out, *args)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    assert (st == 0).all(), (np.bincount(st), np.nonzero(st)[0][:20])
    assert torch.equal(res.tau, out.tau) and torch.equal(res.x, out.x)
    _certify(_kkt(*_batched_qp(robot, *args), out.x, out.y), robot)

    model = load_model(robot)
    envs = np.arange(nenv)
    tau = res.tau.cpu().numpy()
    M, C, J, b = (t.cpu().numpy() for t in (k.M, k.C, k.J, k.b))
    if nenv <= 8192:   # every env, the full oracle over a host process pool
        xo, _ = solve_batch(robot, M, C, J, b, T, mask)
    else:              # every env, the oracle seeded by the GPU's active set and certified
        xo, _ = seeded_batch(robot, M, C, J, b, T, mask, out.y.cpu().numpy())
    ref = xo[:, model.nv:model.nv + model.nu]
    nw, el = _rel_errors(tau[envs], ref)
    worst = int(envs[np.argmax(nw)])
    print(f"\n{robot} joint states {nenv} envs (range {jr}, mask {mask_mode}): every env vs "
          f"the exact optimum, worst normwise {nw.max():.2e} (env {worst}), worst elementwise "
          f"{el.max():.2e}")
    assert nw.max() <= NORM_ACH and el.max() <= ELEM_ACH, (nw.max(), el.max(), worst)
    chain = []
    m = kin.KinModel(tree)
    for e in envs[:16]:   # the oracle chain from the oracle's own kinematics
        Mo, Co, Jo, bo = kin.kinematics(m, qpos[e], qvel[e])
        ao = (Mo, Co, Jo, bo, T[e], mask[e])
        chain.append(torque(model, solve_exact(model, build_qp(model, *ao), Mo, Co, Jo).x))
    nwc, _ = _rel_errors(tau[envs[:16]], np.array(chain))
    assert nwc.max() <= CONTRACT, nwc.max()


@pytest.mark.parametrize("seed", [11, 13, 14])
def test_joint_state_census_every_env_refined(gpu, seed):
    """Round 5's status census batches (tools/status_diag.py): 65,536 Go2 envs from joint states
    (joint_range 1.0), where 1 / 4 / 7 envs came back OSC_SOLVE_UNREFINED before the refinement's
    one-change rounds (their inputs and exact optima: tests/golden/go2_unrefined_joint_states.npz)
    -- every env OK now, and those envs' torques at the exact optimum."""
    robot, nenv = "unitree_go2", 65536
    tree, kb, solver = _setup(robot)
    qpos, qvel = random_states(tree, nenv, seed, joint_range=1.0)
    d = generate(robot, nenv, seed, "standing", "ones")
    k = kb.compute(qpos, qvel, want_sites=False)
    args = solver.prepare(k.M, k.C, k.J, k.b, d["T"], d["mask"])
    out = solver.alloc_outputs(nenv)
    solver.solve_into(out, *args)
    torch.cuda.synchronize()
    st = out.status.cpu().numpy()
    assert (st == 0).all(), (np.bincount(st), np.nonzero(st)[0][:20])
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "go2_unrefined_joint_states.npz"))
    sel = g["seed"] == seed
    envs = g["envs"][sel]
    np.testing.assert_allclose(k.M.cpu().numpy()[envs], g["M"][sel], rtol=0, atol=1e-12)
    nw, el = _rel_errors(out.tau.cpu().numpy()[envs], g["tau"][sel])
    assert nw.max() <= NORM_ACH and el.max() <= ELEM_ACH, (nw.max(), el.max())


@pytest.mark.parametrize("robot,seed,jr,fixture", [
    ("unitree_go2", 22, 0.5, "go2_stalled_joint_states.npz"),
    ("walter_sr", 23, 1.5, "walter_stalled_joint_states.npz"),
])
def test_joint_state_census_stalled_envs_fixed_up(gpu, robot, seed, jr, fixture):
    """Round 5's wider census (48 x 65,536 joint-state envs): an env the adaptive fraction to the
    boundary stalls at max_iter is re-solved cold (eta 0.99, mu <= 1e-12) by the fix-up pass -- in
    the same launch (Go2), or in the third launch after the lockstep compaction's two (WaLTER at
    65,536) -- so every env of these batches comes back OK, at the exact optimum."""
    nenv = 65536
    tree, kb, solver = _setup(robot)
    qpos, qvel = random_states(tree, nenv, seed, joint_range=jr)
    d = generate(robot, nenv, seed, "standing", "ones")
    k = kb.compute(qpos, qvel, want_sites=False)
    args = solver.prepare(k.M, k.C, k.J, k.b, d["T"], d["mask"])
    out = solver.alloc_outputs(nenv)
    solver.solve_into(out, *args)
    torch.cuda.synchronize()
    st = out.status.cpu().numpy()
    assert (st == 0).all(), (np.bincount(st), np.nonzero(st)[0][:20])
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", fixture))
    sel = g["seed"] == seed
    envs = g["envs"][sel]
    np.testing.assert_allclose(k.M.cpu().numpy()[envs], g["M"][sel], rtol=0, atol=1e-12)
    nw, el = _rel_errors(out.tau.cpu().numpy()[envs], g["tau"][sel])
    assert nw.max() <= NORM_ACH and el.max() <= ELEM_ACH, (nw.max(), el.max())


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_joint_state_ticks(gpu, robot):
    """Ten consecutive 4,096-env ticks of a joint-space walk (hinge angles +-0.01 rad, velocities
    +-1 % per tick, base orientation fixed): cold (osc_batch_solve_qpos) and warm-started
    (osc_batch_solve_qpos_warm) ticks report every env OK, and agree to the refinement's accuracy."""
    tree, kb, solver = _setup(robot)
    nenv = 4096
    qpos, qvel, T, mask = _batch(robot, nenv, 0.5, "ones", seed=SEED + 1)
    rng = np.random.default_rng(3)
    hinge = np.zeros(qpos.shape[1], bool)
    hinge[7:] = True   # free base first (7 qpos): every other coordinate a hinge angle
    dev = gpu
    Td, md = torch.from_numpy(T).to(dev), torch.from_numpy(mask).to(dev)
    cold, warm = solver.alloc_outputs(nenv), solver.alloc_outputs(nenv)
    wstate = solver.alloc_warm_state(nenv)
    ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64, device=dev)
    for tick in range(10):
        qp = torch.from_numpy(qpos).to(dev)
        qv = torch.from_numpy(qvel).to(dev)
        kb.solve_into(solver, cold, qp, qv, Td, md, ws)
        torch.cuda.synchronize()
        kb.solve_warm_into(solver, warm, wstate, qp, qv, Td, md, ws)
        torch.cuda.synchronize()
        for name, o in (("cold", cold), ("warm", warm)):
            st = o.status.cpu().numpy()
            assert (st == 0).all(), (tick, name, np.bincount(st), np.nonzero(st)[0][:20])
        nw, _ = _rel_errors(warm.tau.cpu().numpy(), cold.tau.cpu().numpy())
        assert nw.max() <= 1e-8, (tick, nw.max())
        qpos = qpos + np.where(hinge, rng.uniform(-0.01, 0.01, qpos.shape), 0.0)
        qvel = qvel * (1.0 + 0.01 * rng.standard_normal(qvel.shape))
