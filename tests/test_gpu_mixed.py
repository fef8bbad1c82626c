"""BASELINE configs[4] on one GPU: Go2 and WaLTER Sr shards solved together (4,096 + 4,096 envs,
the per-GPU share of the 65,536-env 8-GPU job; SURVEY.md §8(e): one kernel instantiation per
model, no collective).

Both ways bench.py can run them are checked:
  * osc_batch_solve_multi -- one assembly grid + one interior-point grid for both models;
  * two osc_batch_solve calls on two streams (the round-1 bench path).
Each must give every env converged and, per model, torques BITWISE equal to that model's solo
solve (same kernels, same per-env arithmetic), and a subsample of each model's envs must match
the exact oracle within the tolerance of tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from osc_amd.synth import SEED_BASE, generate
from osc_qp import build_qp, load_model, torque
from qp_exact import solve_exact

pytestmark = pytest.mark.gpu

NENV = 4096
NORM_TOL = 1e-9          # achieved bound of tests/test_gpu_parity.py
ROBOTS = ("unitree_go2", "walter_sr")


def _setup():
    from osc_amd.solver import OSCBatchSolver
    jobs, data = [], []
    for i, robot in enumerate(ROBOTS):
        s = OSCBatchSolver(robot)
        d = generate(robot, NENV, SEED_BASE + 4 + 500 * i, "tumbling" if i else "standing",
                     "bernoulli" if i else "ones")
        jobs.append((s, s.alloc_outputs(NENV, want_x=True), s.prepare(**d)))
        data.append(d)
    return jobs, data


def _solo(jobs):
    out = []
    for s, _, inputs in jobs:
        o = s.alloc_outputs(NENV, want_x=True)
        s.solve_into(o, *inputs)
        out.append(o)
    torch.cuda.synchronize()
    return [(o.tau.cpu().numpy(), o.x.cpu().numpy(), o.status.cpu().numpy()) for o in out]


def _check_vs_solo(jobs, solo):
    for (s, out, _), (tau, x, st) in zip(jobs, solo):
        assert (out.status.cpu().numpy() == 0).all(), s.robot
        assert (st == 0).all()
        assert np.array_equal(out.tau.cpu().numpy(), tau), f"{s.robot}: not bitwise the solo solve"
        assert np.array_equal(out.x.cpu().numpy(), x)


def test_mixed_multi_bitwise_solo_and_oracle(gpu):
    from osc_amd.solver import solve_multi_into
    jobs, data = _setup()
    solo = _solo(jobs)
    for _, out, _ in jobs:                       # poison the outputs: the multi call must write
        out.tau.fill_(float("nan"))
        out.status.fill_(-1)
    solve_multi_into(jobs)
    torch.cuda.synchronize()
    _check_vs_solo(jobs, solo)
    # >= 64 envs per model against the exact oracle (spread over the whole batch)
    for (s, out, _), d in zip(jobs, data):
        model = load_model(s.robot)
        tau = out.tau.cpu().numpy()
        worst = 0.0
        for e in np.linspace(0, NENV - 1, 64).astype(int):
            args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
            ref = torque(model, solve_exact(model, build_qp(model, *args), *args[:3]).x)
            worst = max(worst, np.abs(tau[e] - ref).max() / max(np.abs(ref).max(), 1.0))
        assert worst <= NORM_TOL, (s.robot, worst)


def test_mixed_two_streams_bitwise_solo(gpu):
    jobs, _ = _setup()
    solo = _solo(jobs)
    main = torch.cuda.current_stream()
    streams = [torch.cuda.Stream() for _ in jobs]
    for st, (s, out, inputs) in zip(streams, jobs):
        st.wait_stream(main)
        s.solve_into(out, *inputs, stream=st)
    for st in streams:
        main.wait_stream(st)
    torch.cuda.synchronize()
    _check_vs_solo(jobs, solo)


def test_multi_fallback_paths(gpu):
    """Same-model pairs, one job, a zero-env job and large batches take the one-after-another
    path; results are still the solo ones."""
    from osc_amd.solver import OSCBatchSolver, solve_multi_into
    s = OSCBatchSolver("unitree_go2")
    d1 = generate("unitree_go2", 100, SEED_BASE + 41, "tumbling", "bernoulli")
    d2 = generate("unitree_go2", 37, SEED_BASE + 42, "standing", "ones")
    jobs = [(s, s.alloc_outputs(100), s.prepare(**d1)), (s, s.alloc_outputs(37), s.prepare(**d2)),
            (s, s.alloc_outputs(0), s.prepare(**generate("unitree_go2", 0, 1, "standing", "ones")))]
    solve_multi_into(jobs)
    torch.cuda.synchronize()
    for _, out, inputs in jobs[:2]:
        ref = s.alloc_outputs(out.tau.shape[0])
        s.solve_into(ref, *inputs)
        torch.cuda.synchronize()
        assert np.array_equal(out.tau.cpu().numpy(), ref.tau.cpu().numpy())


def test_multi_rejects_bad_jobs(gpu):
    import ctypes
    from osc_amd import _lib
    from osc_amd.solver import OSCBatchSolver, solve_multi_into
    s = OSCBatchSolver("unitree_go2")
    d = generate("unitree_go2", 8, SEED_BASE + 43, "standing", "ones")
    out = s.alloc_outputs(8)
    out.workspace = out.workspace[:16]           # too small
    with pytest.raises(_lib.OSCError) as e:
        solve_multi_into([(s, out, s.prepare(**d))])
    assert e.value.code == 1
    assert _lib.lib().osc_batch_solve_multi(None, 1, None) == 1
    assert _lib.lib().osc_batch_solve_multi(None, 0, None) == 0


def test_multi_fixup_rescues_stalled_envs(gpu):
    """The two-model kernels run the cold fix-up pass too (a second interior-point launch over the
    envs the solve left not OK): the census's stalled and formerly unrefined joint-state envs
    (tests/golden/*_joint_states.npz), solved as one Go2 + WaLTER call, all come back OK, bitwise
    the solo solves (whose fix-up runs in the same launch) and at the fixtures' optimum."""
    import os
    from osc_amd.solver import OSCBatchSolver, solve_multi_into
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    keys = ("M", "C", "J", "b", "T", "mask")
    sets = {"unitree_go2": ("go2_stalled_joint_states.npz", "go2_unrefined_joint_states.npz"),
            "walter_sr": ("walter_stalled_joint_states.npz",)}
    jobs, refs = [], []
    for robot in ROBOTS:
        gs = [np.load(os.path.join(gdir, f)) for f in sets[robot]]
        d = {k: np.concatenate([g[k] for g in gs]) for k in keys + ("tau",)}
        s = OSCBatchSolver(robot)
        jobs.append((s, s.alloc_outputs(d["M"].shape[0], want_x=True),
                     s.prepare(*(d[k] for k in keys))))
        refs.append(d["tau"])
    solo = _solo_sized(jobs)
    solve_multi_into(jobs)
    torch.cuda.synchronize()
    for (s, out, _), (tau, x, st), ref in zip(jobs, solo, refs):
        got = out.tau.cpu().numpy()
        assert (out.status.cpu().numpy() == 0).all(), (s.robot, out.status.cpu().numpy())
        assert (st == 0).all()
        assert np.array_equal(got, tau) and np.array_equal(out.x.cpu().numpy(), x), s.robot
        err = np.abs(got - ref).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), 1.0)
        assert err.max() <= NORM_TOL, (s.robot, err.max())


def _solo_sized(jobs):
    out = []
    for s, o, inputs in jobs:
        r = s.alloc_outputs(o.tau.shape[0], want_x=True)
        s.solve_into(r, *inputs)
        out.append(r)
    torch.cuda.synchronize()
    return [(r.tau.cpu().numpy(), r.x.cpu().numpy(), r.status.cpu().numpy()) for r in out]
