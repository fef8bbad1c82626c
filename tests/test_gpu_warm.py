"""Warm start across control ticks (osc_batch_solve_warm; the reference's SetWarmStart,
operational_space_controller.h:519-526): every tick of a 1 % random walk (SURVEY.md §8d warm runs)
must still hit the exact optimum within the parity tolerance of test_gpu_parity.py, with fewer
interior-point iterations than cold solves; a zero-filled state is exactly the cold solve."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from osc_amd.synth import SEED_BASE, generate, random_walk
from osc_qp import build_qp, load_model, torque
from qp_exact import solve_exact

pytestmark = pytest.mark.gpu
NORM_TOL = 1e-9          # achieved bound of tests/test_gpu_parity.py (refined solves)


def _oracle_tau(robot, d, e):
    model = load_model(robot)
    args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
    return torque(model, solve_exact(model, build_qp(model, *args), *args[:3]).x)


@pytest.mark.parametrize("robot,scenario,mask_mode", [("unitree_go2", "standing", "ones"),
                                                      ("walter_sr", "standing", "ones"),
                                                      ("walter_sr", "tumbling", "bernoulli")])
def test_warm_ticks_match_oracle_with_fewer_iterations(gpu, robot, scenario, mask_mode):
    from osc_amd.solver import OSCBatchSolver
    solver = OSCBatchSolver(robot)
    nenv, ticks = 64, 5
    d = generate(robot, nenv, SEED_BASE + 21, scenario, mask_mode)
    rng = np.random.default_rng(21)
    warm = solver.alloc_warm_state(nenv)
    out = solver.alloc_outputs(nenv)
    cold_it, warm_it = [], []
    for k in range(ticks):
        if k > 0:
            d = random_walk(d, rng, 0.01)
            if mask_mode == "bernoulli":            # contact-mode switching between ticks
                d["mask"] = (rng.uniform(size=d["mask"].shape) < 0.75).astype(np.float64)
        args = solver.prepare(**d)
        solver.solve_warm_into(out, warm, *args)
        cold = solver.solve(*args)
        torch.cuda.synchronize()
        assert (out.status.cpu().numpy() == 0).all()
        tau = out.tau.cpu().numpy()
        ct = cold.tau.cpu().numpy()
        for e in range(0, nenv, 8):
            ref = _oracle_tau(robot, d, e)
            assert np.abs(tau[e] - ref).max() / max(np.abs(ref).max(), 1.0) <= NORM_TOL, (k, e)
        assert (np.abs(tau - ct).max(axis=1) / np.maximum(np.abs(ct).max(axis=1), 1.0)).max() <= 2 * NORM_TOL
        if k == 0:
            assert torch.equal(out.tau, cold.tau)   # zero-filled state = cold start, bitwise
        else:
            cold_it.append(cold.iters.double().mean().item())
            warm_it.append(out.iters.double().mean().item())
    assert np.mean(warm_it) < np.mean(cold_it), (warm_it, cold_it)


def test_warm_state_api_errors(gpu):
    from osc_amd import _lib
    from osc_amd.solver import OSCBatchSolver
    solver = OSCBatchSolver("unitree_go2")
    nenv = 8
    args = solver.prepare(**generate("unitree_go2", nenv, SEED_BASE + 22))
    out = solver.alloc_outputs(nenv)
    with pytest.raises(_lib.OSCError):
        solver.solve_warm_into(out, None, *args)
    short = solver.alloc_warm_state(nenv)[:-2]          # one env's state short
    with pytest.raises(_lib.OSCError):
        solver.solve_warm_into(out, short, *args)


@pytest.mark.parametrize("nenv", [4096, 8192])
def test_warm_fixup_rescues_unrefined(gpu, nenv):
    """an env whose refinement finds no KKT point (OSC_SOLVE_UNREFINED) goes to the cold
    fix-up pass like a MAX_ITER env (include/osc_batch.h: the warm entry re-solves every env its
    warm pass leaves not OK) -- at 8,192 (two rounds of wavefronts: the two-wave kernel, which
    refines in a separate pass, then the fix-up launch) and at 4,096 (the one-wave kernel, whose
    wavefronts run the fix-up in the same launch right after their warm pass, round 5).  Forced
    here: refine_max_move = 0 rejects every refinement, so every env is re-solved cold to
    mu <= 1e-12 (iters reported as max_iter + the fix-up's count).  Its refinement is rejected
    again, so it stays UNREFINED -- but the returned iterate is the 1e-12 one, within the 1e-5
    contract of the default solve, not the warm early stop's (up to ~3e-2, test_gpu_wheels::
    test_rejected_refinement_is_reported)."""
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver("unitree_go2", tuning={"refine_max_move": 0.0})
    ref = OSCBatchSolver("unitree_go2")
    d = generate("unitree_go2", nenv, SEED_BASE + 23, "tumbling", "bernoulli")
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv)
    s.solve_warm_into(out, s.alloc_warm_state(nenv), *args)
    good = ref.solve(*args)
    torch.cuda.synchronize()
    st, it = out.status.cpu().numpy(), out.iters.cpu().numpy()
    # (UNREFINED everywhere, except an env whose 1e-12 iterate is already the optimum -- its
    # refinement does not move y, which even refine_max_move = 0 accepts: 4 of 8,192 measured)
    assert np.isin(st, [0, 3]).all() and (st == 3).sum() >= nenv - nenv // 128, np.bincount(st)
    assert (it > s.desc.max_iter).all(), it.min()
    assert (good.status.cpu().numpy() == 0).all()
    tau, gt = out.tau.cpu().numpy(), good.tau.cpu().numpy()
    nw = (np.abs(tau - gt).max(axis=1) / np.maximum(np.abs(gt).max(axis=1), 1.0))
    assert nw.max() <= 1e-5, (nw.max(), int(np.argmax(nw)))
