"""GPU stage parity: the reduced QP osc_batch_assemble builds (setup kernel, phases A-D) is checked against the
oracle's full QP (oracle/osc_qp.py) through properties that do not depend on how the
reduction is computed:
  * x(y) satisfies the dynamics equality M dv + C - B u - Jc z = 0 for ANY y (autogen.py:87;
    checks X and U), in either reduced coordinate system the kernel uses:
      y = (dv_a, z): dv_b = X[y;1] (nb rows of X), dv_a = y_u, u = U[y;1]      (walter_sr)
      y = (u, z):    dv = X[y;1] (nv rows of X), u = y_u, no U stored           (unitree_go2)
  * 1/2 y'Hr y + g'y differs from the full objective 1/2 x'Hx + f'x by a constant
    (checks Hr and g against H, f of autogen.py:304-319)
"""
import ctypes
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from osc_amd import _lib
from osc_amd.robots import dims
from osc_amd.synth import SEED_BASE, generate
from osc_qp import b_matrix, build_qp, contact_jacobian, load_model

pytestmark = pytest.mark.gpu


def unpack_hr(block, ny):
    """The workspace's compact Hr (include/osc_batch.h): A = rows 16..ny-1 (ny columns each),
    then T = the upper triangle of Hr[0:16, 0:16] row by row."""
    Hr = np.zeros((ny, ny))
    A = block[:(ny - 16) * ny].reshape(ny - 16, ny)
    Hr[16:, :] = A
    Hr[:, 16:] = A.T
    t = (ny - 16) * ny
    for a in range(16):
        Hr[a, a:16] = block[t:t + 16 - a]
        Hr[a:16, a] = block[t:t + 16 - a]
        t += 16 - a
    return Hr


@pytest.mark.parametrize("robot,mask_mode", [("unitree_go2", "bernoulli"), ("walter_sr", "bernoulli"),
                                             ("unitree_go2", "zeros")])
def test_reduced_qp_consistent_with_oracle_qp(gpu, robot, mask_mode):
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver(robot)
    d = dims(robot)
    nv, nu, nc, nz = d["nv"], d["nu"], d["nc"], d["nz"]
    nb, ny = nv - nu, nu + nz
    nenv = 16
    inp = generate(robot, nenv, SEED_BASE + 31, "tumbling", mask_mode)
    args = s.prepare(**inp)
    L = _lib.lib()
    nbytes, ebytes = ctypes.c_size_t(), ctypes.c_size_t()
    assert L.osc_workspace_bytes(s._h, nenv, ctypes.byref(nbytes)) == 0
    assert L.osc_workspace_env_bytes(s._h, ctypes.byref(ebytes)) == 0
    sz = ebytes.value // 8
    assert nbytes.value >= sz * 8 * nenv
    ev = lambda a: (a + 1) // 2 * 2
    ny1p = ev(ny + 1)
    # layout documented in include/osc_batch.h: torque coordinates (both robots by default,
    # Dims<..., TY = true> in csrc/osc_batch.hip): [g | Hr | X (nv rows) | H_dv | f_dv | sol]
    # (sol = the interior point's y / active multipliers / status for the refinement pass)
    o_g, o_u = 0, ev(ny)
    ty = True
    nxr = nv if ty else nb
    o_hr = o_u + (0 if ty else nu * ny1p)
    # Hr compact (round 6; osc_device.hpp hr_off): rows 16.. whole, then the leading 16 x 16
    # block's upper triangle packed row-major
    hr_size = (ny - 16) * ny + 16 * 17 // 2
    o_x = o_hr + ev(hr_size)
    o_hd = o_x + nxr * ny1p
    o_gd = o_hd + nv * nv
    nrl = (2 * nu + 6 * nc + 15) // 16
    assert sz == o_gd + ev(nv) + ev(ny) + nrl * 16 + 2
    dbg = torch.zeros((nbytes.value // 8,), dtype=torch.float64, device=gpu)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = L.osc_batch_assemble(s._h, nenv, *[p(a) for a in args], p(dbg), nbytes,
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    D = dbg.cpu().numpy()[:nenv * sz].reshape(nenv, sz)
    model = load_model(robot)
    rng = np.random.default_rng(0)
    for e in range(nenv):
        Hr = unpack_hr(D[e, o_hr:o_hr + hr_size], ny)
        g = D[e, o_g:o_g + ny]
        U = np.eye(nu, ny + 1) if ty else D[e, o_u:o_hr].reshape(nu, ny1p)[:, :ny + 1]
        X = D[e, o_x:o_hd].reshape(nxr, ny1p)[:, :ny + 1]
        # H_dv / f_dv: the dv blocks of the oracle's H and f (autogen.py:304-319)
        a_ = [inp[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp_ = build_qp(model, *a_)
        Hd, gd = D[e, o_hd:o_gd].reshape(nv, nv), D[e, o_gd:o_gd + nv]
        assert np.abs(Hd - qp_.H[:nv, :nv]).max() <= 1e-12 * np.abs(qp_.H[:nv, :nv]).max()
        assert np.abs(gd - qp_.f[:nv]).max() <= 1e-12 * max(np.abs(qp_.f[:nv]).max(), 1.0)
        np.testing.assert_array_equal(Hr, Hr.T)
        a = [inp[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *a)
        M, C, J = a[0], a[1], a[2]
        pinned = np.repeat(a[5] == 0, 3)

        def x_of(y):
            y1 = np.append(y, 1.0)
            dv = X @ y1 if nxr == nv else np.concatenate([X @ y1, y[:nu]])
            return np.concatenate([dv, U @ y1, y[nu:]])

        objs = []
        for _ in range(4):
            y = 10.0 * rng.standard_normal(ny)
            y[nu:][pinned] = 0.0
            x = x_of(y)
            dv, u, z = x[:nv], x[nv:nv + nu], x[nv + nu:]
            res = M @ dv + C - b_matrix(model) @ u - contact_jacobian(model, J) @ z
            assert np.abs(res).max() <= 1e-10 * (1 + np.abs(M).max() * np.abs(x).max())
            full = 0.5 * x @ qp.H @ x + qp.f @ x
            red = 0.5 * y @ Hr @ y + g @ y
            objs.append((full, red, abs(full) + 0.5 * np.abs(x) @ np.abs(qp.H) @ np.abs(x)))
        for (f0, r0, s0), (f1, r1, s1) in zip(objs, objs[1:]):
            assert abs((f1 - f0) - (r1 - r0)) <= 1e-11 * max(s0, s1)


def test_split_stages_equal_fused_solve(gpu):
    """osc_batch_assemble + osc_batch_solve_assembled == osc_batch_solve, bit for bit."""
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver("unitree_go2")
    inp = generate("unitree_go2", 256, SEED_BASE + 32, "tumbling", "bernoulli")
    args = s.prepare(**inp)
    a = s.alloc_outputs(256, want_x=True)
    b = s.alloc_outputs(256, want_x=True)
    s.solve_into(a, *args)
    s.assemble_into(b, *args)
    s.solve_assembled_into(b, args[5])
    torch.cuda.synchronize()
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_refine_steps_above_round_length_clamped(gpu):
    """without wheel rows a refinement round runs at most 8 steps, and an env counts as
    converged only from its refine_steps-th step on, so a tuning of refine_steps = 12 used to
    leave EVERY env UNREFINED.  osc_model_create_tuned clamps it to 8: every env OK, bitwise the
    refine_steps = 8 solve."""
    from osc_amd.solver import OSCBatchSolver
    inp = generate("unitree_go2", 512, SEED_BASE + 34, "tumbling", "bernoulli")
    outs = []
    for steps in (12, 8):
        s = OSCBatchSolver("unitree_go2", tuning={"refine_steps": steps})
        args = s.prepare(**inp)
        o = s.alloc_outputs(512, want_x=True)
        s.solve_into(o, *args)
        torch.cuda.synchronize()
        outs.append(o)
    st = outs[0].status.cpu().numpy()
    assert (st == 0).all(), np.bincount(st)
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(outs[0], k), getattr(outs[1], k)), k


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr"])
def test_ipm_variants_bitwise_equal(gpu, robot):
    """The one-wave-per-SIMD variant (Hr in LDS where it fits, AGPR spill space) and the
    two-waves variant (Hr streamed from L2) run the same arithmetic: identical outputs."""
    from osc_amd.solver import OSCBatchSolver
    inp = generate(robot, 512, SEED_BASE + 33, "tumbling", "bernoulli")
    outs = []
    for force in (100000000, 0):
        s = OSCBatchSolver(robot, tuning={"small_batch_max": force})
        args = s.prepare(**inp)
        o = s.alloc_outputs(512, want_x=True)
        s.solve_into(o, *args)
        torch.cuda.synchronize()
        outs.append(o)
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(outs[0], k), getattr(outs[1], k)), k


@pytest.mark.parametrize("robot,nenv,scenario,park", [
    ("walter_sr", 20480, "tumbling", None),     # the default park iteration (compaction on: 5 rounds)
    ("unitree_go2", 20480, "tumbling", "11"),   # forced: the two-wave kernel's park / resume
    ("walter_sr", 16387, "standing", None),     # ragged: a partial last wavefront, parked slots
    ("unitree_go2", 16390, "standing", "12"),   # not a multiple of four
])
def test_compaction_bitwise_equal(gpu, robot, nenv, scenario, park):
    """Lockstep compaction (ParkArgs): envs not converged at the park iteration
    continue in a second pass, packed four to a wavefront -- each env takes exactly the steps it
    takes in one pass, so tau, x, status and iters are bitwise those of the single pass."""
    from osc_amd.solver import OSCBatchSolver
    inp = generate(robot, nenv, SEED_BASE + 34, scenario, "bernoulli")
    outs = []
    for p in (park, "0"):
        s = OSCBatchSolver(robot, tuning=None if p is None else {"park_it": int(p)})
        args = s.prepare(**inp)
        o = s.alloc_outputs(nenv, want_x=True)
        s.solve_into(o, *args)
        torch.cuda.synchronize()
        outs.append(o)
    it = outs[1].iters.cpu().numpy()
    assert (it > int(park or 16)).any() and (it <= int(park or 16)).any()   # both passes ran
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(outs[0], k), getattr(outs[1], k)), k


@pytest.mark.parametrize("robot,nenv,seed", [("walter_sr", 4096, 23), ("unitree_go2", 8192, 22)])
def test_results_independent_of_wave_mates(gpu, robot, nenv, seed):
    """Every env's result is bitwise independent of the envs that share its wavefront: the
    permuted batch returns the permuted results.  (The refinement repeats a round for the whole
    wavefront when one env's refined point violates a row; an env whose round ended without a
    violation keeps that round's result -- before round 3 it was refined again, at rounding
    level, whenever a wave-mate asked.  The seeds are the feature-off fingerprint batches, which
    hold such wavefronts.)"""
    from osc_amd.solver import OSCBatchSolver
    s = OSCBatchSolver(robot)
    inp = generate(robot, nenv, SEED_BASE + seed, "tumbling", "bernoulli")
    perm = np.random.default_rng(5).permutation(nenv)
    a = s.solve(**inp, want_x=True)
    b = s.solve(**{k: v[perm] for k, v in inp.items()}, want_x=True)
    torch.cuda.synchronize()
    pt = torch.from_numpy(perm).to(a.tau.device)
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(a, k)[pt], getattr(b, k)), k
