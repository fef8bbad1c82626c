"""GPU tests of the opt-in wheel no-slip rows, the dual solution export, the
UNREFINED status, and the bitwise-unchanged feature-off path.

Wheel rows: walter_sr_wheels/autogen/autogen.py:128-240 (commented out in the reference), joint
lookup :64-94; oracle: oracle/osc_qp.py wheel_rows + oracle/qp_exact.py (phase-1 start, active
set, KKT certificate), pinned to the literal design by tests/test_oracle.py.  Tolerances as
tests/test_gpu_parity.py: normwise <= 1e-9, elementwise (above 1 % of the norm) <= 1e-7 against
the certified exact optimum; the rows themselves hold to 1e-9 at the returned x.

Duals (the reference's OsqpSolver::dual_solution, operational_space_controller.h:534-535):
checked by the OSQP-form KKT certificate of (x, y) on EVERY env of the BASELINE-size batches,
batched in torch on the GPU (stated tolerances below).
"""
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from osc_amd.robots import config_path, dims
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions
from osc_qp import BIG_NUMBER, WheelRows, build_qp, load_model, torque
from qp_exact import solve_exact

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
NOSLIP_YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                           "walter_sr_wheels_noslip_config.yaml")
NORM_ACH, ELEM_ACH = 1e-9, 1e-7
# With the wheel rows on: 1e-8 normwise.  Seven or eight grounded wheels put 14-16 rows on nv = 14
# accelerations; the oracle's own torques move by up to 1e-11 under 1e-16 relative noise in J
# (condition ~1e5, tools/wheel_ipm_model.py), and the product's fp64 transforms of the rows
# (Gram-Schmidt in dv and y space) land within 1.7e-8 of the oracle on the worst of
# 1,024 numpy-restated envs, median 1e-13 -- hence also a median bar.
WHEEL_NORM, WHEEL_ELEM, WHEEL_MEDIAN = 1e-8, 1e-6, 1e-10
# Tumbling envs with the wheel rows: the interior point stalls on ~0.5 % (2,048-env census,
# tools/wheel_census.py, DESIGN.md §3.1: 9-11 per 2,048 at seeds 86/91/93, 0 standing) and the
# active-set fallback (osc_gi_kernel) takes every one of them in the censuses (profiles/r04r/):
# no non-OK status is allowed; were one to appear it could only be MAX_ITER, never a wrong OK.
WHEEL_MAX_ITER_PER_2048 = 0


def _wheel_statuses(st, scenario, where):
    """OK, or MAX_ITER with the census rate bound; standing: OK everywhere."""
    bad = st != 0
    assert set(np.unique(st[bad]).tolist()) <= {1}, (where, np.bincount(st))
    limit = 0 if scenario == "standing" else WHEEL_MAX_ITER_PER_2048 * len(st) // 2048
    assert bad.sum() <= limit, (where, np.bincount(st), np.nonzero(bad)[0][:20])
# KKT certificate of the GPU's (x, y), each residual scaled as oracle/qp_exact.kkt_certificate.
# Stationarity: the duals are recovered from x (osc_dual_kernel), so it measures x's optimality
# through H_dv and M^-1 -- a design vector 1e-9 off in dv shows up as ~1e-8..1e-7 here (WaLTER).
# Complementarity: the contact multipliers go on rows within 1e-8 (relative) of their bound, so a
# design vector 1e-9 off leaves products up to ~1e-8 of the scale.  One-sided rows only (round 4):
# an equality row's multiplier is free and its residual is the primal measure -- the nearly
# dependent wheel rows carry multipliers ~1e13 (the exact oracle's too), whose product with a 1e-9
# residual is no complementarity gap (the 1-2 per 2,048 envs round 4's census flagged, all of them).
KKT_STAT, KKT_PRIMAL, KKT_DUAL, KKT_COMP = 1e-6, 1e-9, 1e-9, 1e-7

_solvers = {}


def solver(key):
    from osc_amd.solver import OSCBatchSolver
    if key not in _solvers:
        _solvers[key] = (OSCBatchSolver("walter_sr_wheels", NOSLIP_YAML) if key == "noslip"
                         else OSCBatchSolver(key))
    return _solvers[key]


def _rel_errors(tau, ref):
    tau, ref = np.asarray(tau), np.asarray(ref)
    nrm = np.maximum(np.abs(ref).max(axis=-1, keepdims=True), 1.0)
    normwise = (np.abs(tau - ref) / nrm).max(axis=-1)
    big = np.abs(ref) >= 1e-2 * np.abs(ref).max(axis=-1, keepdims=True)
    elem = np.where(big, np.abs(tau - ref) / np.maximum(np.abs(ref), 1e-300), 0.0).max(axis=-1)
    return normwise, elem


def _wheel():
    return WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))


def test_feature_off_bitwise_unchanged(gpu):
    """Models without wheel rows -- the feature-off path -- give bitwise the results of the
    last intentional numerical change of the default kernels (tests/golden/feature_off_hashes.json,
    made by tests/golden/make_feature_off_hashes.py with that library)."""
    from golden.make_feature_off_hashes import fingerprint
    ref = json.load(open(os.path.join(HERE, "golden", "feature_off_hashes.json")))
    for c in ref["cases"]:
        d = generate(c["robot"], c["nenv"], c["seed"], c["scenario"], c["mask"])
        assert fingerprint(solver(c["robot"]), d) == c["sha256"], c


@pytest.mark.parametrize("scenario,mask_mode,seed", [("standing", "ones", 81),
                                                      ("tumbling", "bernoulli", 82)])
def test_wheel_rows_vs_oracle(gpu, scenario, mask_mode, seed):
    """64 fresh envs with the no-slip rows on: torques against the exact oracle optimum, the
    rows hold at the returned design vector, every env converged and refined."""
    nenv = 64
    model = load_model("walter_sr_wheels")
    wheel = _wheel()
    d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, scenario, mask_mode)
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + seed + 1)
    res = solver("noslip").solve(**d, want_x=True, wheel_dir=wd)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    # every env converges standing; tumbling a stalled interior point is flagged MAX_ITER, never
    # returned as OK: the OK ones are held to the oracle
    _wheel_statuses(st, scenario, "vs_oracle")
    x = res.x.cpu().numpy()
    ref, viol, envs = [], [], []
    for e in range(nenv):
        if st[e] != 0:
            continue
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *args, wheel, wd[e])
        viol.append(np.abs(qp.Aw @ x[e] - qp.bw).max() / (1.0 + np.abs(qp.bw).max()))
        # (the oracle's dual active-set method takes the degenerate envs the primal one refuses:
        # every env is checked)
        ref.append(torque(model, solve_exact(model, qp, *args[:3]).x))
        envs.append(e)
    nw, el = _rel_errors(res.tau.cpu().numpy()[envs], np.array(ref))
    assert nw.max() <= WHEEL_NORM and el.max() <= WHEEL_ELEM, (nw.max(), el.max(), int(np.argmax(nw)))
    assert np.median(nw) <= WHEEL_MEDIAN, np.median(nw)
    assert max(viol) <= 1e-9, max(viol)


def test_wheel_rows_that_vanish_change_nothing(gpu, tmp_path):
    """Rows that vanish (zero directions, no wheel joints) leave the reference's QP: the
    wheel-row kernel then agrees with the feature-off kernel to rounding."""
    from osc_amd.solver import OSCBatchSolver
    text = open(NOSLIP_YAML).read().replace("wheel_dofs: [7, 7, 9, 9, 11, 11, 13, 13]",
                                            "wheel_dofs: [-1, -1, -1, -1, -1, -1, -1, -1]")
    (tmp_path / "nodof.yaml").write_text(text)
    d = generate("walter_sr_wheels", 128, SEED_BASE + 83, "tumbling", "bernoulli")
    off = solver("walter_sr_wheels").solve(**d)
    on = OSCBatchSolver("walter_sr_wheels", str(tmp_path / "nodof.yaml")).solve(
        **d, wheel_dir=np.zeros((128, 8, 6)))
    torch.cuda.synchronize()
    assert (on.status.cpu().numpy() == 0).all()
    nw, _ = _rel_errors(on.tau.cpu().numpy(), off.tau.cpu().numpy())
    assert nw.max() <= 1e-10, nw.max()


def test_wheel_model_entry_points(gpu):
    """A wheel model needs its directions: the plain entries (cold and warm) and a multi-model
    job without them refuse it; split assemble + solve equals the fused call."""
    from osc_amd import _lib
    s = solver("noslip")
    d = generate("walter_sr_wheels", 8, SEED_BASE + 84, "tumbling", "bernoulli")
    wd = torch.from_numpy(wheel_directions("walter_sr_wheels", d, _wheel().dof, _wheel().radius,
                                           SEED_BASE + 85)).cuda()
    args = s.prepare(**d)
    out = s.alloc_outputs(8, want_x=True)
    with pytest.raises(_lib.OSCError) as e:
        s.solve_into(out, *args)
    assert e.value.code == 1
    warm = s.alloc_warm_state(8)
    with pytest.raises(_lib.OSCError) as e:
        s.solve_warm_into(out, warm, *args)
    assert e.value.code == 1
    from osc_amd.solver import solve_multi_into
    with pytest.raises(_lib.OSCError) as e:
        solve_multi_into([(s, out, args)])
    assert e.value.code == 1
    s.solve_into(out, *args, wheel_dir=wd)
    split = s.alloc_outputs(8, want_x=True)
    s.assemble_into(split, *args[:5], args[5], wheel_dir=wd)
    s.solve_assembled_into(split, args[5])
    torch.cuda.synchronize()
    assert torch.equal(out.tau, split.tau) and torch.equal(out.x, split.x)


# ---------------------------------------------------------------------------- duals / KKT
def _batched_qp(robot, M, C, J, b, T, mask, wheel=None, wd=None):
    """The reference QP of oracle/osc_qp.build_qp for a whole batch, on the GPU (torch fp64):
    H, f, A = [Aeq (; Aw); Aineq; I], l, u."""
    m = load_model(robot)
    nv, nu, nz, n, nc, ns = m.nv, m.nu, m.nz, m.n, m.nc, m.ns
    dev, E = M.device, M.shape[0]
    W = torch.as_tensor(np.concatenate([np.repeat(m.w_pos, 3), np.repeat(m.w_rot, 3)]), device=dev)
    t = torch.cat([T[:, :, 0:3].reshape(E, -1), T[:, :, 3:6].reshape(E, -1)], dim=1)
    H = torch.zeros(E, n, n, dtype=torch.float64, device=dev)
    JW = J.transpose(1, 2) * W
    H[:, :nv, :nv] = 2.0 * JW @ J + 2.0 * m.w_reg * torch.eye(nv, device=dev, dtype=torch.float64)
    idx = torch.arange(nv, n, device=dev)
    H[:, idx, idx] = torch.where(idx < nv + nu, 2.0 * (m.w_torque + m.w_reg), 2.0 * m.w_reg).double()
    f = torch.zeros(E, n, dtype=torch.float64, device=dev)
    f[:, :nv] = 2.0 * torch.einsum("eij,ej->ei", JW, b - t)
    r0 = 3 * ns - nz
    Jc = J[:, r0:3 * ns, :].transpose(1, 2)
    Aeq = torch.zeros(E, nv, n, dtype=torch.float64, device=dev)
    Aeq[:, :, :nv] = M
    Aeq[:, nv - nu:, nv:nv + nu] = -torch.eye(nu, device=dev, dtype=torch.float64)
    Aeq[:, :, nv + nu:] = -Jc
    rows, lo, hi = [Aeq], [-C], [-C]
    if wheel is not None:
        Aw = torch.zeros(E, 2 * nc, n, dtype=torch.float64, device=dev)
        bw = torch.zeros(E, 2 * nc, dtype=torch.float64, device=dev)
        for i in range(nc):
            Jp, bi = J[:, r0 + 3 * i:r0 + 3 * i + 3, :], b[:, r0 + 3 * i:r0 + 3 * i + 3]
            for side in range(2):
                dvec = wd[:, i, 3 * side:3 * side + 3]
                Aw[:, 2 * i + side, :nv] = torch.einsum("ec,ecj->ej", dvec, Jp)
                if side == 0 and wheel.dof[i] >= 0:
                    Aw[:, 2 * i, wheel.dof[i]] -= wheel.radius[i]
                bw[:, 2 * i + side] = -(dvec * bi).sum(dim=1)
            Aw[:, 2 * i:2 * i + 2] *= mask[:, i, None, None]
            bw[:, 2 * i:2 * i + 2] *= mask[:, i, None]
        rows.append(Aw)
        lo.append(bw)
        hi.append(bw)
    Ain = torch.zeros(E, 4 * nc, n, dtype=torch.float64, device=dev)
    for k in range(nc):
        for r, (sx, sy) in enumerate(((1, 1), (-1, 1), (1, -1), (-1, -1))):
            Ain[:, 4 * k + r, nv + nu + 3 * k:nv + nu + 3 * k + 3] = torch.tensor(
                [sx, sy, -m.mu], dtype=torch.float64, device=dev)
    rows += [Ain, torch.eye(n, dtype=torch.float64, device=dev).expand(E, n, n)]
    inf = 1e30
    mrep = mask.repeat_interleave(3, dim=1)
    zlb = torch.tensor([-inf, -inf, 0.0] * nc, dtype=torch.float64, device=dev)
    zub = torch.tensor([inf, inf, BIG_NUMBER] * nc, dtype=torch.float64, device=dev)
    full = lambda v: torch.full((E, v[0]), v[1], dtype=torch.float64, device=dev)
    lo += [full((4 * nc, -inf)), full((nv, -inf)),
           torch.as_tensor(m.u_lb, device=dev).expand(E, nu), zlb * mrep]
    hi += [full((4 * nc, 0.0)), full((nv, inf)),
           torch.as_tensor(m.u_ub, device=dev).expand(E, nu), zub * mrep]
    return H, f, torch.cat(rows, dim=1), torch.cat(lo, dim=1), torch.cat(hi, dim=1)


def _kkt(H, f, A, l, u, x, y):
    """Per-env residuals as oracle/qp_exact.kkt_certificate, batched.  These SCALED residuals
    certify optimality up to a relative tolerance -- they do not by themselves bound the torque
    error at 1e-5 (stationarity 1e-6 of a gradient scale up to 1e4 is an absolute
    residual up to 1e-2 along directions of curvature 2 w_reg = 2e-4).  The torque contract is
    checked against the exact optimum itself, every env (oracle/parallel.py: the full oracle at
    4,096 envs, the GPU-seeded certified oracle at 65,536)."""
    Ax = torch.einsum("emn,en->em", A, x)
    grad = torch.einsum("eij,ej->ei", H, x) + f
    Aty = torch.einsum("emn,em->en", A, y)
    stat = (grad + Aty).abs().amax(dim=1)
    scale_d = 1.0 + torch.maximum(grad.abs().amax(dim=1), Aty.abs().amax(dim=1))
    lo_fin, hi_fin = l > -1e20, u < 1e20
    viol = torch.maximum(torch.where(hi_fin, Ax - u, -1e300), torch.where(lo_fin, l - Ax, -1e300))
    viol = viol.clamp_min(0.0).amax(dim=1)
    bnd = (torch.where(hi_fin, u.abs(), 0.0) + torch.where(lo_fin, l.abs(), 0.0)).amax(dim=1)
    scale_p = 1.0 + torch.maximum(Ax.abs().amax(dim=1), bnd)
    yp, ym = y.clamp_min(0.0), (-y).clamp_min(0.0)
    dual = torch.maximum(torch.where(hi_fin, 0.0, yp).amax(dim=1),
                         torch.where(lo_fin, 0.0, ym).amax(dim=1))
    scale_y = 1.0 + torch.where(l != u, y.abs(), 0.0).amax(dim=1)   # one-sided rows' multipliers
    one_sided = l != u   # (equality rows: free multipliers, residual in `primal`)
    comp = torch.maximum((yp * torch.where(hi_fin & one_sided, u - Ax, 0.0)).abs(),
                         (ym * torch.where(lo_fin & one_sided, Ax - l, 0.0)).abs()).amax(dim=1)
    return dict(stationarity=stat / scale_d, primal=viol / scale_p, dual=dual / scale_y,
                complementarity=comp / (scale_d * scale_p))


def _certify(cert, where):
    for k, tol in (("stationarity", KKT_STAT), ("primal", KKT_PRIMAL), ("dual", KKT_DUAL),
                   ("complementarity", KKT_COMP)):
        v = cert[k]
        assert v.max().item() <= tol, (where, k, v.max().item(), int(v.argmax().item()))


@pytest.mark.parametrize("robot,nenv,scenario,mask_mode", [
    ("unitree_go2", 65536, "tumbling", "bernoulli"),     # BASELINE north-star batch
    ("walter_sr", 8192, "tumbling", "bernoulli"),        # BASELINE configs[3]
    ("unitree_go2", 4096, "standing", "ones"),           # BASELINE configs[1]
])
def test_full_size_every_env_exact(gpu, robot, nenv, scenario, mask_mode):
    """EVERY env of a BASELINE-size batch against the exact optimum of the reference QP: the
    scaled KKT residuals of the exported duals y with x (stationarity H x + f + A'y = 0, primal
    feasibility, dual sign on one-sided rows, complementarity -- an optimality certificate up to a
    relative tolerance), then the torque contract itself: the exact optimum of every env from the
    working set the GPU's duals mark active, solved and certified by the oracle
    (oracle/parallel.seeded_batch; an env whose set does not certify gets the full oracle),
    normwise <= 1e-9 and elementwise <= 1e-7 (the achieved bars of test_gpu_parity.py)."""
    s = solver(robot)
    d = generate(robot, nenv, SEED_BASE + 9, scenario, mask_mode)
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv, want_y=True)
    s.solve_into(out, *args)
    torch.cuda.synchronize()
    st = out.status.cpu().numpy()
    assert (st == 0).all(), np.bincount(st)
    _certify(_kkt(*_batched_qp(robot, *args), out.x, out.y), robot)
    # the duals leave the torques and the design vector bitwise as the plain solve returns them
    ref = s.alloc_outputs(nenv, want_x=True)
    s.solve_into(ref, *args)
    torch.cuda.synchronize()
    assert torch.equal(ref.tau, out.tau) and torch.equal(ref.x, out.x)
    from parallel import seeded_batch
    model = load_model(robot)
    xo, seeded = seeded_batch(robot, d["M"], d["C"], d["J"], d["b"], d["T"], d["mask"],
                              out.y.cpu().numpy())
    nw, el = _rel_errors(out.tau.cpu().numpy(), xo[:, model.nv:model.nv + model.nu])
    print(f"\n{robot} {scenario} {nenv} envs: every env vs the exact optimum ({int(seeded.sum())} "
          f"from the GPU's certified active set, {int((~seeded).sum())} by the full oracle): "
          f"worst normwise {nw.max():.2e} (env {int(np.argmax(nw))}), worst elementwise "
          f"{el.max():.2e}")
    assert nw.max() <= NORM_ACH and el.max() <= ELEM_ACH, (nw.max(), el.max(), int(np.argmax(nw)))


def test_wheel_rows_kkt_certificate(gpu):
    """The same certificate with the wheel rows in A (their multipliers exported too)."""
    wheel = _wheel()
    s = solver("noslip")
    nenv = 2048
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 86, "tumbling", "bernoulli")
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 87)
    args = s.prepare(**d)
    wdt = torch.from_numpy(wd).cuda()
    out = s.alloc_outputs(nenv, want_y=True)
    s.solve_into(out, *args, wheel_dir=wdt)
    torch.cuda.synchronize()
    st = out.status.cpu().numpy()
    _wheel_statuses(st, "tumbling", "kkt")
    cert = _kkt(*_batched_qp("walter_sr_wheels", *args, wheel, wdt), out.x, out.y)
    ok = torch.from_numpy(st == 0).cuda()
    # every env reported OK is certified (the rows' multipliers from stationarity itself,
    # osc_dual_kernel, round 4: was 98 % with them from the refinement's last residual)
    for k, tol in (("stationarity", KKT_STAT), ("primal", KKT_PRIMAL), ("dual", KKT_DUAL),
                   ("complementarity", KKT_COMP)):
        v = cert[k][ok]
        assert v.max().item() <= tol, (k, v.max().item(), int(torch.nonzero(ok)[v.argmax()].item()))


def test_rejected_refinement_is_reported(gpu):
    """An env whose full-space refinement is rejected keeps the interior point's iterate and is
    reported as OSC_SOLVE_UNREFINED (3), not OK; its torques are only as accurate as the
    interior point's stop (Go2 eps_mu 1e-6: up to ~1e-2 normwise)."""
    from osc_amd.solver import OSCBatchSolver
    # every refinement moves y: all rejected
    s = OSCBatchSolver("unitree_go2", tuning={"refine_max_move": 0.0})
    d = generate("unitree_go2", 64, SEED_BASE + 88, "tumbling", "bernoulli")
    res = s.solve(**d)
    good = solver("unitree_go2").solve(**d)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    assert (st == 3).all(), np.bincount(st)
    assert (good.status.cpu().numpy() == 0).all()
    nw, _ = _rel_errors(res.tau.cpu().numpy(), good.tau.cpu().numpy())
    assert nw.max() <= 3e-2 and nw.max() > 0.0, nw.max()


def test_wheel_duals_leave_primal_unchanged(gpu):
    """Asking for the duals (osc_solve_extras.y) does not change the wheel model's solve: x, tau,
    status and iters are bitwise those of the call without them (the refinement runs the same
    fixed step count either way)."""
    wheel = _wheel()
    s = solver("noslip")
    nenv = 512
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 90, "tumbling", "bernoulli")
    wdt = torch.from_numpy(wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius,
                                            SEED_BASE + 91)).cuda()
    args = s.prepare(**d)
    a = s.alloc_outputs(nenv, want_y=True)
    s.solve_into(a, *args, wheel_dir=wdt)
    b = s.alloc_outputs(nenv, want_x=True)
    s.solve_into(b, *args, wheel_dir=wdt)
    torch.cuda.synchronize()
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


@pytest.mark.parametrize("scenario,mask_mode", [("standing", "ones"), ("tumbling", "bernoulli")])
def test_wheel_rows_warm_start(gpu, scenario, mask_mode):
    """Warm start with the wheel rows (osc_batch_solve_warm_ex; the reference's wheels controller
    warm-starts every tick, walter_sr_wheels/operational_space_controller.h:583, 591-600): five
    ticks of a 1 % random walk of the inputs (the wheel directions follow), masks fixed.  Every tick's
    warm solve agrees with the cold solve of the same tick to the wheel rows' tolerance, reports
    the same statuses, and takes fewer interior-point iterations on average after the first."""
    from osc_amd.synth import random_walk
    wheel = _wheel()
    s = solver("noslip")
    nenv = 1024
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 95, scenario, mask_mode)
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 96)
    rng = np.random.default_rng(7)
    warm = s.alloc_warm_state(nenv)
    wo, co = s.alloc_outputs(nenv), s.alloc_outputs(nenv)
    for tick in range(5):
        args = s.prepare(**d)
        wdt = torch.from_numpy(wd).cuda()
        s.solve_warm_into(wo, warm, *args, wheel_dir=wdt)
        s.solve_into(co, *args, wheel_dir=wdt)
        torch.cuda.synchronize()
        sw, sc = wo.status.cpu().numpy(), co.status.cpu().numpy()
        _wheel_statuses(sw, scenario, ("warm", tick))
        _wheel_statuses(sc, scenario, ("cold", tick))
        ok = (sw == 0) & (sc == 0)
        nw, _ = _rel_errors(wo.tau.cpu().numpy()[ok], co.tau.cpu().numpy()[ok])
        assert nw.max() <= WHEEL_NORM, (tick, nw.max())
        if tick > 0:   # (over the envs the interior point solved: the fallback's are < 0)
            ip = (wo.iters >= 0) & (co.iters >= 0)
            assert wo.iters[ip].float().mean() < co.iters[ip].float().mean(), tick
        d = random_walk(d, rng)
        # (directions re-derived from the walked state with the same seed: they move continuously
        # and stay consistent -- eight grounded wheels put 16 rows on 14 accelerations)
        wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 96)


# MAX_ITER envs of the round-4 census at max_iter 200 (seed offset 86, 2,048 tumbling envs,
# directions seed 87): the interior point stalls on them (multipliers 1e7-3e8).  At today's wheel
# max_iter 25 the refinement brings 9 of them to OK and the fallback takes 986 (split entries,
# profiles/r04_fbtest/): they are the hard envs of this batch whichever stage finishes them
STALLED_86 = (37, 75, 328, 357, 506, 555, 986, 1157, 1479, 1862)


def test_wheel_fallback_takes_the_stalled_envs(gpu):
    """The batch's hard envs (multipliers 1e7-3e8) -- finished by the refinement or by the
    Goldfarb-Idnani fallback on the full QP (osc_gi_kernel) -- reported OK and within the
    wheel-row tolerance of the exact oracle (tools/gi_fallback_model.py restates the fallback's
    sequence: <= 1e-11)."""
    wheel = _wheel()
    model = load_model("walter_sr_wheels")
    nenv = 2048
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 86, "tumbling", "bernoulli")
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 87)
    res = solver("noslip").solve(**d, want_x=True, wheel_dir=wd)
    torch.cuda.synchronize()
    st = res.status.cpu().numpy()
    _wheel_statuses(st, "tumbling", "fallback")
    assert (st[list(STALLED_86)] == 0).all(), st[list(STALLED_86)]
    # iters < 0 marks the envs the fallback solved (-(its steps), include/osc_batch.h)
    it = res.iters.cpu().numpy()
    assert it[986] < 0 and (it < 0).sum() >= 1, (it[list(STALLED_86)], (it < 0).sum())
    tau = res.tau.cpu().numpy()
    ref = []
    for e in STALLED_86:
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *args, wheel, wd[e])
        ref.append(torque(model, solve_exact(model, qp, *args[:3]).x))
    nw, el = _rel_errors(tau[list(STALLED_86)], np.array(ref))
    assert nw.max() <= WHEEL_NORM and el.max() <= WHEEL_ELEM, (nw.max(), el.max())


def test_wheel_fallback_runs_in_every_entry(gpu):
    """The active-set fallback runs behind every entry point: the assembly copies
    the raw rows it needs (M, C, J's and b's contact rows, the wheel directions) into the
    workspace, so split assemble + solve gives bitwise the fused call's x, tau, status and iters
    on every env -- all OK.  (Before round 5 the split path left 11 of these 2,048 envs MAX_ITER or
    UNREFINED.)  The envs the fallback solved (iters < 0) are within the wheel-row tolerance of
    the exact oracle."""
    wheel = _wheel()
    s = solver("noslip")
    nenv = 2048
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 86, "tumbling", "bernoulli")
    wdt = torch.from_numpy(wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius,
                                            SEED_BASE + 87)).cuda()
    args = s.prepare(**d)
    fused = s.alloc_outputs(nenv, want_x=True)
    s.solve_into(fused, *args, wheel_dir=wdt)
    split = s.alloc_outputs(nenv, want_x=True)
    s.assemble_into(split, *args[:5], args[5], wheel_dir=wdt)
    s.solve_assembled_into(split, args[5])
    torch.cuda.synchronize()
    sf = fused.status.cpu().numpy()
    assert (sf == 0).all(), np.bincount(sf)
    for k in ("tau", "x", "status", "iters"):
        assert torch.equal(getattr(fused, k), getattr(split, k)), k
    rest = np.nonzero(fused.iters.cpu().numpy() < 0)[0]
    assert len(rest) > 0, "no env needed the fallback in this batch"
    model = load_model("walter_sr_wheels")
    wd = wdt.cpu().numpy()
    ref = []
    for e in rest:
        a = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        ref.append(torque(model, solve_exact(model, build_qp(model, *a, wheel, wd[e]), *a[:3]).x))
    nw, el = _rel_errors(fused.tau.cpu().numpy()[rest], np.array(ref))
    assert nw.max() <= WHEEL_NORM and el.max() <= WHEEL_ELEM, (nw.max(), el.max())


def test_wheel_model_in_solve_multi(gpu):
    """osc_batch_solve_multi takes a wheel-row model (its job's wheel_dir, ABI 4) beside Go2 and
    WaLTER jobs: every job's results are bitwise those of its own call."""
    from osc_amd.solver import solve_multi_into
    wheel = _wheel()
    jobs, solo = [], []
    for key, robot, nenv, seed in (("unitree_go2", "unitree_go2", 512, 201),
                                   ("noslip", "walter_sr_wheels", 256, 202),
                                   ("walter_sr", "walter_sr", 384, 203)):
        s = solver(key)
        d = generate(robot, nenv, SEED_BASE + seed, "tumbling", "bernoulli")
        args = s.prepare(**d)
        wdt = None
        if key == "noslip":
            wdt = torch.from_numpy(wheel_directions(robot, d, wheel.dof, wheel.radius,
                                                    SEED_BASE + seed + 1)).cuda()
        o = s.alloc_outputs(nenv, want_x=True)
        jobs.append((s, o, args) + ((wdt,) if wdt is not None else ()))
        r = s.alloc_outputs(nenv, want_x=True)
        s.solve_into(r, *args, wheel_dir=wdt)
        solo.append(r)
    solve_multi_into(jobs)
    torch.cuda.synchronize()
    for (s, o, *_), r in zip(jobs, solo):
        for k in ("tau", "x", "status", "iters"):
            assert torch.equal(getattr(o, k), getattr(r, k)), (s.robot, k)


@pytest.mark.parametrize("order", [("noslip", "unitree_go2"), ("unitree_go2", "noslip"),
                                   ("noslip", "walter_sr"), ("walter_sr", "noslip")])
def test_wheel_model_in_two_job_multi(gpu, order):
    """Two jobs, one of them a wheel-row model: the two-model grid is only for
    {walter_sr, unitree_go2}, so either order runs each job as its own call -- bitwise."""
    from osc_amd.solver import solve_multi_into
    wheel = _wheel()
    robots = {"unitree_go2": "unitree_go2", "noslip": "walter_sr_wheels", "walter_sr": "walter_sr"}
    jobs, solo = [], []
    for i, key in enumerate(order):
        s = solver(key)
        robot = robots[key]
        d = generate(robot, 192 + 64 * i, SEED_BASE + 211 + i, "tumbling", "bernoulli")
        args = s.prepare(**d)
        wdt = None
        if key == "noslip":
            wdt = torch.from_numpy(wheel_directions(robot, d, wheel.dof, wheel.radius,
                                                    SEED_BASE + 221 + i)).cuda()
        n = d["M"].shape[0]
        o = s.alloc_outputs(n, want_x=True)
        jobs.append((s, o, args) + ((wdt,) if wdt is not None else ()))
        r = s.alloc_outputs(n, want_x=True)
        s.solve_into(r, *args, wheel_dir=wdt)
        solo.append(r)
    solve_multi_into(jobs)
    torch.cuda.synchronize()
    for (s, o, *_), r in zip(jobs, solo):
        assert (r.status.cpu().numpy() == 0).all(), s.robot
        for k in ("tau", "x", "status", "iters"):
            assert torch.equal(getattr(o, k), getattr(r, k)), (s.robot, k)
