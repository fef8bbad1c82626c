"""CPU tests of the oracle (oracle/osc_qp.py + oracle/qp_exact.py) against the golden fixtures
and analytic known-answer cases.  No GPU, no product code on the solve path.

The reference holds no tests or golden vectors: the fixtures are oracle-made and
parity is unpinned against the reference's own outputs; each case here checks a property the
reference's QP definition implies (file:line cited per test).
"""
import glob
import os

import numpy as np
import pytest

from osc_qp import (BIG_NUMBER, OSQP_INFTY, b_matrix, build_qp, contact_jacobian, load_model,
                    task_targets_vector, task_weights, torque)
from qp_exact import certified, kkt_certificate, solve_exact

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def _load(path):
    z = np.load(path)          # allow_pickle=False (default): data only
    return {k: z[k] for k in z.files}


def _args(g, e):
    return [g[k][e] for k in ("M", "C", "J", "b", "T", "mask")]


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_golden_resolves_and_certifies(path):
    """Oracle re-solve reproduces every committed golden solution; KKT certificate <= 1e-9."""
    g = _load(path)
    model = load_model(str(g["robot"]))
    for e in range(g["M"].shape[0]):
        qp = build_qp(model, *_args(g, e))
        sol = solve_exact(model, qp, *_args(g, e)[:3])
        assert certified(sol.cert), sol.cert
        np.testing.assert_allclose(sol.x, g["x"][e], rtol=0, atol=1e-9 * (1 + np.abs(g["x"][e]).max()))
        np.testing.assert_array_equal(torque(model, g["x"][e]), g["tau"][e])
        assert certified(kkt_certificate(qp, g["x"][e], g["y"][e]))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_golden_dynamics_and_bounds(path):
    """x satisfies M dv + C - B u - Jc z = 0 (autogen.py:87), the friction pyramid
    (autogen.py:112-117), torque limits (osc.h:285-296) and masked force bounds (osc.h:492-497)."""
    g = _load(path)
    model = load_model(str(g["robot"]))
    nv, nu, nz = model.nv, model.nu, model.nz
    for e in range(g["M"].shape[0]):
        x = g["x"][e]
        dv, u, z = x[:nv], x[nv:nv + nu], x[nv + nu:]
        Jc = contact_jacobian(model, g["J"][e])
        res = g["M"][e] @ dv + g["C"][e] - b_matrix(model) @ u - Jc @ z
        assert np.abs(res).max() <= 1e-9 * (1 + np.abs(g["C"][e]).max())
        assert np.all(u <= model.u_ub + 1e-9) and np.all(u >= model.u_lb - 1e-9)
        for k in range(model.nc):
            fx, fy, fz = z[3 * k:3 * k + 3]
            if g["mask"][e][k] == 0:
                assert fx == 0 and fy == 0 and fz == 0          # pinned by l = u = 0
            else:
                assert abs(fx) + abs(fy) <= model.mu * fz + 1e-9
                assert -1e-9 <= fz <= BIG_NUMBER + 1e-9


def test_qp_structure_matches_reference():
    """Closed forms of the CasADi outputs (autogen.py:274-319) and OSQP stacking (osc.h:483-497)."""
    model = load_model("unitree_go2")
    g = _load(os.path.join(os.path.dirname(__file__), "golden", "go2_tumbling_mask.npz"))
    M, C, J, b, T, mask = _args(g, 0)
    qp = build_qp(model, M, C, J, b, T, mask)
    nv, nu, nz, n = model.nv, model.nu, model.nz, model.n
    assert (n, qp.A.shape) == (42, (76, 42))
    W = task_weights(model)
    np.testing.assert_allclose(qp.H[:nv, :nv], 2 * J.T @ np.diag(W) @ J + 2e-4 * np.eye(nv))
    np.testing.assert_array_equal(np.diag(qp.H)[nv:nv + nu], 2 * (1e-4 + 1e-4))
    np.testing.assert_array_equal(np.diag(qp.H)[nv + nu:], 2 * 1e-4)
    assert np.count_nonzero(qp.H[:nv, nv:]) == 0
    np.testing.assert_allclose(qp.f[:nv], 2 * J.T @ (W * (b - task_targets_vector(model, T))))
    np.testing.assert_array_equal(qp.Aeq[:, :nv], M)
    np.testing.assert_array_equal(qp.Aeq[:, nv:nv + nu], -b_matrix(model))
    np.testing.assert_array_equal(qp.Aeq[:, nv + nu:], -J[3 * model.ns - nz:3 * model.ns].T)
    np.testing.assert_array_equal(qp.beq, -C)
    np.testing.assert_array_equal(qp.l[:nv], qp.u[:nv])
    assert np.all(qp.l[nv:nv + 4 * model.nc] == -OSQP_INFTY)
    np.testing.assert_array_equal(qp.u[nv:nv + 4 * model.nc], 0.0)
    off = nv + 4 * model.nc + nv
    np.testing.assert_array_equal(qp.u[off:off + nu], model.u_ub)
    for k in range(model.nc):
        lo, hi = qp.l[off + nu + 3 * k:off + nu + 3 * k + 3], qp.u[off + nu + 3 * k:off + nu + 3 * k + 3]
        if mask[k] == 0:
            assert np.all(lo == 0) and np.all(hi == 0)
        else:
            assert list(lo) == [-OSQP_INFTY, -OSQP_INFTY, 0.0]
            assert list(hi) == [OSQP_INFTY, OSQP_INFTY, BIG_NUMBER]


def test_known_answer_equality_only():
    """With every contact masked and WaLTER's +-1000 N m limits slack, only the dynamics rows
    bind: the optimum is the single KKT solve  [H Aeq'; Aeq 0] [x; nu] = [-f; beq]  with z = 0."""
    g = _load(os.path.join(os.path.dirname(__file__), "golden", "walter_no_contact.npz"))
    model = load_model("walter_sr")
    nv, nu, nz, n = model.nv, model.nu, model.nz, model.n
    for e in range(g["M"].shape[0]):
        qp = build_qp(model, *_args(g, e))
        Aeq = np.vstack([qp.Aeq, np.hstack([np.zeros((nz, nv + nu)), np.eye(nz)])])
        beq = np.concatenate([qp.beq, np.zeros(nz)])
        k = Aeq.shape[0]
        K = np.block([[qp.H, Aeq.T], [Aeq, np.zeros((k, k))]])
        x = np.linalg.solve(K, np.concatenate([-qp.f, beq]))[:n]
        assert np.all(np.abs(x[nv:nv + nu]) < 1000), "limits must be slack for this check"
        np.testing.assert_allclose(g["x"][e], x, rtol=0, atol=1e-9 * (1 + np.abs(x).max()))


def test_weights_follow_yaml_site_order():
    """Weight keys map to sites in autogen.py's split order (go2 autogen.py:160-219)."""
    m = load_model("unitree_go2")
    np.testing.assert_array_equal(m.w_pos, [100, 10, 10, 10, 10])
    w = load_model("walter_sr")
    assert list(w.w_rot[1:5]) == [300.0] * 4 and list(w.w_pos[5:9]) == [100.0] * 4
    ww = load_model("walter_sr_wheels")
    assert ww.w_pos[5] == 800.0 and ww.w_rot[0] == 100.0


def test_reference_port_converges_to_exact_optimum():
    """oracle/osc_ref_port.c (reference CPU path: CasADi-equivalent assembly + OSQP 0.6.3 ADMM)
    approaches the exact oracle optimum as its tolerance tightens -- a cross-check of both
    restatements (Go2: ADMM converges quickly in every direction)."""
    from ref_port import RefPort
    g = _load(os.path.join(os.path.dirname(__file__), "golden", "go2_standing.npz"))
    for e in range(4):
        port = RefPort("unitree_go2")
        port.set_tolerances(1e-10, 1e-10, 200000)
        tau, it = port.step(*_args(g, e))
        ref = g["tau"][e]
        assert np.abs(tau - ref).max() / max(np.abs(ref).max(), 1.0) < 1e-6, (e, it)


def test_reference_port_default_settings_converge():
    """With OSQP's defaults (eps 1e-3, check every 25 iterations) the restated reference path
    terminates well before max_iter (cold start, as on the reference's first tick) and lands
    within ~1e-1 normwise of the exact optimum on Go2 -- the reference's own accuracy level."""
    from ref_port import RefPort
    g = _load(os.path.join(os.path.dirname(__file__), "golden", "go2_tumbling_mask.npz"))
    for e in range(g["M"].shape[0]):
        port = RefPort("unitree_go2")
        tau, it = port.step(*_args(g, e))
        assert 0 < it < 4000
        ref = g["tau"][e]
        assert np.abs(tau - ref).max() / max(np.abs(ref).max(), 1.0) < 0.2


@pytest.mark.parametrize("robot", ["unitree_go2", "walter_sr", "walter_sr_wheels"])
def test_closed_form_equals_literal_autogen_objective(robot):
    """build_qp's H and f against the objective written term by named term as autogen.py writes
    it (oracle/autogen_literal.py), with the reference's own weights file when it is present:
    the literal objective is a quadratic, so its Hessian and gradient at x = 0 follow exactly
    from values at 0, +-e_i and e_i + e_j."""
    import autogen_literal as lit
    from osc_amd.robots import config_path
    from osc_amd.synth import SEED_BASE, generate
    ref_yaml = os.path.join("/root/reference/config", robot, f"{robot}_config.yaml")
    yaml_path = ref_yaml if os.path.exists(ref_yaml) else config_path(robot)
    weights = lit.weights_config(yaml_path)
    model = load_model(robot)
    d = generate(robot, 2, SEED_BASE + 61, "tumbling", "bernoulli")
    for e in range(2):
        M, C, J, b, T, mask = (d[k][e] for k in ("M", "C", "J", "b", "T", "mask"))
        qp = build_qp(model, M, C, J, b, T, mask)
        H, g = lit.hessian_gradient_at_zero(
            lambda x: lit.objective(robot, weights, x, T, J, b, model.nv, model.nu), model.n)
        scale = np.abs(qp.H).max()
        assert np.abs(H - qp.H).max() <= 1e-9 * scale, np.abs(H - qp.H).max() / scale
        assert np.abs(g - qp.f).max() <= 1e-9 * max(np.abs(qp.f).max(), 1.0)


def _wheel_setup(robot="walter_sr_wheels"):
    from osc_qp import WheelRows
    from osc_amd.synth import WALTER_WHEEL_DOFS, WHEEL_RADIUS
    model = load_model(robot)
    wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(model.nc, WHEEL_RADIUS))
    return model, wheel


def test_wheel_rows_equal_literal_design():
    """The no-slip rows of osc_qp.wheel_rows against the constraints written exactly as the
    commented design in walter_sr_wheels/autogen/autogen.py:185-240 writes them (an affine map
    of the design vector: its jacobian and value at x = 0 give Aeq and -beq, the CasADi
    convention of the dynamics rows, autogen.py:274-287).  The Jacobian-dot bias the design
    forms from J_dot_wheel_p @ joint_velocities_current is the contact rows of b."""
    import autogen_literal as lit
    from osc_amd.synth import SEED_BASE, generate
    model, wheel = _wheel_setup()
    nc, nv, r0 = model.nc, model.nv, 3 * model.ns - model.nz
    rng = np.random.default_rng(SEED_BASE + 71)
    d = generate(model.name, 2, SEED_BASE + 71, "tumbling", "ones")
    for e in range(2):
        M, C, J, b, T, mask = (d[k][e].copy() for k in ("M", "C", "J", "b", "T", "mask"))
        Jdot = rng.standard_normal((3 * nc, nv))
        qd = rng.standard_normal(nv)
        b[r0:r0 + 3 * nc] = Jdot @ qd
        wd = rng.standard_normal((nc, 6))
        qp = build_qp(model, M, C, J, b, T, mask, wheel, wd)
        Jw, f0 = lit.jacobian_value_at_zero(
            lambda x: lit.wheel_constraints(x, J[r0:r0 + 3 * nc], Jdot, qd, wheel.radius, wd,
                                            wheel.dof, nv), model.n)
        assert np.abs(qp.Aw - Jw).max() <= 1e-12 * np.abs(Jw).max()
        assert np.abs(qp.bw + f0).max() <= 1e-12 * max(np.abs(f0).max(), 1.0)
        # stacked after the dynamics rows, as equality rows (autogen.py:236-239)
        assert np.array_equal(qp.A[nv:nv + 2 * nc], qp.Aw)
        assert np.array_equal(qp.l[nv:nv + 2 * nc], qp.bw) and np.array_equal(qp.u[nv:nv + 2 * nc], qp.bw)
    # a wheel off the ground (mask 0) contributes the trivial rows 0 = 0
    mask = np.ones(nc)
    mask[[1, 6]] = 0.0
    qp = build_qp(model, M, C, J, b, T, mask, wheel, wd)
    assert not qp.Aw[[2, 3, 12, 13]].any() and not qp.bw[[2, 3, 12, 13]].any()


def test_wheel_qp_exact_optimum_certified():
    """With the no-slip rows the oracle's exact solve (phase-1 LP start, active set, KKT
    refinement) certifies at 1e-9 and the rows hold at the optimum; the optimum moves away from
    the wheel-free one (the rows bind)."""
    from osc_amd.synth import SEED_BASE, generate, wheel_directions
    model, wheel = _wheel_setup()
    d = generate(model.name, 3, SEED_BASE + 72, "tumbling", "bernoulli")
    wd = wheel_directions(model.name, d, wheel.dof, wheel.radius, SEED_BASE + 73)
    for e in range(3):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *args, wheel, wd[e])
        sol = solve_exact(model, qp, *args[:3])
        assert certified(sol.cert), sol.cert
        assert np.abs(qp.Aw @ sol.x - qp.bw).max() <= 1e-9 * (1 + np.abs(qp.bw).max())
        free = solve_exact(model, build_qp(model, *args), *args[:3])
        assert np.abs(torque(model, free.x) - torque(model, sol.x)).max() > 1e-3


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p)[:-4] for p in GOLDEN])
def test_dual_active_set_agrees_with_primal(path):
    """The oracle's two exact methods -- the primal active-set method and Goldfarb-Idnani's dual
    one (qp_exact._dual_active_set) -- share no iteration logic; on every golden env they return
    the same optimum to 1e-12 and both certify."""
    g = _load(path)
    model = load_model(str(g["robot"]))
    wheel = None
    if "wheel_dir" in g:
        model, wheel = _wheel_setup()
    for e in range(g["M"].shape[0]):
        args = _args(g, e)
        qp = build_qp(model, *args, *((wheel, g["wheel_dir"][e]) if wheel is not None else ()))
        a = solve_exact(model, qp, *args[:3], method="primal")
        b = solve_exact(model, qp, *args[:3], method="dual")
        assert certified(b.cert), b.cert
        assert np.abs(a.x - b.x).max() <= 1e-12 * (1 + np.abs(a.x).max())


def test_dual_active_set_takes_degenerate_wheel_envs():
    """Wheel-row tumbling envs on which the primal active-set method cycles (Bland's rule does not
    resolve every dependent working set: 'active set did not converge') or ends on a wrong,
    nearly dependent working set (not certified): the dual method certifies each at 1e-9 and
    solve_exact ("auto") returns that solution -- the oracle now accepts every env of the wheel census (4 seeds x 2,048 envs,
    DESIGN.md §2)."""
    from osc_amd.synth import SEED_BASE, generate, wheel_directions
    model, wheel = _wheel_setup()
    d = generate(model.name, 2048, SEED_BASE + 82, "tumbling", "bernoulli")   # (the census batch)
    wd = wheel_directions(model.name, d, wheel.dof, wheel.radius, SEED_BASE + 83)
    for e in (178, 665, 1436):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *args, wheel, wd[e])
        try:   # (665: a nearly dependent primal working set, wrong -- not certified)
            bad = solve_exact(model, qp, *args[:3], method="primal")
            assert not certified(bad.cert)
        except RuntimeError:
            pass
        sol = solve_exact(model, qp, *args[:3])
        assert certified(sol.cert), (e, sol.cert)
        assert np.abs(qp.Aw @ sol.x - qp.bw).max() <= 1e-9 * (1 + np.abs(qp.bw).max())


def test_parallel_pool_equals_serial_oracle():
    """oracle/parallel.solve_batch (the process pool the GPU parity tests use to check every env
    of a 4,096-env batch) returns bitwise the serial oracle's optimum, env by env, in env order."""
    from osc_amd.synth import generate
    from parallel import solve_batch
    model = load_model("unitree_go2")
    d = generate("unitree_go2", 70, 4242, "tumbling", "bernoulli")
    xs, cert = solve_batch("unitree_go2", d["M"], d["C"], d["J"], d["b"], d["T"], d["mask"],
                           envs=np.arange(3, 70), workers=2)
    assert xs.shape == (67, model.n) and (cert <= 1e-8).all()
    for e in (3, 40, 66, 69):
        a = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        ref = solve_exact(model, build_qp(model, *a), *a[:3]).x
        assert np.array_equal(xs[e - 3], ref)


def test_seeded_oracle_equals_full_oracle():
    """oracle/parallel.seeded_batch (every env of a 65,536-env batch against the exact optimum,
    the working set seeded from the GPU's duals and certified by the oracle's KKT test) returns
    the full oracle's optimum: seeded with the exact duals every env certifies and agrees to 1e-12;
    seeded with nothing (y = 0) the certificate refuses the unconstrained face wherever a row is
    active, and the full oracle answers."""
    from osc_amd.synth import generate
    from parallel import seeded_batch
    model = load_model("unitree_go2")
    d = generate("unitree_go2", 24, 4343, "tumbling", "bernoulli")
    a = [d[k] for k in ("M", "C", "J", "b", "T", "mask")]
    ref = [solve_exact(model, build_qp(model, *[v[e] for v in a]), *[v[e] for v in a[:3]])
           for e in range(24)]
    y = np.array([r.y for r in ref])
    xs, seeded = seeded_batch("unitree_go2", *a, y, workers=2)
    assert seeded.all()
    xr = np.array([r.x for r in ref])
    assert np.abs(xs - xr).max() <= 1e-12 * max(1.0, np.abs(xr).max())
    xs0, seeded0 = seeded_batch("unitree_go2", *a, np.zeros_like(y), workers=2)
    assert not seeded0.any()
    assert np.array_equal(xs0, xr)
