"""The whole tumbling control tick as one device pipeline (bench.py tumbling_pipeline; SURVEY.md
§8(f) rows 1 + 3): kinematics -> tumbling targets -> contact mask -> solve.  Each stage's output
is checked against its oracle on the same inputs, and the torques against the oracle chain
(kinematics oracle -> targets oracle -> mask oracle -> reference QP -> exact optimum)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import kinematics as kin
from osc_qp import build_qp, load_model, torque
from producers import WHEEL_SITES_MUJOCO, contact_geom_table, contact_mask_from_contacts, \
    tumbling_targets
from qp_exact import solve_exact

pytestmark = pytest.mark.gpu


def test_tumbling_tick_pipeline_vs_oracle(gpu):
    from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
    from osc_amd.producers import contact_mask_into, tumbling_targets_into
    from osc_amd.producers import contact_geom_table as native_table
    from osc_amd.solver import OSCBatchSolver
    tree = load_tree("walter_sr")
    nenv = 70
    q0, v0 = random_states(tree, nenv, 77, joint_range=0.5)
    rng = np.random.default_rng(78)
    q = q0 + 0.02 * rng.standard_normal(q0.shape)
    q[:, 3:7] /= np.linalg.norm(q[:, 3:7], axis=1, keepdims=True)
    q[:, 0:3] = 0.0
    v = v0 * (1 + 0.01 * rng.standard_normal(v0.shape))
    t0, t = np.zeros(nenv), np.full(nenv, 0.004)
    geom_body, site_body = np.arange(20), np.arange(17)
    table = native_table(geom_body, site_body, WHEEL_SITES_MUJOCO)
    np.testing.assert_array_equal(table, contact_geom_table(geom_body, site_body))
    max_con = 6
    ncon = rng.integers(0, max_con + 1, nenv).astype(np.int32)
    pairs = np.stack([np.zeros((nenv, max_con), np.int32),
                      rng.integers(0, 20, (nenv, max_con)).astype(np.int32)], axis=2)

    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    kb = KinematicsBatch(tree=tree)
    init = kb.compute(d(q0), d(v0), want_sites=True)
    ko = kb.compute(d(q), d(v), want_sites=True)
    T = torch.empty((nenv, 17, 6), dtype=torch.float64, device=gpu)
    mask = torch.empty((nenv, 8), dtype=torch.float64, device=gpu)
    tumbling_targets_into(T, d(q), d(v), ko.site_xpos, d(t), d(t0), d(q0), init.site_xpos)
    contact_mask_into(mask, d(ncon), d(pairs), d(table))
    solver = OSCBatchSolver("walter_sr")
    out = solver.alloc_outputs(nenv)
    solver.solve_into(out, ko.M, ko.C, ko.J, ko.b, T, mask)
    torch.cuda.synchronize()
    Tg, mg, tau = T.cpu().numpy(), mask.cpu().numpy(), out.tau.cpu().numpy()
    assert (out.status.cpu().numpy() == 0).all()
    km = kin.KinModel(tree)
    model = load_model("walter_sr")
    for e in range(0, nenv, 7):
        M, C, J, b = kin.kinematics(km, q[e], v[e])
        X = kin.site_positions(km, q[e])
        X0 = kin.site_positions(km, q0[e])
        Tr = tumbling_targets(q[e], v[e], X, t[e], t0[e], q0[e], X0)
        # targets: site positions agree to 1e-12, amplified by the finite-difference gain
        # kv / dt = 300 / 0.004 on the thigh rows
        np.testing.assert_allclose(Tg[e], Tr, rtol=1e-8, atol=1e-7)
        mr = contact_mask_from_contacts(8, ncon[e], pairs[e], table)
        np.testing.assert_array_equal(mg[e], mr)
        ref = torque(model, solve_exact(model, build_qp(model, M, C, J, b, Tg[e], mr),
                                        M, C, J).x)
        assert np.abs(tau[e] - ref).max() <= 1e-5 * max(np.abs(ref).max(), 1.0)
