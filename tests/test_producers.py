"""Batched input producers (csrc/osc_producers.hip, include/osc_producers.h): the oracle
restatement (oracle/producers.py) against known answers on CPU, and the HIP kernels against the
oracle on the GPU (contact mask bit-exact; PD targets within 1e-13 relative: hipcc may contract
a*b + c into one fma)."""
import ctypes

import numpy as np
import pytest

from producers import contact_mask_from_contacts, pd_base_targets, quat_mul


def test_pd_targets_known_answers():
    # at rest on the reference pose: zero targets
    T = pd_base_targets(5, np.zeros(3), [1, 0, 0, 0], np.zeros(3), np.zeros(3), np.zeros(3),
                        [1, 0, 0, 0])
    assert np.all(T == 0)
    # 90 deg about z: q = (cos45, 0, 0, sin45); vec(q_id * conj(q)) = (0, 0, -sin45)
    s = np.sqrt(0.5)
    T = pd_base_targets(5, np.array([0.1, 0, 0]), [s, 0, 0, s], np.array([0, 0, 1.0]),
                        np.array([0, 2.0, 0]), np.zeros(3), [1, 0, 0, 0])
    np.testing.assert_allclose(T[0], [150 * -0.1, 0, -25.0, 0, -20.0, 50 * -s], rtol=1e-15)
    assert np.all(T[1:] == 0)
    # Hamilton product sanity: i * j = k
    np.testing.assert_array_equal(quat_mul([0, 1, 0, 0], [0, 0, 1, 0]), [0, 0, 0, 1])


def test_contact_mask_known_answers():
    g2s = np.array([-1, 0, 1, 2, 3, -1])          # geom 0 = floor, geoms 1..4 on feet 0..3
    assert list(contact_mask_from_contacts(4, 0, [], g2s)) == [0, 0, 0, 0]
    pairs = [[0, 2], [4, 0], [5, 0]]              # foot 1, foot 3 (either side), non-foot
    assert list(contact_mask_from_contacts(4, 3, pairs, g2s)) == [0, 1, 0, 1]
    assert list(contact_mask_from_contacts(4, 1, pairs, g2s)) == [0, 1, 0, 0]   # only ncon used


@pytest.mark.gpu
def test_pd_targets_gpu_vs_oracle(gpu):
    import torch
    from osc_amd import _lib
    rng = np.random.default_rng(5)
    nenv, ns = 4099, 5
    pos, lin, ang = (rng.standard_normal((nenv, 3)) for _ in range(3))
    q = rng.standard_normal((nenv, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    pref = rng.standard_normal((nenv, 3))
    qref = np.array([1.0, 0, 0, 0])
    gains = (ctypes.c_double * 4)(150.0, 25.0, 50.0, 10.0)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    d = [dev(a) for a in (pos, q, lin, ang, pref, qref)]
    out = torch.full((nenv, ns, 6), np.nan, dtype=torch.float64, device=gpu)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = _lib.lib().osc_pd_base_targets(nenv, ns, p(d[0]), p(d[1]), p(d[2]), p(d[3]), p(d[4]), 1,
                                        p(d[5]), 0, gains, p(out), None)
    assert rc == 0
    got = out.cpu().numpy()
    for e in list(range(64)) + [nenv - 1]:
        ref = pd_base_targets(ns, pos[e], q[e], lin[e], ang[e], pref[e], qref)
        np.testing.assert_allclose(got[e], ref, rtol=1e-13, atol=1e-13)
    assert np.all(got[:, 1:] == 0)


@pytest.mark.gpu
def test_contact_mask_gpu_vs_oracle(gpu):
    import torch
    from osc_amd import _lib
    rng = np.random.default_rng(6)
    nenv, nc, max_con, ngeom = 5003, 8, 12, 30
    g2s = np.full(ngeom, -1, dtype=np.int32)
    g2s[rng.choice(ngeom, nc, replace=False)] = np.arange(nc)
    ncon = rng.integers(-1, max_con + 3, nenv).astype(np.int32)      # includes out-of-range
    pairs = rng.integers(-1, ngeom + 2, (nenv, max_con, 2)).astype(np.int32)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    d_ncon, d_pairs, d_g2s = dev(ncon), dev(pairs), dev(g2s)
    out = torch.full((nenv, nc), -7.0, dtype=torch.float64, device=gpu)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    rc = _lib.lib().osc_contact_mask_from_contacts(nenv, nc, max_con, p(d_ncon), p(d_pairs),
                                                   ngeom, p(d_g2s), p(out), None)
    assert rc == 0
    got = out.cpu().numpy()
    ref = np.stack([contact_mask_from_contacts(nc, min(max(ncon[e], 0), max_con), pairs[e], g2s)
                    for e in range(nenv)])
    np.testing.assert_array_equal(got, ref)


# ---- tumbling driver (examples/walter_sr_true_tumbling_mjjoint.cc) ----

from producers import TUMBLING_DEFAULTS, WHEEL_SITES_MUJOCO, contact_geom_table, tumbling_targets


def _tumbling_state(rng, nq=15, nv=14):
    q0 = np.zeros(nq)
    q0[0:3] = rng.standard_normal(3)
    qq = rng.standard_normal(4)
    q0[3:7] = qq / np.linalg.norm(qq)
    q0[7:] = rng.uniform(-1, 1, nq - 7)
    x0 = rng.standard_normal((17, 3))
    q = q0 + 0.05 * rng.standard_normal(nq)
    q[3:7] /= np.linalg.norm(q[3:7])
    x = x0 + 0.01 * rng.standard_normal((17, 3))
    v = rng.standard_normal(nv)
    return q, v, x, q0, x0


def test_tumbling_targets_known_answers():
    rng = np.random.default_rng(3)
    q, v, x, q0, x0 = _tumbling_state(rng)
    t0, t = 0.5, 0.75
    T = tumbling_targets(q, v, x, t, t0, q0, x0)
    p = TUMBLING_DEFAULTS
    # shin tl: angle qpos[8] (jnt_qposadr[2]); target uses absolute time, velocity vs. initial
    th, th0 = q[8], q0[8]
    w = (th - th0) / (t - t0)
    assert T[1, 4] == p["shin_kp"] * (th0 + 4.0 * t - th) + p["shin_kv"] * (4.0 - w)
    assert np.count_nonzero(T[1:5, [0, 1, 2, 3, 5]]) == 0
    # thigh hl (row 7): linear-z only
    z, z0 = x[7, 2], x0[7, 2]
    assert T[7, 2] == 2000.0 * ((z0 - 0.0 - 0.025) - z) + 300.0 * (0.0 - (z - z0) / (t - t0))
    assert np.count_nonzero(T[5:9, [0, 1, 3, 4, 5]]) == 0
    # torso gains are 0 in the example; wheels untouched
    assert np.all(T[0] == 0) and np.all(T[9:] == 0)
    # with torso gains: x-only linear command, angular = kp vec(conj q) + kv (0 - w)
    T2 = tumbling_targets(q, v, x, t, t0, q0, x0, torso_lin_kp=2.0, torso_ang_kp=3.0,
                          torso_ang_kv=0.5)
    assert T2[0, 0] == 2.0 * (q0[0] + 0.2 * t - q[0]) + 0.0 * (0.2 - v[0])
    assert T2[0, 1] == 0 and T2[0, 2] == 0
    np.testing.assert_allclose(T2[0, 3:], 3.0 * -q[4:7] + 0.5 * (0.0 - v[3:6]), rtol=1e-15)
    # first pass of the example (t == t0): non-finite velocities, as the reference
    with np.errstate(divide="ignore", invalid="ignore"):
        assert not np.all(np.isfinite(tumbling_targets(q0, v, x0, t0, t0, q0, x0)))


def test_contact_geom_table_reference_rule():
    """The list {3, 4, 7, 8, 11, 12, 15, 16} read as GEOM ids, then as SITE ids (:436, :523-558).
    A made-up model: 20 geoms, 17 sites; site s on body site_body[s]."""
    site_body = np.array([1, 2, 3, 3, 4, 5, 6, 6, 7, 8, 9, 9, 10, 11, 12, 12, 13])
    geom_body = np.array([0, 1, 2, 3, 3, 4, 5, 6, 6, 7, 8, 9, 9, 10, 11, 12, 12, 13, 2, 6])
    table = contact_geom_table(geom_body, site_body)
    for g in range(len(geom_body)):
        if g not in WHEEL_SITES_MUJOCO:
            assert table[g] == -1
    # geom 3 (listed) is on body 3, whose first site is 2 -> site 2 is not listed -> no mark
    assert table[3] == -1
    # geom 7 (listed) on body 6: first site 6 -> not listed; geom 8 likewise
    assert table[7] == -1 and table[8] == -1
    # geom 4 (listed) on body 3 -> site 2 -> unlisted; geom 11 on body 9 -> first site 10, unlisted
    assert table[4] == -1 and table[11] == -1
    # geom 12 on body 9 -> site 10 -> no; geom 15 on body 12 -> first site 14 -> no;
    # geom 16 on body 12 -> site 14 -> no: in this model only lists whose site ids coincide mark
    site_body2 = np.arange(17)          # site s on body s
    geom_body2 = np.arange(20)          # geom g on body g
    t2 = contact_geom_table(geom_body2, site_body2)
    assert [t2[g] for g in WHEEL_SITES_MUJOCO] == list(range(8))
    assert sum(t2 >= 0) == 8
    # the library builds the same table
    from osc_amd.producers import contact_geom_table as native
    for gb, sb in ((geom_body, site_body), (geom_body2, site_body2)):
        np.testing.assert_array_equal(native(gb, sb, WHEEL_SITES_MUJOCO),
                                      contact_geom_table(gb, sb))


@pytest.mark.gpu
def test_tumbling_targets_gpu_vs_oracle(gpu):
    import torch
    from osc_amd.producers import tumbling_params, tumbling_targets_into
    rng = np.random.default_rng(9)
    nenv = 2051
    states = [_tumbling_state(rng) for _ in range(nenv)]
    t0 = rng.uniform(0, 1, nenv)
    t = t0 + rng.uniform(0.002, 0.5, nenv)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    q, v, x, q0, x0 = (dev(np.stack([s[i] for s in states])) for i in range(5))
    out = torch.full((nenv, 17, 6), np.nan, dtype=torch.float64, device=gpu)
    params = dict(torso_lin_kp=2.0, torso_lin_kv=0.3, torso_ang_kp=3.0, torso_ang_kv=0.5)
    tumbling_targets_into(out, q, v, x, dev(t), dev(t0), q0, x0, tumbling_params(**params))
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for e in list(range(48)) + [nenv - 1]:
        s = states[e]
        ref = tumbling_targets(s[0], s[1], s[2], t[e], t0[e], s[3], s[4], **params)
        np.testing.assert_allclose(got[e], ref, rtol=1e-13, atol=1e-12)
