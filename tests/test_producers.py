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
