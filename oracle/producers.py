"""CPU oracle for the batched input producers (csrc/osc_producers.hip).

TEST INFRASTRUCTURE ONLY (tests/ may import it, the product never does).  Restates, per
environment, the example drivers' per-tick logic (paths relative to the reference root):
  * pd_base_targets: examples/standing.cc:143-155 -- TaskspaceTargets::Zero(), then row 0 =
    [150 (p0 - p) + 25 (0 - v), 50 vec(q_id * conj(q)) + 10 (0 - w)] (Eigen Hamilton product,
    quaternions (w, x, y, z)); the gains and the reference pose are parameters here.
  * contact_mask_from_contacts: examples/walter_sr_true_tumbling_mjjoint.cc:473-558 -- for
    every contact whose geom[1] (:523-532) or geom[0] (:534-543) lies on a contact-site body,
    that site is marked; the mask is the 0/1 indicator over the contact sites (:547-558).
Parity unpinned against the examples themselves (they need MuJoCo); pinned by known answers
in tests/test_producers.py.
"""
import numpy as np


def quat_mul(a, b):
    """Hamilton product of (w, x, y, z) quaternions (Eigen::Quaternion operator*)."""
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz,
                     aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw])


def pd_base_targets(ns, pos, quat, lin_vel, ang_vel, pos_ref, quat_ref,
                    gains=(150.0, 25.0, 50.0, 10.0)):
    """One environment: (ns, 6) targets."""
    kp_l, kd_l, kp_a, kd_a = gains
    T = np.zeros((ns, 6))
    conj = np.array([quat[0], -quat[1], -quat[2], -quat[3]])
    rot_err = quat_mul(np.asarray(quat_ref, float), conj)[1:]
    T[0, 0:3] = kp_l * (np.asarray(pos_ref) - pos) + kd_l * (0.0 - np.asarray(lin_vel))
    T[0, 3:6] = kp_a * rot_err + kd_a * (0.0 - np.asarray(ang_vel))
    return T


def contact_mask_from_contacts(nc, ncon, geom_pairs, geom_to_site):
    """One environment: contact list (ncon pairs of geom ids) -> (nc,) 0/1 mask."""
    mask = np.zeros(nc)
    for c in range(max(0, min(int(ncon), len(geom_pairs)))):
        for g in geom_pairs[c]:
            if 0 <= g < len(geom_to_site) and geom_to_site[g] >= 0:
                mask[geom_to_site[g]] = 1.0
    return mask
