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


# ---- examples/walter_sr_true_tumbling_mjjoint.cc: contact geom table and per-site targets ----

WHEEL_SITES_MUJOCO = (3, 4, 7, 8, 11, 12, 15, 16)   # :436


def contact_geom_table(geom_bodyid, site_bodyid, ids=WHEEL_SITES_MUJOCO):
    """geom -> contact-site index under the example's rule (:523-558): a contact geom counts when
    its GEOM id is in `ids` (contains(wheel_sites_mujoco, geom), :526/:538); it marks the first
    site of its body (getSiteIdsOnSameBodyAsGeom(...)[0], :106-149); the mask is the indicator of
    `ids` read as SITE ids among the marked sites (getBinaryRepresentation_std_find, :152-163)."""
    table = np.full(len(geom_bodyid), -1, dtype=np.int32)
    for g, body in enumerate(geom_bodyid):
        if g not in ids:
            continue
        on_body = [s for s, sb in enumerate(site_bodyid) if sb == body]
        if not on_body:
            continue
        if on_body[0] in ids:
            table[g] = list(ids).index(on_body[0])
    return table


TUMBLING_DEFAULTS = dict(
    shin_rot_vel=0.1 * 8.0 * 5.0, shin_kp=800.0 * 3.0, shin_kv=800.0 * 3.0,      # :694-757
    thigh_lin_vel=0.0, thigh_lin_kp=4000.0 * 0.5, thigh_lin_kv=600.0 * 0.5,     # :866-874
    thigh_height_offset=-0.025,                                                 # :897
    torso_lin_vel=0.2, torso_lin_kp=0.0, torso_lin_kv=0.0,                      # :981-1002
    torso_ang_kp=0.0, torso_ang_kv=0.0,                                         # :1013-1014
    shin_qadr=(8, 10, 12, 14))                                                  # :698-701


def tumbling_targets(qpos, qvel, site_xpos, t, t0, init_qpos, init_site_xpos, **kw):
    """One environment's (17, 6) TaskspaceTargets of the tumbling driver (:622-1019), written the
    way the example writes it, leg by leg.  The example's "last" values are the ones captured
    before its loop (:363-433) on every tick -- the in-loop updates declare shadowing locals
    (:684-687, :767-770, :926-931) -- so each velocity is (now - initial) / (t - t0)."""
    p = dict(TUMBLING_DEFAULTS, **kw)
    T = np.zeros((17, 6))
    last_time = t0
    current_time = t
    # shins, rows 1-4: angular-y
    for i, adr in enumerate(p["shin_qadr"]):
        initial_angular_position = init_qpos[adr]           # :379-397
        last_angular_position = initial_angular_position
        angular_position = qpos[adr]                        # :698-711
        angular_velocity = (angular_position - last_angular_position) / (current_time - last_time)
        angular_position_target = initial_angular_position + p["shin_rot_vel"] * current_time
        angular_velocity_target = p["shin_rot_vel"]
        angular_control = (p["shin_kp"] * (angular_position_target - angular_position) +
                           p["shin_kv"] * (angular_velocity_target - angular_velocity))
        T[1 + i] = [0, 0, 0, 0, angular_control, 0]         # :778-802
    # thighs, rows 5-8: linear-z
    for i in range(4):
        r = 5 + i
        last_linear_position = np.asarray(init_site_xpos[r])          # :423-426
        linear_position = np.asarray(site_xpos[r])                     # :878-881
        linear_velocity = (linear_position - last_linear_position) / (current_time - last_time)
        linear_position_error = ((init_site_xpos[r][2] - 0.0 + p["thigh_height_offset"]) -
                                 linear_position[2])                   # :900-903
        linear_velocity_error = p["thigh_lin_vel"] - linear_velocity[2]
        linear_control = (p["thigh_lin_kp"] * linear_position_error +
                          p["thigh_lin_kv"] * linear_velocity_error)
        T[r] = [0, 0, linear_control, 0, 0, 0]              # :943-973
    # torso, row 0
    initial_position = np.asarray(init_qpos[0:3])          # :247
    position_target = np.array([initial_position[0] + p["torso_lin_vel"] * current_time,
                                initial_position[1], initial_position[2]])
    velocity_target = np.array([p["torso_lin_vel"], 0.0, 0.0])
    body_position = np.asarray(qpos[0:3])
    conj = np.array([qpos[3], -qpos[4], -qpos[5], -qpos[6]])
    rotation_error = quat_mul([1.0, 0.0, 0.0, 0.0], conj)[1:]
    position_error = position_target - body_position
    velocity_error = velocity_target - np.asarray(qvel[0:3])
    angular_velocity_error = 0.0 - np.asarray(qvel[3:6])
    linear_control = p["torso_lin_kp"] * position_error + p["torso_lin_kv"] * velocity_error
    angular_control = p["torso_ang_kp"] * rotation_error + p["torso_ang_kv"] * angular_velocity_error
    T[0] = [linear_control[0], 0, 0, angular_control[0], angular_control[1], angular_control[2]]
    return T
