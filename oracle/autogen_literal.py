"""CPU oracle, literal form of the reference's QP objective -- TEST INFRASTRUCTURE ONLY (see
osc_qp.py).  osc_qp.build_qp states H and f in closed form (2 [J e]' W [J e] + ...); this module
instead evaluates the objective value the way autogen.py WRITES it, term by named term, so a
test can recover its Hessian and gradient at x = 0 by exact quadratic identities and compare
them with build_qp's H and f (tests/test_oracle.py).

Followed line by line (paths relative to /root/reference/operational-space-control):
  unitree_go2/autogen/autogen.py:131-238  (objective, _objective_tracking, _objective_regularization)
  walter_sr/autogen/autogen.py:135-345    (same structure, 17 named sites)
  walter_sr_wheels/autogen/autogen.py     (same names as walter_sr)
  * ddx_task = J_task @ dv + task_bias; vertsplit_n(ddx_task, 2) -> (p, r); each vertsplit_n(., ns)
    into the named per-site 3-vectors, in the order the autogen unpacks them;
  * desired_task_ddx (ns x 6): horzsplit_n(., 2) -> (p, r) columns; vertsplit_n(., ns) rows, .T;
  * term '<name>_translational_tracking' = sumsqr(ddx_<name>_p - desired_<name>_p), likewise
    rotational; 'torque' = sumsqr(u); 'regularization' = sumsqr(q) (the whole design vector);
  * objective = sum over terms of term * weights_config[key].
  walter_sr_wheels/autogen/autogen.py:128-240 (the commented-out no-slip design) for
  wheel_constraints(), with the wheel joint -> dof lookup of :64-94 passed in as
  wheel_joint_ids_in_nv.
"""
from __future__ import annotations

import numpy as np
import yaml

# the unpacking order of each autogen's vertsplit_n calls
SITE_NAMES = {
    "unitree_go2": ["base", "fr", "fl", "hr", "hl"],                          # G :160-161
    "walter_sr": ["torso", "tls", "trs", "hls", "hrs", "tlh", "trh", "hlh", "hrh",
                  "tlf", "tlr", "trf", "trr", "hlf", "hlr", "hrf", "hrr"],     # W :167-168
}
SITE_NAMES["walter_sr_wheels"] = SITE_NAMES["walter_sr"]


def weights_config(yaml_path: str) -> dict:
    with open(yaml_path) as fh:
        return {k: float(v) for k, v in yaml.safe_load(fh)["weights_config"].items()}


def sumsqr(v) -> float:
    v = np.asarray(v, dtype=np.float64).ravel()
    return float(v @ v)


def objective(robot: str, weights: dict, q, desired_task_ddx, J_task, task_bias, nv: int,
              nu: int) -> float:
    names = SITE_NAMES[robot]
    ns = len(names)
    q = np.asarray(q, dtype=np.float64)
    dv, u = q[:nv], q[nv:nv + nu]
    ddx_task = np.asarray(J_task) @ dv + np.asarray(task_bias)
    ddx_task_p, ddx_task_r = np.split(ddx_task, 2)
    ddx_p = dict(zip(names, np.split(ddx_task_p, ns)))
    ddx_r = dict(zip(names, np.split(ddx_task_r, ns)))
    desired_task_p, desired_task_r = np.hsplit(np.asarray(desired_task_ddx, dtype=np.float64), 2)
    desired_p = dict(zip(names, (x.T.ravel() for x in np.vsplit(desired_task_p, ns))))
    desired_r = dict(zip(names, (x.T.ravel() for x in np.vsplit(desired_task_r, ns))))
    terms = {}
    for name in names:
        terms[f"{name}_translational_tracking"] = sumsqr(ddx_p[name] - desired_p[name])
        terms[f"{name}_rotational_tracking"] = sumsqr(ddx_r[name] - desired_r[name])
    terms["torque"] = sumsqr(u)
    terms["regularization"] = sumsqr(q)
    return sum(v * weights[k] for k, v in terms.items())


def hessian_gradient_at_zero(fun, n: int):
    """Exact for a quadratic f: H_ij = f(e_i + e_j) - f(e_i) - f(e_j) + f(0),
    g_i = (f(e_i) - f(-e_i)) / 2 (the gradient at 0, CasADi's `gradient` output of hessian())."""
    E = np.eye(n)
    f0 = fun(np.zeros(n))
    fi = np.array([fun(E[i]) for i in range(n)])
    fm = np.array([fun(-E[i]) for i in range(n)])
    H = np.empty((n, n))
    for i in range(n):
        for j in range(i, n):
            H[i, j] = H[j, i] = (fun(E[i] + E[j]) - fi[i] - fi[j] + f0) if i != j else \
                fi[i] + fm[i] - 2.0 * f0
    return H, (fi - fm) / 2.0


def wheel_constraints(q, J_wheel_p, J_dot_wheel_p, joint_velocities_current, wheel_radii,
                      wheel_directions, wheel_joint_ids_in_nv, nv: int):
    """The no-slip equality constraints exactly as walter_sr_wheels/autogen/autogen.py:185-240
    writes them (commented out upstream): per wheel i, contact_lin_accel_i = J_p_i @ dv +
    J_dot_p_i @ joint_velocities_current (:216); longitudinal_slip = dot(contact_lin_accel_i,
    d_roll_i) - r_wheel * ddq_k (:226); lateral_slip = dot(contact_lin_accel_i, d_lat_i) (:230);
    appended in that order (:227, :231).  (A wheel without a joint -- index -1 -- has no ddq_k
    term: the extension osc_qp.WheelRows allows.)"""
    q = np.asarray(q, dtype=np.float64)
    dv = q[:nv]
    num_wheels = len(wheel_radii)
    wheel_constraints = []
    for i in range(num_wheels):
        J_p_i = np.asarray(J_wheel_p)[3 * i:3 * (i + 1), :]
        J_dot_p_i = np.asarray(J_dot_wheel_p)[3 * i:3 * (i + 1), :]
        wheel_jnt_dof_idx = wheel_joint_ids_in_nv[i]
        ddq_k = dv[wheel_jnt_dof_idx] if wheel_jnt_dof_idx >= 0 else 0.0
        r_wheel = wheel_radii[i]
        contact_lin_accel_i = J_p_i @ dv + J_dot_p_i @ np.asarray(joint_velocities_current)
        d_roll_i = np.asarray(wheel_directions)[i, 0:3]
        d_lat_i = np.asarray(wheel_directions)[i, 3:6]
        longitudinal_slip = float(np.dot(contact_lin_accel_i, d_roll_i)) - r_wheel * ddq_k
        wheel_constraints.append(longitudinal_slip)
        lateral_slip = float(np.dot(contact_lin_accel_i, d_lat_i))
        wheel_constraints.append(lateral_slip)
    return np.array(wheel_constraints)


def jacobian_value_at_zero(fun, n: int):
    """Exact for an affine f: jacobian columns f(e_i) - f(0), value f(0)."""
    f0 = np.asarray(fun(np.zeros(n)))
    E = np.eye(n)
    return np.stack([np.asarray(fun(E[i])) - f0 for i in range(n)], axis=1), f0
