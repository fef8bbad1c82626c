"""Seeded synthetic post-kinematics inputs for the batched OSC solve.

The robot XMLs live in the un-vendored ``mujoco-models`` archive, so no real ``mjData`` exists
offline.  These generators produce inputs with the *shape and structure* of what
``update_osc_data`` (unitree_go2/operational_space_controller.h:376-455) hands to the QP
assembly: an SPD mass matrix, bias forces with gravity on the base-z row, tree-sparse site
Jacobians, task bias accelerations, task targets and a contact mask.

Layout (env-major, row-major per env, fp64) -- the layout the C-ABI consumes:
  M (nenv, nv, nv)   C (nenv, nv)   J (nenv, 6ns, nv)   b (nenv, 6ns)
  T (nenv, ns, 6)    mask (nenv, nc)
"""
from __future__ import annotations

import numpy as np

from .robots import ROBOTS

SEED_BASE = 20251015


def _site_row_dofs(robot: str):
    r = ROBOTS[robot]
    ns = len(r["site_keys"])
    rows = []
    for i in range(ns):                       # translational rows of site i
        rows += [r["site_dofs"][i]] * 3
    for i in range(ns):                       # rotational rows of site i
        d = r["site_dofs"][i]
        rows += [[3, 4, 5] if i == 0 else d] * 3   # base site rotation: base angular dofs only
    return rows


def generate(robot: str, nenv: int, seed: int, scenario: str = "standing",
             mask_mode: str = "ones", mask_p: float = 0.75) -> dict:
    r = ROBOTS[robot]
    nv, nc = r["nv"], r["nc"]
    ns = len(r["site_keys"])
    s = 6 * ns
    rng = np.random.default_rng(seed)

    # M = Q diag(lambda) Q^T + 1e-6 I, lambda log-uniform on [1e-2, 2e1]
    G = rng.standard_normal((nenv, nv, nv))
    Q, _ = np.linalg.qr(G)
    lam = np.exp(rng.uniform(np.log(1e-2), np.log(2e1), size=(nenv, nv)))
    M = np.einsum("eij,ej,ekj->eik", Q, lam, Q) + 1e-6 * np.eye(nv)
    M = 0.5 * (M + np.transpose(M, (0, 2, 1)))

    C = 2.0 * rng.standard_normal((nenv, nv))
    C[:, 2] += r["base_mass"] * 9.81

    J = 0.3 * rng.standard_normal((nenv, s, nv))
    struct = np.zeros((s, nv))
    for row, dofs in enumerate(_site_row_dofs(robot)):
        struct[row, dofs] = 1.0
    J *= struct

    b = rng.standard_normal((nenv, s))

    T = np.zeros((nenv, ns, 6))
    if scenario == "standing":
        T[:, 0, :] = 10.0 * rng.standard_normal((nenv, 6))
    elif scenario == "tumbling":
        T[:] = 10.0 * rng.standard_normal((nenv, ns, 6))
    else:
        raise ValueError(scenario)

    if mask_mode == "ones":
        mask = np.ones((nenv, nc))
    elif mask_mode == "bernoulli":
        mask = (rng.uniform(size=(nenv, nc)) < mask_p).astype(np.float64)
    elif mask_mode == "zeros":
        mask = np.zeros((nenv, nc))
    else:
        raise ValueError(mask_mode)
    return dict(M=np.ascontiguousarray(M), C=C, J=np.ascontiguousarray(J), b=b, T=T, mask=mask)


# walter_sr_wheels/autogen/autogen.py:64 (the commented no-slip design): self.wheel_radius = 0.065
WHEEL_RADIUS = 0.065
# The illustrative WaLTER tree (config/walter_sr.xml) has no wheel joints (its 14 dofs are the
# floating base and 4 x (thigh, shin)); the rolling term -r ddq_k of wheel i then stands on the
# shin joint of its leg, 2 wheels per leg in contact-site order (tlf, tlr, trf, trr, hlf, ...).
WALTER_WHEEL_DOFS = [7, 7, 9, 9, 11, 11, 13, 13]


def wheel_directions(robot: str, d: dict, dof, radius, seed: int) -> np.ndarray:
    """Per-env wheel directions (nenv, nc, 6) = (d_roll, d_lat) per wheel for the no-slip rows
    (walter_sr_wheels/autogen/autogen.py:128-240), consistent with a strictly feasible point so
    the synthetic QPs stay feasible: at x0 = (dv0, u = 0, z = (0, 0, 1) per contact in touch),
    dv0 = M^-1 (Jc z - C), every wheel in contact has d_lat . a_i = 0 and
    d_roll . a_i = r_i dv0[k_i] for its contact-point acceleration a_i = J_p,i dv0 + b_i -- as the
    real robot's no-slip kinematics are consistent.  d_lat is a random unit vector orthogonal to
    a_i; d_roll a unit vector orthogonal to d_lat with the required projection on a_i (scaled
    off the unit sphere only if |r dv0[k]| > |a_i|)."""
    r = ROBOTS[robot]
    nv, nc, ns = r["nv"], r["nc"], len(r["site_keys"])
    M, C, J, b, mask = d["M"], d["C"], d["J"], d["b"], d["mask"]
    nenv = M.shape[0]
    rng = np.random.default_rng(seed)
    r0 = 3 * ns - 3 * nc
    Jc = np.transpose(J[:, r0:3 * ns, :], (0, 2, 1))            # (nenv, nv, 3nc)
    z0 = np.zeros((nenv, 3 * nc))
    z0[:, 2::3] = (mask != 0).astype(np.float64)
    dv0 = np.linalg.solve(M, (np.einsum("eij,ej->ei", Jc, z0) - C)[..., None])[..., 0]
    out = np.zeros((nenv, nc, 6))
    for i in range(nc):
        a = np.einsum("ecj,ej->ec", J[:, r0 + 3 * i:r0 + 3 * i + 3, :], dv0) + b[:, r0 + 3 * i:r0 + 3 * i + 3]
        an = np.linalg.norm(a, axis=1, keepdims=True)
        ah = a / an
        g = rng.standard_normal((nenv, 3))
        lat = g - np.sum(g * ah, axis=1, keepdims=True) * ah
        lat /= np.linalg.norm(lat, axis=1, keepdims=True)
        w = np.cross(lat, ah)                                      # unit, orthogonal to lat and a
        c = (radius[i] * dv0[:, dof[i]] if dof[i] >= 0 else np.zeros(nenv))[:, None]
        cos = c / an
        sin = np.sqrt(np.maximum(1.0 - cos ** 2, 0.0))
        roll = cos * ah + sin * w                                  # |roll| = 1 when |cos| <= 1
        roll = np.where(np.abs(cos) <= 1.0, roll, c / an * ah)
        out[:, i, :3], out[:, i, 3:] = roll, lat
    return np.ascontiguousarray(out)


def random_walk(inputs: dict, rng: np.random.Generator, scale: float = 0.01) -> dict:
    """One step of the 1 % random walk used for warm-start runs: C, J, b, T
    entrywise multiplicative; M by a congruence M' = A M A' with A = I + scale E / sqrt(nv), E
    standard normal, so M stays symmetric positive definite (an entrywise 1 % walk of M drifts
    indefinite within a few dozen steps, its smallest eigenvalue being 1e-2 of the largest)."""
    out = {}
    for k, v in inputs.items():
        if k == "mask":
            out[k] = v.copy()
            continue
        if k == "M":
            n = v.shape[-1]
            A = np.eye(n) + scale / np.sqrt(n) * rng.standard_normal(v.shape)
            w = np.einsum("eij,ejk,elk->eil", A, v, A)
            w = 0.5 * (w + np.transpose(w, (0, 2, 1)))
        else:
            w = v * (1.0 + scale * rng.standard_normal(v.shape))
        out[k] = w
    return out
