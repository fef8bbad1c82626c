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
