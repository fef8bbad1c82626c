"""Generate the golden fixtures under tests/golden/ (committed; re-run only to regenerate).

    python tests/golden/make_golden.py

PROVENANCE.  The reference ships no tests, fixtures or golden vectors, and neither its C++
path nor its Python codegen can be built or imported here (MuJoCo / CasADi / OSQP / Eigen /
abseil absent, no network).  These vectors therefore come from the CPU
oracle (oracle/osc_qp.py restating the reference's CasADi QP; oracle/qp_exact.py solving it
exactly with a KKT certificate) on seeded synthetic inputs (osc_amd.synth).
Parity is *unpinned* against the reference's own outputs; every stored solution carries a KKT
certificate (all residuals <= 1e-9) instead.

Each .npz holds, per environment: inputs M, C, J, b, T, mask; the exact design vector x
(dv, u, z), the OSQP-convention duals y, torques tau = x[nv:nv+nu] and the certificate.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "operational-space-control_amd")]

from osc_qp import build_qp, load_model, torque  # noqa: E402
from qp_exact import certified, solve_exact  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

# (name, robot, scenario, mask mode, nenv, seed)   -- seeds follow SURVEY.md §8d: 20251015 + config
CASES = [
    ("go2_standing", "unitree_go2", "standing", "ones", 8, SEED_BASE + 2),
    ("go2_tumbling_mask", "unitree_go2", "tumbling", "bernoulli", 8, SEED_BASE + 102),
    ("go2_no_contact", "unitree_go2", "standing", "zeros", 4, SEED_BASE + 202),
    ("walter_standing", "walter_sr", "standing", "ones", 8, SEED_BASE + 3),
    ("walter_tumbling_mask", "walter_sr", "tumbling", "bernoulli", 8, SEED_BASE + 4),
    ("walter_no_contact", "walter_sr", "tumbling", "zeros", 4, SEED_BASE + 204),
    ("wheels_tumbling_mask", "walter_sr_wheels", "tumbling", "bernoulli", 8, SEED_BASE + 5),
]


def make_case(name, robot, scenario, mask_mode, nenv, seed):
    model = load_model(robot)
    d = generate(robot, nenv, seed, scenario, mask_mode)
    xs, ys, taus, certs = [], [], [], []
    for e in range(nenv):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        qp = build_qp(model, *args)
        sol = solve_exact(model, qp, *args[:3])
        assert certified(sol.cert), (name, e, sol.cert)
        xs.append(sol.x)
        ys.append(sol.y)
        taus.append(torque(model, sol.x))
        certs.append([sol.cert[k] for k in ("stationarity", "primal", "dual", "complementarity")])
    out = dict(d, x=np.array(xs), y=np.array(ys), tau=np.array(taus), cert=np.array(certs),
               robot=np.array(robot), scenario=np.array(scenario), seed=np.array(seed))
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    return path, max(max(c) for c in certs)


if __name__ == "__main__":
    for case in CASES:
        path, worst = make_case(*case)
        print(f"{os.path.basename(path):28s} worst KKT residual {worst:.2e}")
