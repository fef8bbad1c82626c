"""Regenerate the oracle outputs of tests/golden/go2_unrefined_joint_states.npz (committed; re-run
only to regenerate).

    python tests/golden/make_joint_state_regressions.py

PROVENANCE.  The inputs are the 12 Go2 environments that round 5's status census
(tools/status_diag.py: 65,536-env joint-state batches, random_states seeds 11 / 13 / 14,
joint_range 1.0, standing targets, all contacts on) found OSC_SOLVE_UNREFINED: their M, C, J, b
as the GPU's kinematics kernel computed them (oracle/kinematics.py agrees to 1e-12), with the
batch index (envs) and seed of each.  All 12 had the same cause -- the refinement's rounds cycled
between active sets -- and returned torques up to 4e-3 (normwise) off.  The
outputs (x, y, tau, cert) are the CPU oracle's exact optimum (oracle/qp_exact.py), KKT-certified,
in make_golden.py's format, so test_oracle / test_gpu_parity pick the file up with the others.
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

PATH = os.path.join(HERE, "go2_unrefined_joint_states.npz")
INPUTS = ("M", "C", "J", "b", "T", "mask", "envs", "seed")


def main():
    z = np.load(PATH)
    d = {k: z[k] for k in INPUTS}
    model = load_model("unitree_go2")
    xs, ys, taus, certs = [], [], [], []
    for e in range(d["M"].shape[0]):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        sol = solve_exact(model, build_qp(model, *args), *args[:3])
        assert certified(sol.cert), (e, sol.cert)
        xs.append(sol.x)
        ys.append(sol.y)
        taus.append(torque(model, sol.x))
        certs.append([sol.cert[k] for k in ("stationarity", "primal", "dual", "complementarity")])
    np.savez_compressed(PATH, **d, x=np.array(xs), y=np.array(ys), tau=np.array(taus),
                        cert=np.array(certs), robot=np.array("unitree_go2"),
                        scenario=np.array("joint_states"))
    print(f"{os.path.basename(PATH)}: {len(xs)} envs, worst KKT residual {np.max(certs):.2e}")


if __name__ == "__main__":
    main()
