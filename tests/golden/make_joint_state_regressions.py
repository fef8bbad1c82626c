"""Regenerate the oracle outputs of the joint-state regression fixtures under tests/golden/
(committed; re-run only to regenerate).

    python tests/golden/make_joint_state_regressions.py

PROVENANCE.  The inputs are environments that round 5's status censuses (tools/status_diag.py:
65,536-env joint-state batches, random_states seeds as in each file's `seed`, standing targets,
all contacts on) found not OK, with their M, C, J, b as the GPU's kinematics kernel computed them
(oracle/kinematics.py agrees to 1e-12) and their batch index (`envs`):
* go2_unrefined_joint_states.npz -- 12 Go2 envs (seeds 11 / 13 / 14, joint_range 1.0)
  OSC_SOLVE_UNREFINED: the refinement's rounds cycled between active sets;
* go2_stalled_joint_states.npz -- 3 Go2 envs of the wider census (seeds 21 / 24 joint_range 1.0:
  UNREFINED; seed 22, 0.5: MAX_ITER, the adaptive fraction-to-the-boundary rule stalling);
* walter_stalled_joint_states.npz -- 3 WaLTER envs (seeds 23 / 24 range 1.5, 27 range 1.0:
  MAX_ITER, the same stall).
The outputs (x, y, tau, cert) are the CPU oracle's exact optimum (oracle/qp_exact.py),
KKT-certified, in make_golden.py's format, so test_oracle / test_gpu_parity pick the files up with
the others.
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

CASES = [("go2_unrefined_joint_states.npz", "unitree_go2"),
         ("go2_stalled_joint_states.npz", "unitree_go2"),
         ("walter_stalled_joint_states.npz", "walter_sr")]
INPUTS = ("M", "C", "J", "b", "T", "mask", "envs", "seed")


def make(name, robot):
    path = os.path.join(HERE, name)
    z = np.load(path)
    d = {k: z[k] for k in INPUTS}
    model = load_model(robot)
    xs, ys, taus, certs = [], [], [], []
    for e in range(d["M"].shape[0]):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        sol = solve_exact(model, build_qp(model, *args), *args[:3])
        assert certified(sol.cert), (e, sol.cert)
        xs.append(sol.x)
        ys.append(sol.y)
        taus.append(torque(model, sol.x))
        certs.append([sol.cert[k] for k in ("stationarity", "primal", "dual", "complementarity")])
    np.savez_compressed(path, **d, x=np.array(xs), y=np.array(ys), tau=np.array(taus),
                        cert=np.array(certs), robot=np.array(robot),
                        scenario=np.array("joint_states"))
    print(f"{name}: {len(xs)} envs, worst KKT residual {np.max(certs):.2e}")


if __name__ == "__main__":
    for case in CASES:
        make(*case)
