"""Diagnostic (GPU): the wheel-row solve of the parity test's batch with 0, 2, 5 and 10 refinement
steps (OSC_REFINE_STEPS), per-env torque error against the exact oracle and status; the design
vectors go to an npz for CPU-side study.

    python tools/wheel_diag.py [out.npz] [scenario] [seed]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import torch  # noqa: E402

from osc_amd.robots import config_path  # noqa: E402
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions  # noqa: E402
from osc_qp import WheelRows, build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wheel_diag.npz"
scen = sys.argv[2] if len(sys.argv) > 2 else "standing"
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 81
YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")), "walter_sr_wheels_noslip_config.yaml")
nenv = 64
model = load_model("walter_sr_wheels")
wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))
d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, scen, "ones" if scen == "standing" else "bernoulli")
wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + seed + 1)
ref = []
for e in range(nenv):
    args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
    ref.append(torque(model, solve_exact(model, build_qp(model, *args, wheel, wd[e]), *args[:3]).x))
ref = np.array(ref)
from osc_amd.solver import OSCBatchSolver  # noqa: E402
res = {}
for steps in ("0", "2", "5", "10"):
    os.environ["OSC_REFINE_STEPS"] = steps
    s = OSCBatchSolver("walter_sr_wheels", YAML)
    r = s.solve(**d, want_x=True, wheel_dir=wd)
    torch.cuda.synchronize()
    tau = r.tau.cpu().numpy()
    err = np.abs(tau - ref).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), 1.0)
    res[f"x{steps}"] = r.x.cpu().numpy()
    res[f"st{steps}"] = r.status.cpu().numpy()
    res[f"it{steps}"] = r.iters.cpu().numpy()
    res[f"err{steps}"] = err
    worst = np.argsort(err)[-5:][::-1]
    print(json.dumps({"steps": steps, "status": np.bincount(r.status.cpu().numpy(), minlength=4).tolist(),
                      "err_max": float(err.max()), "err_med": float(np.median(err)),
                      "worst": [(int(i), float(err[i])) for i in worst]}), flush=True)
    s.close()
np.savez(out, ref=ref, **res)
