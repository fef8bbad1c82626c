"""Study of the wheel no-slip rows' interior-point settings (GPU): for each (penalty, row
tolerance, eps_mu) the convergence status counts, iterations and torque error against the exact
oracle on a sample of envs.

    python tools/wheel_sweep.py [nenv] [noracle]
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

YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")), "walter_sr_wheels_noslip_config.yaml")
nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 512
nor = int(sys.argv[2]) if len(sys.argv) > 2 else 16
model = load_model("walter_sr_wheels")
wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))
cases = []
for scen, mm in (("tumbling", "bernoulli"), ("standing", "ones")):
    d = generate("walter_sr_wheels", nenv, SEED_BASE + 91, scen, mm)
    wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + 92)
    ref = []
    for e in range(nor):
        args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
        ref.append(torque(model, solve_exact(model, build_qp(model, *args, wheel, wd[e]), *args[:3]).x))
    cases.append((scen, d, wd, np.array(ref)))

from osc_amd.solver import OSCBatchSolver  # noqa: E402
settings = [(p, t, e) for p in ("1e2", "1e3", "1e4") for t in ("1e-8", "1e-6") for e in ("1e-12", "1e-9")]
for pen, tol, eps in settings:
    os.environ["OSC_WHEEL_PENALTY"], os.environ["OSC_WHEEL_TOL"] = pen, tol
    s = OSCBatchSolver("walter_sr_wheels", YAML, eps_mu=float(eps))
    for scen, d, wd, ref in cases:
        res = s.solve(**d, wheel_dir=wd)
        torch.cuda.synchronize()
        st = res.status.cpu().numpy()
        it = res.iters.cpu().numpy()
        tau = res.tau.cpu().numpy()[:nor]
        err = (np.abs(tau - ref).max(axis=1) / np.maximum(np.abs(ref).max(axis=1), 1.0))
        print(json.dumps({"penalty": pen, "tol": tol, "eps_mu": eps, "scenario": scen,
                          "status": np.bincount(st, minlength=4).tolist(),
                          "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                          "err_max": float(err.max()), "err_med": float(np.median(err))}), flush=True)
    s.close()
