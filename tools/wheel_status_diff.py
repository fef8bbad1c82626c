"""Wheel no-slip rows: which envs of a tumbling batch change status between two library builds,
and how far each newly-OK env is from the exact optimum (oracle/qp_exact.py).  GPU box.

    python tools/wheel_status_diff.py OLD_LIB NEW_LIB NENV SEED
Each build runs in a child process (OSC_LIB_PATH); the parent only compares and runs the oracle.
"""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

if sys.argv[1] == "--child":
    import torch
    from osc_amd.robots import config_path
    from osc_amd.solver import OSCBatchSolver
    from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions
    nenv, seed, out = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    yaml = os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                        "walter_sr_wheels_noslip_config.yaml")
    d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, "tumbling", "bernoulli")
    wd = wheel_directions("walter_sr_wheels", d, np.array(WALTER_WHEEL_DOFS), np.full(8, WHEEL_RADIUS),
                          SEED_BASE + seed + 1)
    r = OSCBatchSolver("walter_sr_wheels", yaml).solve(**d, wheel_dir=wd)
    torch.cuda.synchronize()
    np.savez(out, tau=r.tau.cpu().numpy(), status=r.status.cpu().numpy(), iters=r.iters.cpu().numpy())
    sys.exit(0)

old, new, nenv, seed = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
res = {}
for tag, lib in (("old", old), ("new", new)):
    path = f"/tmp/wsd_{tag}.npz"
    env = dict(os.environ, OSC_LIB_PATH=lib)
    subprocess.run([sys.executable, __file__, "--child", str(nenv), str(seed), path], env=env, check=True)
    res[tag] = np.load(path)
so, sn = res["old"]["status"], res["new"]["status"]
changed = np.nonzero(so != sn)[0]
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions  # noqa: E402
from osc_qp import WheelRows, build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402
model = load_model("walter_sr_wheels")
wheel = WheelRows(dof=np.array(WALTER_WHEEL_DOFS), radius=np.full(8, WHEEL_RADIUS))
d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, "tumbling", "bernoulli")
wd = wheel_directions("walter_sr_wheels", d, wheel.dof, wheel.radius, SEED_BASE + seed + 1)
rows = []
for e in changed:
    args = [d[k][e] for k in ("M", "C", "J", "b", "T", "mask")]
    try:
        ref = torque(model, solve_exact(model, build_qp(model, *args, wheel, wd[e]), *args[:3]).x)
        err = float(np.abs(res["new"]["tau"][e] - ref).max() / max(np.abs(ref).max(), 1.0))
    except Exception as ex:   # the oracle refuses inconsistent / degenerate equality sets
        err = f"oracle refused: {type(ex).__name__}"
    rows.append({"env": int(e), "old": int(so[e]), "new": int(sn[e]), "err": err})
print(json.dumps({"nenv": nenv, "seed": seed, "old_status": np.bincount(so, minlength=4).tolist(),
                  "new_status": np.bincount(sn, minlength=4).tolist(), "changed": rows}))
