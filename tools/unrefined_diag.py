"""Diagnostic (GPU): the Go2 joint-state envs the round-5 census left OSC_SOLVE_UNREFINED
(tests/golden/go2_unrefined_joint_states.npz), solved alone under tuning variants, with their
normwise torque error against the oracle.  OSC_LIB_PATH picks the library (an OSC_REFINE_DIAG
build reports why each refinement was rejected in the status bits).

    python tools/unrefined_diag.py ['{"refine_steps": 4}' ...]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402

z = np.load(os.path.join(REPO, "tests", "golden", "go2_unrefined_joint_states.npz"))
variants = [json.loads(a) for a in sys.argv[1:]] or [{}]
xo = z["x"]
for tune in variants:
    s = OSCBatchSolver("unitree_go2", tuning=tune)
    args = s.prepare(*(torch.from_numpy(z[k]).cuda() for k in ("M", "C", "J", "b", "T", "mask")))
    out = s.alloc_outputs(len(xo), want_x=True)
    s.solve_into(out, *args)
    torch.cuda.synchronize()
    x = out.x.cpu().numpy()
    err = np.abs(x[:, 18:30] - xo[:, 18:30]).max(1) / (1 + np.abs(xo[:, 18:30]).max(1))
    print(json.dumps({"tuning": tune, "status": out.status.cpu().tolist(),
                      "iters": out.iters.cpu().tolist(),
                      "tau_err": [float(f"{e:.2e}") for e in err]}), flush=True)
