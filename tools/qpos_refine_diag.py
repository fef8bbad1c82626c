"""Diagnostic (GPU): cold solves from joint states (Go2, the bench's front-end states) -- status
counts, and for envs whose full-space refinement was rejected, why (OSC_REFINE_DIAG build:
3 + 16 rows still violated after the last round + 32 move too large / not finite) and how far
the returned torques are from the exact oracle.

    OSC_LIB_PATH=<diag lib> python tools/qpos_refine_diag.py [nenv] [env,env,...]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from osc_amd.kinematics import KinematicsBatch, load_tree, random_states  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402
from osc_qp import build_qp, load_model, torque  # noqa: E402
from qp_exact import solve_exact  # noqa: E402

nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
robot, seed = "unitree_go2", shard_seed(0) + 7
solver = OSCBatchSolver(robot)
tree = load_tree(robot)
kb = KinematicsBatch(tree=tree)
qpos, qvel = random_states(tree, nenv, seed, joint_range=0.5)
qpos, qvel = torch.from_numpy(qpos).cuda(), torch.from_numpy(qvel).cuda()
d = generate(robot, nenv, seed, "standing", "ones")
T, mask = torch.from_numpy(d["T"]).cuda(), torch.from_numpy(d["mask"]).cuda()
kout = kb.compute(qpos, qvel)
res = solver.solve(kout.M, kout.C, kout.J, kout.b, T, mask)
torch.cuda.synchronize()
st = res.status.cpu().numpy()
vals, cnt = np.unique(st, return_counts=True)
print(json.dumps({"status_codes": dict(zip(map(int, vals), map(int, cnt)))}), flush=True)
model = load_model(robot)
bad = np.nonzero(st != 0)[0][:12]
if len(sys.argv) > 2:   # also these envs, whatever their status (e.g. an earlier build's rejects)
    bad = np.union1d(bad, np.array([int(v) for v in sys.argv[2].split(",")]))
M, C, J, b = (t.cpu().numpy() for t in (kout.M, kout.C, kout.J, kout.b))
Tn, mk = d["T"], d["mask"]
tau = res.tau.cpu().numpy()
for e in bad:
    args = [M[e], C[e], J[e], b[e], Tn[e], mk[e]]
    try:
        ref = torque(model, solve_exact(model, build_qp(model, *args), *args[:3]).x)
        err = float(np.abs(tau[e] - ref).max() / max(np.abs(ref).max(), 1.0))
    except Exception as ex:
        err = f"oracle refused: {type(ex).__name__}"
    print(json.dumps({"env": int(e), "status": int(st[e]), "iters": int(res.iters[e]), "err": err}), flush=True)
