"""Diagnostic (GPU): envs of a joint-state batch that do not come back OK -- their status,
iterations, the kinematics' M, C, J, b and the targets saved to gpurun_out/status_diag_<tag>.npz for
the CPU oracle.  python tools/status_diag.py ROBOT NENV SEED JOINT_RANGE [MASK]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import json  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.kinematics import KinematicsBatch, load_tree, random_states  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402

robot, nenv, seed, jr = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), float(sys.argv[4])
mask_mode = sys.argv[5] if len(sys.argv) > 5 else "ones"
tree = load_tree(robot)
kb, solver = KinematicsBatch(tree=tree), OSCBatchSolver(robot)
q, v = random_states(tree, nenv, seed, joint_range=jr)
d = generate(robot, nenv, seed, "standing" if mask_mode == "ones" else "tumbling", mask_mode)
k = kb.compute(q, v, want_sites=False)
args = solver.prepare(k.M, k.C, k.J, k.b, d["T"], d["mask"])
out = solver.alloc_outputs(nenv, want_x=True)
solver.solve_into(out, *args)
torch.cuda.synchronize()
st, it = out.status.cpu().numpy(), out.iters.cpu().numpy()
bad = np.nonzero(st != 0)[0]
print(json.dumps({"robot": robot, "nenv": nenv, "seed": seed, "jr": jr, "counts": np.bincount(st).tolist(),
                  "bad": bad[:50].tolist(), "status": st[bad[:50]].tolist(), "iters": it[bad[:50]].tolist()}))
if len(bad):
    sel = bad[:64]
    np.savez(os.path.join(REPO, "gpurun_out", f"status_diag_{robot}_{nenv}_{seed}.npz"),
             envs=sel, status=st[sel], iters=it[sel], x=out.x.cpu().numpy()[sel],
             M=k.M.cpu().numpy()[sel], C=k.C.cpu().numpy()[sel], J=k.J.cpu().numpy()[sel],
             b=k.b.cpu().numpy()[sel], T=d["T"][sel], mask=d["mask"][sel])
