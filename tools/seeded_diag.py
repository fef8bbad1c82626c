"""Diagnostic (GPU): why the GPU's active set (from its exported duals) does not certify in the
oracle's seeded check (oracle/parallel.seeded_batch) for most envs.  Solves a small batch with the
duals, saves inputs, x, y to gpurun_out/seeded_diag.npz for analysis on the CPU.
    python tools/seeded_diag.py [robot] [nenv]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 256
s = OSCBatchSolver(robot)
d = generate(robot, nenv, SEED_BASE + 9, "tumbling", "bernoulli")
out = s.alloc_outputs(nenv, want_y=True)
s.solve_into(out, *s.prepare(**d))
torch.cuda.synchronize()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", f"seeded_diag_{robot}.npz"), x=out.x.cpu().numpy(),
         y=out.y.cpu().numpy(), status=out.status.cpu().numpy(), **d)
print("saved", nenv)
