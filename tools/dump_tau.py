"""Diagnostic (GPU box): solve one seeded synthetic batch and save tau / iters / status to an npz
(for tools/hardest_envs.py, which finds the environments farthest from the exact oracle).
Usage: python tools/dump_tau.py robot scenario mask nenv seed_offset out.npz"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot, scenario, mask, nenv, off, out = sys.argv[1:7]
d = generate(robot, int(nenv), SEED_BASE + int(off), scenario, mask)
res = OSCBatchSolver(robot).solve(**d)
torch.cuda.synchronize()
np.savez(out, tau=res.tau.cpu().numpy(), iters=res.iters.cpu().numpy(),
         status=res.status.cpu().numpy())
print("saved", out, "max iters", int(res.iters.max()), "unconverged", int((res.status != 0).sum()))
