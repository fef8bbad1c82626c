"""Dump tau / x / status / iters of fixed seeded cold solves to an .npz (GPU), for comparing two
library builds (OSC_LIB_PATH selects the library):

    OSC_LIB_PATH=<lib> python tools/dump_cases.py OUT.npz
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "operational-space-control_amd"))
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

CASES = [("unitree_go2", "standing", "ones", 4096, 21), ("unitree_go2", "tumbling", "bernoulli", 8192, 22),
         ("walter_sr", "tumbling", "bernoulli", 4096, 23), ("walter_sr", "tumbling", "bernoulli", 32768, 25)]
out = {}
for robot, scen, mask, nenv, seed in CASES:
    s = OSCBatchSolver(robot)
    r = s.solve(**generate(robot, nenv, SEED_BASE + seed, scen, mask), want_x=True)
    torch.cuda.synchronize()
    k = f"{robot}_{scen}_{nenv}"
    for f in ("tau", "x", "status", "iters"):
        out[f"{k}.{f}"] = getattr(r, f).cpu().numpy()
np.savez(sys.argv[1], **out)
