"""Setup (assembly) kernel time against batch size (GPU, HIP events, median of 50): where the
assembly grid needs a second round of wavefronts per SIMD.

    python tools/setup_scaling.py ROBOT N1,N2,...
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "operational-space-control_amd"))
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1]
s = OSCBatchSolver(robot)
res = []
for n in [int(v) for v in sys.argv[2].split(",")]:
    args = s.prepare(**generate(robot, n, SEED_BASE + 2, "standing", "ones"))
    out = s.alloc_outputs(n)
    ts, ti = [], []
    for r in range(60):
        a, b, c = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        a.record()
        s.assemble_into(out, *args)
        b.record()
        s.solve_assembled_into(out, args[5])
        c.record()
        torch.cuda.synchronize()
        if r >= 10:
            ts.append(a.elapsed_time(b))
            ti.append(b.elapsed_time(c))
    res.append({"nenv": n, "setup_ms": float(np.median(ts)), "ipm_ms": float(np.median(ti))})
    print(json.dumps(res[-1]), flush=True)
