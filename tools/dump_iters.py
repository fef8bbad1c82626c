"""Per-env interior-point iteration counts of cold solves (GPU), for the lockstep/compaction study.

    python tools/dump_iters.py OUT.npz

Writes iters[config] for Go2 / WaLTER standing and tumbling batches (bench seeds)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "operational-space-control_amd"))
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402

out = {}
for robot, nenv, scen, mask in (("unitree_go2", 65536, "standing", "ones"),
                                ("unitree_go2", 65536, "tumbling", "bernoulli"),
                                ("walter_sr", 65536, "standing", "ones"),
                                ("walter_sr", 65536, "tumbling", "bernoulli")):
    s = OSCBatchSolver(robot)
    d = generate(robot, nenv, shard_seed(0), scen, mask)
    r = s.solve(**d)
    torch.cuda.synchronize()
    it = r.iters.cpu().numpy()
    st = r.status.cpu().numpy()
    key = f"{robot}_{scen}_{nenv}"
    out[key] = it
    w = it.reshape(-1, 4).max(axis=1)
    print(key, "mean env", it.mean(), "mean wave", w.mean(), "max", it.max(),
          "status", np.bincount(st), flush=True)
np.savez(sys.argv[1], **out)
