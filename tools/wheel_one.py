"""Diagnostic (GPU): solve a single env of a wheel batch alone (status, iterations, torques; a
library built with a printf in the interior-point loop, OSC_LIB_PATH=..., traces it).

    python tools/wheel_one.py scenario seed nenv env
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import torch  # noqa: E402

from osc_amd.robots import config_path  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions  # noqa: E402

scen, seed, nenv, e = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")), "walter_sr_wheels_noslip_config.yaml")
d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, scen, "ones" if scen == "standing" else "bernoulli")
wd = wheel_directions("walter_sr_wheels", d, np.array(WALTER_WHEEL_DOFS), np.full(8, WHEEL_RADIUS),
                      SEED_BASE + seed + 1)
d1 = {k: np.asarray(v)[e:e + 1] for k, v in d.items()}
s = OSCBatchSolver("walter_sr_wheels", YAML)
r = s.solve(**d1, wheel_dir=wd[e:e + 1])
torch.cuda.synchronize()
print("status", r.status.cpu().numpy(), "iters", r.iters.cpu().numpy(), "tau", r.tau.cpu().numpy())
