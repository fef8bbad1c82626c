"""Diagnostic: dump torques / status / iterations of one library build (OSC_LIB_PATH) on the
golden inputs and on large synthetic batches, for an offline accuracy comparison of two builds.
    OSC_LIB_PATH=lib.so python tools/ty_acc.py out.npz"""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

res = {}
for path in sorted(glob.glob(os.path.join(REPO, "tests", "golden", "*.npz"))):
    g = np.load(path)
    r = OSCBatchSolver(str(g["robot"])).solve(g["M"], g["C"], g["J"], g["b"], g["T"], g["mask"])
    res["gold_" + os.path.basename(path)[:-4]] = r.tau.cpu().numpy()
for robot, nenv, scen, mk in [("walter_sr", 32768, "standing", "ones"),
                              ("walter_sr", 32768, "tumbling", "bernoulli"),
                              ("walter_sr_wheels", 16384, "tumbling", "bernoulli"),
                              ("unitree_go2", 32768, "tumbling", "bernoulli")]:
    d = generate(robot, nenv, SEED_BASE + 7, scen, mk)
    r = OSCBatchSolver(robot).solve(**d)
    key = f"{robot}_{scen}_{mk}"
    res[key + "_tau"] = r.tau.cpu().numpy()
    res[key + "_st"] = r.status.cpu().numpy()
    res[key + "_it"] = r.iters.cpu().numpy()
np.savez(sys.argv[1], **res)
print("saved", sys.argv[1], len(res))
