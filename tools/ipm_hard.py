"""Diagnostic: evaluate IPM variants (tools/ipm_model.py) on the hard environments collected by
tools/stall_sweep.sh (gpurun_out/stalls_*.npz) and on a random sample."""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402
import ipm_model as im  # noqa: E402
from osc_qp import load_model  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

KEYS = ("M", "C", "J", "b", "T", "mask")
hard = []
for f in sorted(glob.glob(os.path.join(REPO, "gpurun_out", "stalls_*_*_*_*.npz"))):
    robot = [r for r in ("walter_sr_wheels", "walter_sr", "unitree_go2")
             if os.path.basename(f)[7:].startswith(r)][0]
    z = np.load(f)
    m = load_model(robot)
    hard += [im.reduce_qp(m, *(z[k][e] for k in KEYS))[:4] for e in range(len(z["idx"]))]
rand = []
for robot, n in (("unitree_go2", 256), ("walter_sr", 128)):
    m = load_model(robot)
    d = generate(robot, n, SEED_BASE + 77, "tumbling", "bernoulli")
    rand += [im.reduce_qp(m, *(d[k][e] for k in KEYS))[:4] for e in range(n)]
base = ("etam0.1", "cap1e-5", "y0_nofz", "sig2")
for v in sys.argv[1:] or ["-"]:
    var = base + (tuple(v.split("+")) if v != "-" else ())
    hi = np.array([im.ipm(*p, variant=var)[1] for p in hard])
    ri = np.array([im.ipm(*p, variant=var)[1] for p in rand])
    npass = None
    print(f"{v:28s} hard: fail {int((hi >= 40).sum()):3d} mean {hi.mean():5.2f} max {hi.max():2d}"
          f" | random: fail {int((ri >= 40).sum())} mean {ri.mean():5.2f} max {ri.max():2d}", flush=True)
