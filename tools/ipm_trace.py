"""Diagnostic: per-iteration trace (mu, affine step, step, sigma, residuals) of the environments
that take the most interior-point iterations in a batch (tools/ipm_model.py restatement).
    python tools/ipm_trace.py [robot] [nenv] [variant]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402
import ipm_model as im  # noqa: E402
from osc_qp import load_model  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
var = ("etam0.1", "cap1e-5", "y0_nofz", "sig2") + (tuple(sys.argv[3].split("+")) if len(sys.argv) > 3 else ())
model = load_model(robot)
d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
probs = [im.reduce_qp(model, *(d[k][e] for k in ("M", "C", "J", "b", "T", "mask")))[:4]
         for e in range(nenv)]
its = np.array([im.ipm(*p, variant=var)[1] for p in probs])
print("hist", np.bincount(its).tolist())
for e in np.argsort(-its)[:4]:
    im.TRACE = []
    im.ipm(*probs[e], variant=var)
    print(f"env {e}: {its[e]} iterations")
    for t in im.TRACE:
        print("  it %2d mu %9.2e a_aff %6.3f a %6.3f alpha %6.3f sig %8.1e |rp| %8.1e |rd| %8.1e" % t)
    im.TRACE = None
