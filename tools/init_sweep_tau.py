"""Diagnostic (CPU): interior-point variants of tools/ipm_model.py on the torque-coordinate
reduction (Go2's kernel path), iteration statistics over a 4,096-env batch: mean, 4-env wave
mean, 99.9th percentile and max (the kernel's time at 4,096 envs is its slowest wave's).
    python tools/init_sweep_tau.py nenv variant1 variant2 ...   (variant: a+b+c, "base")"""
import os
import sys
from multiprocessing import Pool

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402
import ipm_model as im  # noqa: E402
from osc_qp import load_model  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

KVAR = ("etam0.1", "cap1e-5", "y0_nofz", "sig2", "rpcarry1e-6", "recenter28")
ROBOT = os.environ.get("ROBOT", "unitree_go2")
SCEN = os.environ.get("SCEN", "standing,ones").split(",")
NENV = int(sys.argv[1])
MODEL = load_model(ROBOT)
D = generate(ROBOT, NENV, SEED_BASE + int(os.environ.get("SEED", "2")), SCEN[0], SCEN[1])
EPS = float(os.environ.get("EPS", "1e-9"))


def one(args):
    e, var = args
    p = im.reduce_qp_tau(MODEL, *(D[k][e] for k in ("M", "C", "J", "b", "T", "mask")))[:4]
    if "nobig" in var or "nofz0" in var:
        Hr, g, G, h = p
        keep = np.ones(len(h), bool)
        if "nobig" in var:
            keep &= ~np.isclose(h, im.BIG_NUMBER)
        if "nofz0" in var:
            keep &= ~((h == 0) & (np.abs(G).sum(1) == 1) & (G.sum(1) == -1))
        p = (Hr, g, G[keep], h[keep])
    if "jacobi" in var or "rownorm" in var:
        Hr, g, G, h = p
        d = np.ones(len(g))
        if "jacobi" in var:
            d = 1.0 / np.sqrt(np.abs(np.diag(Hr)))
        Hr, g, G = d[:, None] * Hr * d[None, :], d * g, G * d[None, :]
        if "rownorm" in var:
            rn = 1.0 / np.linalg.norm(G, axis=1)
            G, h = G * rn[:, None], h * rn
        p = (Hr, g, G, h)
    return im.ipm(*p, eps_mu=EPS, max_iter=50, variant=var)[1]


if __name__ == "__main__":
    for v in sys.argv[2:]:
        var = KVAR + (tuple(v.split("+")) if v != "base" else ())
        var = tuple(x for x in var if not (v != "base" and x in ("y0_nofz",) and "noy0" in v))
        with Pool(8) as pool:
            its = np.array(pool.map(one, [(e, var) for e in range(NENV)], chunksize=32))
        w = its.reshape(-1, 4).max(1)
        print(f"{v:28s} mean {its.mean():5.2f} wave_mean {w.mean():5.2f} p99.9 "
              f"{np.percentile(its, 99.9):5.1f} max {its.max():2d} fail {(its >= 50).sum()}", flush=True)
