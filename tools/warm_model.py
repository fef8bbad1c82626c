"""Diagnostic (CPU): the warm start of osc_ipm_kernel in the numpy model of
tools/ipm_model.py -- iteration counts of warm-started ticks along the 1 % random walk of
SURVEY.md §8d, for the kernel's rule and for candidate rules (the slowest warm env
sets the 4,096-env kernel time).  Not a test and not product code.

    python tools/warm_model.py [nenv] [ticks] [rule ...]
rules: kernel (delta 1, centre 1), d<x>c<y> (floors delta x, centring y), mu<k> (every pair on
the central path at mu = k x the previous tick's final mu... floored), cold
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import numpy as np  # noqa: E402

import ipm_model as im  # noqa: E402
from osc_amd.synth import SEED_BASE, generate, random_walk  # noqa: E402
from osc_qp import load_model  # noqa: E402

KERNEL = ("y0_nofz", "sig2", "etam0.1", "cap1e-5", "recenter28", "rpcarry1e-6")


def warm_init(G, h, y, lam_prev, rule):
    """The warm starting point from the previous tick's (y, lambda) for this tick's rows."""
    m = len(h)
    if rule == "kernel" or rule.startswith("d"):
        dl, c = 1.0, 1.0
        if rule.startswith("d"):
            dl, c = (float(v) for v in rule[1:].split("c"))
        s = np.maximum(h - G @ y, dl)
        lam = np.maximum(lam_prev, dl)
        mu0 = c * (s @ lam) / m
        lam = np.maximum(lam, mu0 / s)
        s = np.maximum(s, mu0 / lam)
        return y, s, lam
    if rule.startswith("mu"):
        k = float(rule[2:])
        sl = np.maximum(h - G @ y, 0.0)
        mu0 = k
        s = np.maximum(sl, np.sqrt(mu0))
        lam = np.maximum(lam_prev, mu0 / s)
        s = np.maximum(s, mu0 / lam)
        return y, s, lam
    raise ValueError(rule)


def main():
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    rules = sys.argv[3:] or ["kernel"]
    model = load_model("unitree_go2")
    d = generate("unitree_go2", nenv, SEED_BASE + 21, "standing", "ones")
    rng = np.random.default_rng(21)
    state = {r: [None] * nenv for r in rules}
    for t in range(ticks):
        if t > 0:
            d = random_walk(d, rng, 0.01)
        probs = [im.reduce_qp_tau(model, *(d[k][e] for k in ("M", "C", "J", "b", "T", "mask")))
                 for e in range(nenv)]
        cold = []
        for p in probs:
            y, it, ok = im.ipm(*p[:4], eps_mu=1e-6, max_iter=50, variant=KERNEL)
            cold.append(it)
        line = [f"tick {t}: cold mean {np.mean(cold):5.2f} max {max(cold):2d} |"]
        for r in rules:
            its = []
            for e, p in enumerate(probs):
                st = state[r][e]
                init = None if (st is None or r == "cold") else warm_init(p[2], p[3], st[0], st[1], r)
                y, it, ok = im.ipm(*p[:4], eps_mu=1e-6, max_iter=50, variant=KERNEL, init=init)
                state[r][e] = (y, im.FINAL["lam"].copy())
                its.append(it)
            its = np.array(its)
            line.append(f"{r}: mean {its.mean():5.2f} p99 {np.percentile(its, 99):4.1f} max {its.max():2d}")
        print(" ".join(line), flush=True)


if __name__ == "__main__":
    main()
