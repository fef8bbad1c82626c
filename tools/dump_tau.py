"""Diagnostic (GPU box): solve one seeded synthetic batch and save tau / iters / status to an npz
(for tools/hardest_envs.py, which finds the environments farthest from the exact oracle).
With a reference file from tools/ref_tau.py as 7th argument, the per-env errors against it are
saved instead of the torques (small enough to ship back from a sweep).
Usage: python tools/dump_tau.py robot scenario mask nenv seed_offset out.npz [ref.npz]"""
import json
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
tau = res.tau.cpu().numpy()
iters = res.iters.cpu().numpy()
status = res.status.cpu().numpy()
if len(sys.argv) > 7:
    refs = np.load(sys.argv[7])["tau"]
    nrm = np.maximum(np.abs(refs).max(axis=1, keepdims=True), 1.0)
    normwise = (np.abs(tau - refs) / nrm).max(axis=1)
    floor = 1e-2 * np.abs(refs).max(axis=1, keepdims=True)
    big = np.abs(refs) >= floor
    elem = np.where(big, np.abs(tau - refs) / np.maximum(np.abs(refs), 1e-300), 0.0).max(axis=1)
    lock = iters.reshape(-1, 4).max(axis=1) if iters.size % 4 == 0 else iters
    np.savez(out, normwise=normwise, elem=elem, iters=iters.astype(np.int16), status=status)
    print(json.dumps({"file": out, "max_normwise": float(normwise.max()),
                      "max_elem": float(elem.max()), "n_norm_gt_1e-6": int((normwise > 1e-6).sum()),
                      "worst": [int(i) for i in np.argsort(normwise)[::-1][:5]],
                      "mean_iters": float(iters.mean()), "max_iters": int(iters.max()),
                      "lockstep_mean": float(lock.mean()),
                      "unconverged": int((status != 0).sum())}))
else:
    np.savez(out, tau=tau, iters=iters, status=status)
    print("saved", out, "max iters", int(iters.max()), "unconverged", int((status != 0).sum()))
