"""Diagnostic (GPU): round 5's first AB_WARM perturbed batch -- a 1 % elementwise perturbation
of M (symmetrised: ~1 % of the WaLTER M come out indefinite or near-singular), C, J, b, T of the
SEED_BASE + 2 standing batch -- solved COLD: statuses, iterations, and the inputs of every env
not OK saved to gpurun_out/perturbed_<robot>.npz for the CPU oracle.

    python tools/perturbed_diag.py [robot] [nenv]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "walter_sr"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
g = generate(robot, nenv, SEED_BASE + 2)
t = [torch.from_numpy(g[k]).cuda().contiguous() for k in ("M", "C", "J", "b", "T", "mask")]
gen = torch.Generator(device="cuda").manual_seed(5)
t2 = [x if i == 5 else (x * (1.0 + 0.01 * torch.randn(x.shape, generator=gen, device="cuda",
                                                       dtype=x.dtype))).contiguous()
      for i, x in enumerate(t)]
t2[0] = (0.5 * (t2[0] + t2[0].transpose(1, 2))).contiguous()
for tune in ({}, {"refine_steps": 0}):
    s = OSCBatchSolver(robot, tuning=tune)
    out = s.alloc_outputs(nenv, want_x=True)
    s.solve_into(out, *s.prepare(*t2))
    torch.cuda.synchronize()
    st, it = out.status.cpu().numpy(), out.iters.cpu().numpy()
    bad = np.nonzero(st != 0)[0]
    print(json.dumps({"robot": robot, "tuning": tune, "counts": np.bincount(st).tolist(),
                      "bad": bad[:40].tolist(), "status": st[bad[:40]].tolist(),
                      "iters": it[bad[:40]].tolist(),
                      "min_eig_M": float(torch.linalg.eigvalsh(t2[0]).min().item())}), flush=True)
    if not tune and len(bad):
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        np.savez(os.path.join(REPO, "gpurun_out", f"perturbed_{robot}.npz"), envs=bad,
                 status=st[bad], iters=it[bad], x=out.x.cpu().numpy()[bad],
                 **{k: v.cpu().numpy()[bad] for k, v in zip(("M", "C", "J", "b", "T", "mask"), t2)})
