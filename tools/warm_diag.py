"""Diagnostic (GPU): the warm-started ticks of bench.py's warm line (Go2 4,096, 1 % random walk,
ping-pong) -- per tick the iteration histogram, the per-wave maximum (4 envs per wave), the envs
past max_iter (the cold fix-up pass) and the statuses.  Run under rocprofv3 --kernel-trace
--stats for the per-kernel split.

    python tools/warm_diag.py [robot] [nenv] [ticks] [pingpong]
(pingpong: tools/ab_time.py's AB_WARM inputs instead -- the batch and a 1 % elementwise-perturbed
copy, alternating)
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 18
solver = OSCBatchSolver(robot)
d = generate(robot, nenv, SEED_BASE + 1, "standing", "ones")
inputs = solver.prepare(*(torch.from_numpy(d[k]).cuda() for k in ("M", "C", "J", "b", "T", "mask")))
g = torch.Generator(device="cuda").manual_seed(SEED_BASE + 7)
nv = inputs[0].shape[1]
eye = torch.eye(nv, dtype=torch.float64, device="cuda")
seq = [inputs]
for _ in range(9):   # bench.py warm_ticks' walk
    new = []
    for i, t in enumerate(seq[-1]):
        if i == 5:
            new.append(t)
            continue
        if i == 0:
            A = eye + 0.01 / nv ** 0.5 * torch.randn(t.shape, generator=g, device="cuda", dtype=t.dtype)
            w = A @ t @ A.transpose(1, 2)
            w = 0.5 * (w + w.transpose(1, 2))
        else:
            w = t * (1.0 + 0.01 * torch.randn(t.shape, generator=g, device="cuda", dtype=t.dtype))
        new.append(w.contiguous())
    seq.append(tuple(new))
order = list(range(10)) + list(range(8, 0, -1))
if len(sys.argv) > 4 and sys.argv[4] == "pingpong":
    gen = torch.Generator(device="cuda").manual_seed(5)
    t2 = [x if i == 5 else (x * (1.0 + 0.01 * torch.randn(x.shape, generator=gen, device="cuda",
                                                           dtype=x.dtype))).contiguous()
          for i, x in enumerate(inputs)]
    # M by a congruence A M A' (SPD kept; an elementwise 1 % perturbation made ~1 % of the
    # WaLTER M indefinite or near-singular: unphysical QPs the reduction flags)
    nv = inputs[0].shape[1]
    A = torch.eye(nv, dtype=torch.float64, device="cuda") + 0.01 / nv ** 0.5 * torch.randn(
        inputs[0].shape, generator=gen, device="cuda", dtype=torch.float64)
    t2[0] = A @ inputs[0] @ A.transpose(1, 2)
    t2[0] = (0.5 * (t2[0] + t2[0].transpose(1, 2))).contiguous()
    seq = [inputs, tuple(t2)]
    order = [0, 1]
warm = solver.alloc_warm_state(nenv)
out = solver.alloc_outputs(nenv)
max_iter = 50
for k in range(ticks + len(order)):
    solver.solve_warm_into(out, warm, *seq[order[k % len(order)]])
    if k < len(order):
        continue
    torch.cuda.synchronize()
    it = out.iters.cpu().numpy()
    st = out.status.cpu().numpy()
    base = np.where(it > max_iter, it - max_iter, it)   # fix-up envs: max_iter + k
    wave = base.reshape(-1, 4).max(1)
    print(json.dumps({"tick": k, "step": order[k % len(order)], "mean": round(float(base.mean()), 3),
                      "max": int(base.max()), "p99": float(np.percentile(base, 99)),
                      "wave_max_mean": round(float(wave.mean()), 3),
                      "hist": np.bincount(base).tolist(), "fixup": int((it > max_iter).sum()),
                      "fallback": int((it < 0).sum()), "status": np.bincount(st).tolist()}), flush=True)
