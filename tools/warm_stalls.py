"""Diagnostic: warm-started ticks over the bench's 1 % random walk (bench.py warm_ticks); dumps
every env that does not converge (inputs of that tick + the warm state it started from) to
gpurun_out/warm_stalls_<robot>.npz.
    python tools/warm_stalls.py [robot] [nenv] [cycles] [scenario] [mask]
mask "bernoulli" redraws a Bernoulli(0.75) contact mask every tick (contact-mode switching)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "walter_sr"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
cycles = int(sys.argv[3]) if len(sys.argv) > 3 else 4
scenario = sys.argv[4] if len(sys.argv) > 4 else "standing"
mask_mode = sys.argv[5] if len(sys.argv) > 5 else "ones"
solver = OSCBatchSolver(robot)
inputs = solver.prepare(**generate(robot, nenv, shard_seed(0), scenario, mask_mode))
g = torch.Generator(device=inputs[0].device).manual_seed(shard_seed(0) + 7)
nv = inputs[0].shape[1]
eye = torch.eye(nv, dtype=torch.float64, device=inputs[0].device)
seq = [inputs]
for _ in range(9):
    new = []
    for i, t in enumerate(seq[-1]):
        if i == 5:
            new.append(t)
            continue
        if i == 0:   # M: congruence A M A' keeps it SPD (osc_amd.synth.random_walk)
            A = eye + 0.01 / nv ** 0.5 * torch.randn(t.shape, generator=g, device=t.device,
                                                     dtype=t.dtype)
            w = A @ t @ A.transpose(1, 2)
            w = 0.5 * (w + w.transpose(1, 2))
        else:
            w = t * (1.0 + 0.01 * torch.randn(t.shape, generator=g, device=t.device,
                                              dtype=t.dtype))
        new.append(w.contiguous())
    seq.append(tuple(new))
order = list(range(10)) + list(range(8, 0, -1))
warm = solver.alloc_warm_state(nenv)
out = solver.alloc_outputs(nenv, want_x=True)
dump = []
for k in range(cycles * len(order)):
    before = warm.clone()
    args = seq[order[k % len(order)]]
    if mask_mode == "bernoulli":
        m = (torch.rand(args[5].shape, generator=g, device=args[5].device) < 0.75).double()
        args = args[:5] + (m,)
    solver.solve_warm_into(out, warm, *args)
    st = out.status.cpu().numpy()
    bad = np.nonzero(st != 0)[0]
    its = out.iters.cpu().numpy()
    fix = np.nonzero(its > solver.desc.max_iter)[0]   # re-solved by the fix-up pass (max_iter + cold)
    print(f"tick {k}: mean_it {its.mean():.2f} max_it {its.max()} bad {bad.tolist()} "
          f"fixed_up {fix.tolist()}", flush=True)
    per = before.numel() // nenv
    for e in list(bad[:8]) + list(fix[:4]):
        dump.append(dict(tick=k, env=int(e), warm=before.view(nenv, per)[e].cpu().numpy(),
                         **{n: a[e].cpu().numpy() for n, a in zip(("M", "C", "J", "b", "T", "mask"), args)}))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
if dump:
    np.savez(os.path.join(REPO, "gpurun_out", f"warm_stalls_{robot}.npz"),
             **{f"{i}_{k}": v for i, d in enumerate(dump) for k, v in d.items()})
print("dumped", len(dump))
