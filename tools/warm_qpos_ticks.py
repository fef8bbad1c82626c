"""Diagnostic: warm-started ticks from joint states (osc_batch_solve_qpos_warm) over the bench's
joint-space walk (bench.py front_end); per tick the iteration statistics.
    python tools/warm_qpos_ticks.py [robot] [nenv] [ticks]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.dist import shard_seed  # noqa: E402
from osc_amd.kinematics import KinematicsBatch, load_tree, random_states  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
ticks = int(sys.argv[3]) if len(sys.argv) > 3 else 36
seed = shard_seed(0)
tree = load_tree(robot)
kb = KinematicsBatch(tree=tree)
solver = OSCBatchSolver(robot)
q, v = random_states(tree, nenv, seed, joint_range=0.5)
q, v = torch.from_numpy(q).cuda(), torch.from_numpy(v).cuda()
d = generate(robot, nenv, seed, "standing", "ones")
T, mask = torch.from_numpy(d["T"]).cuda(), torch.from_numpy(d["mask"]).cuda()
out = solver.alloc_outputs(nenv)
ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64, device="cuda")
g = torch.Generator(device="cuda").manual_seed(seed + 11)
states = [(q, v)]
for _ in range(9):
    q0, v0 = states[-1]
    q1 = q0 + 0.01 * torch.randn(q0.shape, generator=g, device="cuda", dtype=q0.dtype)
    q1[:, 3:7] = q1[:, 3:7] / q1[:, 3:7].norm(dim=1, keepdim=True)
    q1[:, 0:3] = 0.0
    v1 = v0 * (1.0 + 0.01 * torch.randn(v0.shape, generator=g, device="cuda", dtype=v0.dtype))
    states.append((q1.contiguous(), v1.contiguous()))
order = list(range(10)) + list(range(8, 0, -1))
warm = solver.alloc_warm_state(nenv)
mi = solver.desc.max_iter
for k in range(ticks):
    qq, vv = states[order[k % len(order)]]
    kb.solve_warm_into(solver, out, warm, qq, vv, T, mask, ws)
    it = out.iters.cpu().numpy()
    st = out.status.cpu().numpy()
    print(f"tick {k}: mean {it.mean():.2f} max {it.max()} n>15 {(it > 15).sum()} "
          f"n>20 {(it > 20).sum()} fixup {(it > mi).sum()} bad {(st != 0).sum()} "
          f"worst {np.argsort(-it)[:3].tolist()}", flush=True)
