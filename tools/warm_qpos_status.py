"""Diagnostic (GPU): the bench's joint-state warm control loop (bench.py front_end: 10 consecutive
Go2 states, replayed ping-pong, warm state carried) -- per tick the envs the cold fix-up pass
re-solved (iters > max_iter), the status counts and the largest warm iteration count.

    python tools/warm_qpos_status.py [nenv] [ticks]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "operational-space-control_amd"))
from osc_amd.kinematics import KinematicsBatch, load_tree, random_states  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402

nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ticks = int(sys.argv[2]) if len(sys.argv) > 2 else 36
robot, seed = "unitree_go2", shard_seed(0) + 7
solver = OSCBatchSolver(robot)
tree = load_tree(robot)
kb = KinematicsBatch(tree=tree)
qpos, qvel = random_states(tree, nenv, seed, joint_range=0.5)
qpos, qvel = torch.from_numpy(qpos).cuda(), torch.from_numpy(qvel).cuda()
d = generate(robot, nenv, seed, "standing", "ones")
T, mask = torch.from_numpy(d["T"]).cuda(), torch.from_numpy(d["mask"]).cuda()
out = solver.alloc_outputs(nenv)
ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64, device=qpos.device)
g = torch.Generator(device=qpos.device).manual_seed(seed + 11)
states = [(qpos, qvel)]
for _ in range(9):
    q, v = states[-1]
    q = q + 0.01 * torch.randn(q.shape, generator=g, device=q.device, dtype=q.dtype)
    q[:, 3:7] = q[:, 3:7] / q[:, 3:7].norm(dim=1, keepdim=True)
    q[:, 0:3] = 0.0
    v = v * (1.0 + 0.01 * torch.randn(v.shape, generator=g, device=v.device, dtype=v.dtype))
    states.append((q.contiguous(), v.contiguous()))
order = list(range(10)) + list(range(8, 0, -1))
warm = solver.alloc_warm_state(nenv)
mi = solver.desc.max_iter
for k in range(ticks):
    q, v = states[order[k % len(order)]]
    kb.solve_warm_into(solver, out, warm, q, v, T, mask, ws)
    torch.cuda.synchronize()
    it, st = out.iters.cpu().numpy(), out.status.cpu().numpy()
    fixed = np.nonzero(it > mi)[0]
    print(json.dumps({"tick": k, "status": np.bincount(st, minlength=4).tolist(),
                      "fixed_up": fixed[:8].tolist(), "n_fixed": int(len(fixed)),
                      "max_warm_it": int(it[it <= mi].max()), "mean_it": float(it.mean())}), flush=True)
