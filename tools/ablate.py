"""Diagnostic: kernel time vs interior-point iteration cap (setup cost vs per-iteration cost).
Not a benchmark line; prints one JSON object per configuration."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import torch  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402


def time_kernel(solver, inputs, out, reps=10):
    for _ in range(3):
        solver.solve_into(out, *inputs)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        solver.solve_into(out, *inputs)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for robot, nenv in [("unitree_go2", 4096), ("unitree_go2", 65536), ("walter_sr", 4096)]:
    d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    for mi in [0, 1, 2, 4, 8, 40]:
        s = OSCBatchSolver(robot, max_iter=mi)
        inputs = s.prepare(**d)
        out = s.alloc_outputs(nenv)
        ms = time_kernel(s, inputs, out)
        it = float(out.iters.double().mean())
        print(json.dumps({"robot": robot, "nenv": nenv, "max_iter": mi, "ms": round(ms, 4),
                          "mean_iters": it, "us_per_env_wave": None}), flush=True)
