"""Lockstep compaction A/B (ParkArgs in csrc/osc_batch.hip): for each park iteration, the cold
solve's time per launch (HIP events, median of the timed launches) and a bitwise comparison of
tau / x / status / iters with compaction off (osc_model_tuning.park_it = 0).

    python tools/park_sweep.py ROBOT NENV SCENARIO MASK PARK_IT[,PARK_IT...] [REPS]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "operational-space-control_amd"))
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import generate  # noqa: E402
from osc_amd.dist import shard_seed  # noqa: E402

robot, nenv, scen, mask = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
parks = [int(p) for p in sys.argv[5].split(",")]
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 20
d = generate(robot, nenv, shard_seed(0), scen, mask)


def run(park):
    s = OSCBatchSolver(robot, tuning={"park_it": park})
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv, want_x=True)
    for _ in range(3):
        s.solve_into(out, *args)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        s.solve_into(out, *args)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return out, float(np.median(ts))


base, t0 = run(0)
it = base.iters.cpu().numpy()
res = {"robot": robot, "nenv": nenv, "scenario": scen, "mask": mask, "off_ms": t0,
       "mean_iters": float(it.mean()), "mean_wave_iters": float(it.reshape(-1, 4).max(1).mean()),
       "runs": []}
for p in parks:
    out, t = run(p)
    same = all(torch.equal(getattr(base, k), getattr(out, k)) for k in ("tau", "x", "status", "iters"))
    res["runs"].append({"park_it": p, "ms": t, "speedup": t0 / t, "bitwise": same,
                        "parked_frac": float((it > p).mean())})
    print(json.dumps(res["runs"][-1]), file=sys.stderr, flush=True)
print(json.dumps(res))
