"""Diagnostic (GPU box): wall time per step of the Go2 4,096 cold solve with 0, 1 or 3 HIP events
per step, split or fused C-ABI calls.  python tools/event_overhead.py"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import torch  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

s = OSCBatchSolver("unitree_go2")
d = generate("unitree_go2", 4096, SEED_BASE, "standing", "ones")
inp = s.prepare(**d)
out = s.alloc_outputs(4096)
K = 50


def run(mode):
    for _ in range(5):
        s.solve_into(out, *inp)
    torch.cuda.synchronize()
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    t0 = time.perf_counter()
    for k in range(K):
        if mode == "fused0":
            s.solve_into(out, *inp)
        elif mode == "split0":
            s.assemble_into(out, *inp[:5], inp[5])
            s.solve_assembled_into(out, inp[5])
        elif mode == "split1":
            ev[k][0].record()
            s.assemble_into(out, *inp[:5], inp[5])
            s.solve_assembled_into(out, inp[5])
        elif mode == "split3":
            ev[k][0].record()
            s.assemble_into(out, *inp[:5], inp[5])
            ev[k][1].record()
            s.solve_assembled_into(out, inp[5])
            ev[k][2].record()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / K * 1e3


for rep in range(2):
    for m in ("fused0", "split0", "split1", "split3"):
        print(m, round(run(m), 4), "ms/step", flush=True)
