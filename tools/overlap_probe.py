"""Diagnostic: does assembling chunk k+1 (setup kernel, side stream) while chunk k is in the
interior point (main stream) beat the serial fused solve at large batches?  Uses the split
C-ABI (osc_batch_assemble / osc_batch_solve_assembled) with torch streams and events.
    python tools/overlap_probe.py [robot] [nenv]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import torch  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
s = OSCBatchSolver(robot)
args = s.prepare(**generate(robot, nenv, SEED_BASE + 2))
main = torch.cuda.current_stream()
aux = torch.cuda.Stream()


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(main)
    for _ in range(reps):
        fn()
    b.record(main)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


full = s.alloc_outputs(nenv)
ref_ms = timed(lambda: s.solve_into(full, *args))
res = {"robot": robot, "nenv": nenv, "serial_ms": round(ref_ms, 4)}
for k in (2, 4, 8):
    n = nenv // k
    outs = [s.alloc_outputs(n) for _ in range(k)]
    sl = [[a[i * n:(i + 1) * n] for a in args] for i in range(k)]
    evs = [torch.cuda.Event() for _ in range(k)]

    def run():
        aux.wait_stream(main)
        for i in range(k):
            s.assemble_into(outs[i], *sl[i], stream=aux)
            evs[i].record(aux)
        for i in range(k):
            main.wait_event(evs[i])
            s.solve_assembled_into(outs[i], sl[i][5], stream=main)
    ms = timed(run)
    same = all(torch.equal(outs[i].tau, full.tau[i * n:(i + 1) * n]) for i in range(k))
    res[f"chunks{k}_ms"] = round(ms, 4)
    res[f"chunks{k}_bitwise_equal"] = same
print(json.dumps(res), flush=True)
