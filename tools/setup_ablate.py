"""Diagnostic: osc_batch_assemble (setup kernel) time per phase, from libraries built with
-DOSC_SETUP_STOP=n (stop after phase A/B/C) vs the full library."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
lib = sys.argv[1]
os.environ["OSC_LIB_PATH"] = lib
import torch  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

for robot, nenv in [("unitree_go2", 4096), ("unitree_go2", 65536), ("walter_sr", 4096)]:
    s = OSCBatchSolver(robot)
    d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv)
    for _ in range(3):
        s.assemble_into(out, *args)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        s.assemble_into(out, *args)
    b.record()
    torch.cuda.synchronize()
    print(json.dumps({"lib": os.path.basename(lib), "robot": robot, "nenv": nenv,
                      "assemble_ms": round(a.elapsed_time(b) / 20, 4)}), flush=True)
