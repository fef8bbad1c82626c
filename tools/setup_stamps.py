"""Diagnostic: per-phase cycles of the setup kernel from the OSC_STAMPS build
(lib/libosc_batch_stamps.so, or $OSC_STAMPS_LIB): mean over waves and the slowest wave.
    python tools/setup_stamps.py [nenv] [robot ...]   (robots: unitree_go2 walter_sr noslip)"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["OSC_LIB_PATH"] = os.environ.get("OSC_STAMPS_LIB") or os.path.join(REPO, "operational-space-control_amd", "lib",
                                          "libosc_batch_stamps.so")
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from osc_amd import _lib  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

NAMES = ["A: stage inputs", "B: Ha = 2[J e]'W[J e]", "C: X, U (base block) [WH: + X^ = X'T]",
         "D1: T1", "D2: Hr | g", "write workspace", "C2: factor S", "C2: solve",
         "C2: x_b + write", "WH: rows V, Q, X - V'P", "WH: basis T (Gram-Schmidt)"]
SLOTS = 12
nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for robot in (sys.argv[2:] or ["unitree_go2", "walter_sr"]):
    wd = None
    if robot == "noslip":   # the opt-in wheel rows (tools/wheel_census.py's batch shape)
        from osc_amd.robots import config_path
        from osc_amd.synth import WALTER_WHEEL_DOFS, WHEEL_RADIUS, wheel_directions
        yaml = os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                            "walter_sr_wheels_noslip_config.yaml")
        s = OSCBatchSolver("walter_sr_wheels", yaml)
        d = generate("walter_sr_wheels", nenv, SEED_BASE + 86, "tumbling", "bernoulli")
        wd = torch.from_numpy(wheel_directions("walter_sr_wheels", d, np.array(WALTER_WHEEL_DOFS),
                                               np.full(8, WHEEL_RADIUS), SEED_BASE + 87)).cuda()
    else:
        s = OSCBatchSolver(robot)
        d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv)
    for _ in range(2):
        if wd is None:
            s.assemble_into(out, *args)
        else:
            s.solve_into(out, *args, wheel_dir=wd)
    torch.cuda.synchronize()
    nw = nenv
    buf = (ctypes.c_ulonglong * (nw * SLOTS))()
    L = _lib.lib()
    L.osc_debug_setup_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.osc_debug_setup_stamps(ctypes.cast(buf, ctypes.c_void_p), nw) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nw, SLOTS)[:, :len(NAMES)].astype(np.float64)
    tot = a.sum(axis=1)
    print(json.dumps({"robot": robot, "nenv": nenv, "mean_cycles": round(float(tot.mean())),
                      "max_cycles": round(float(tot.max())),
                      "mean": {n: round(float(a[:, k].mean())) for k, n in enumerate(NAMES)}}),
          flush=True)
