"""A/B kernel timing of the cold solve for builds of libosc_batch.so given on the command line
(raw ctypes: only osc_desc_from_yaml / osc_model_create / osc_workspace_bytes / osc_batch_solve,
so older builds load too).  Diagnostic only.
    python tools/ab_time.py lib1.so [lib2.so ...]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import torch  # noqa: E402

from osc_amd._lib import OscModelDesc  # noqa: E402
from osc_amd.robots import config_path  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402


def run(path):
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.osc_batch_solve.argtypes = [vp, ctypes.c_int32] + [vp] * 10 + [vp, ctypes.c_size_t, vp]
    only = os.environ.get("AB_ONLY")   # e.g. "unitree_go2:4096" (one configuration, for rocprof)
    for robot, nenv in (("unitree_go2", 4096), ("unitree_go2", 65536), ("walter_sr", 4096)):
        if only and only != f"{robot}:{nenv}":
            continue
        d = OscModelDesc()
        assert L.osc_desc_from_yaml(robot.encode(), config_path(robot).encode(), ctypes.byref(d)) == 0
        h = vp()
        assert L.osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 0
        nb = ctypes.c_size_t()
        L.osc_workspace_bytes(h, nenv, ctypes.byref(nb))
        g = generate(robot, nenv, SEED_BASE + 2)
        t = [torch.from_numpy(g[k]).cuda().contiguous() for k in ("M", "C", "J", "b", "T", "mask")]
        nu = {"unitree_go2": 12, "walter_sr": 8}[robot]
        tau = torch.empty((nenv, nu), dtype=torch.float64, device="cuda")
        ws = torch.empty((nb.value // 8 + 2,), dtype=torch.float64, device="cuda")
        p = [vp(x.data_ptr()) for x in t]

        def call():
            rc = L.osc_batch_solve(h, nenv, *p, vp(tau.data_ptr()), None, None, None,
                                   vp(ws.data_ptr()), ctypes.c_size_t(ws.numel() * 8),
                                   vp(torch.cuda.current_stream().cuda_stream))
            assert rc == 0
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(30):
            call()
        b.record()
        torch.cuda.synchronize()
        print(json.dumps({"lib": path[-45:], "robot": robot, "nenv": nenv,
                          "ms": round(a.elapsed_time(b) / 30, 4)}), flush=True)


for p in sys.argv[1:]:
    run(p)
