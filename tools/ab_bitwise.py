"""A/B bitwise check of the cold solve's torques between builds of libosc_batch.so (raw ctypes, as
tools/ab_time.py).  Diagnostic only.   python tools/ab_bitwise.py lib1.so lib2.so [...]"""
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

CASES = (("unitree_go2", 4096, "standing", "ones"), ("unitree_go2", 8192, "tumbling", "bernoulli"),
         ("walter_sr", 4096, "standing", "ones"), ("walter_sr", 8192, "tumbling", "bernoulli"),
         ("unitree_go2", 65536, "standing", "ones"))


def solve(path, robot, nenv, sc, mk):
    L = ctypes.CDLL(path)
    vp = ctypes.c_void_p
    L.osc_batch_solve.argtypes = [vp, ctypes.c_int32] + [vp] * 10 + [vp, ctypes.c_size_t, vp]
    d = OscModelDesc()
    assert L.osc_desc_from_yaml(robot.encode(), config_path(robot).encode(), ctypes.byref(d)) == 0
    h = vp()
    assert L.osc_model_create(ctypes.byref(d), ctypes.byref(h)) == 0
    nb = ctypes.c_size_t()
    L.osc_workspace_bytes(h, nenv, ctypes.byref(nb))
    g = generate(robot, nenv, SEED_BASE + 3, sc, mk)
    t = [torch.from_numpy(g[k]).cuda().contiguous() for k in ("M", "C", "J", "b", "T", "mask")]
    nu = {"unitree_go2": 12, "walter_sr": 8}[robot]
    tau = torch.empty((nenv, nu), dtype=torch.float64, device="cuda")
    st = torch.empty((nenv,), dtype=torch.int32, device="cuda")
    it = torch.empty((nenv,), dtype=torch.int32, device="cuda")
    ws = torch.empty((nb.value // 8 + 2,), dtype=torch.float64, device="cuda")
    p = [vp(x.data_ptr()) for x in t]
    rc = L.osc_batch_solve(h, nenv, *p, vp(tau.data_ptr()), None, vp(st.data_ptr()),
                           vp(it.data_ptr()), vp(ws.data_ptr()), ctypes.c_size_t(ws.numel() * 8),
                           vp(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    return tau.cpu(), st.cpu(), it.cpu()


libs = sys.argv[1:]
for case in CASES:
    res = [solve(p, *case) for p in libs]
    t0, s0, i0 = res[0]
    for p, (t, s, i) in zip(libs[1:], res[1:]):
        diff = (t - t0).abs().max().item()
        nrm = t0.abs().max().item()
        print(json.dumps({"case": case, "lib": p[-40:], "bitwise": bool(torch.equal(t, t0)),
                          "max_abs_diff": diff, "rel": diff / max(nrm, 1.0),
                          "iters_equal": bool(torch.equal(i, i0)),
                          "unconverged": int((s != 0).sum())}), flush=True)
