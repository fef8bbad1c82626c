"""Diagnostic: per-phase cycle shares of the IPM kernel from the OSC_STAMPS build
(lib/libosc_batch_stamps.so).  Stamps serialise the wave, so read SHARES, not absolute time.

    python tools/stamps.py [nenv] [robot ...]     (robots: unitree_go2 walter_sr noslip)"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["OSC_LIB_PATH"] = os.environ.get("OSC_STAMPS_LIB") or os.path.join(
    REPO, "operational-space-control_amd", "lib", "libosc_batch_stamps.so")
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from osc_amd import _lib  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

NAMES = ["stage+rows", "iter-head(Gy,mu,D)", "assemble: contact blocks", "LDL^T",
         "rhs (2 passes)", "solve (2 passes)", "Gdy+ratio+reduce (2 passes)", "update",
         "assemble: rd = g + G'lam + Hr y", "assemble: rank-1 U terms",
         "refine: K_A + LDL", "refine: steps"]
for robot in (sys.argv[2:] or ["unitree_go2", "walter_sr"]):
    nenv = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    if robot == "noslip":   # the opt-in wheel rows, 2,048-env-census shape (tumbling, Bernoulli)
        from osc_amd.robots import config_path
        from osc_amd.synth import WALTER_WHEEL_DOFS, WHEEL_RADIUS, wheel_directions
        yaml = os.path.join(os.path.dirname(config_path("walter_sr_wheels")),
                            "walter_sr_wheels_noslip_config.yaml")
        s = OSCBatchSolver("walter_sr_wheels", yaml)
        d = generate("walter_sr_wheels", nenv, SEED_BASE + 86, "tumbling", "bernoulli")
        wd = torch.from_numpy(wheel_directions("walter_sr_wheels", d, WALTER_WHEEL_DOFS,
                                               np.full(8, WHEEL_RADIUS), SEED_BASE + 87)).cuda()
    else:
        s = OSCBatchSolver(robot)
        d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
        wd = None
    args = s.prepare(**d)
    out = s.alloc_outputs(nenv)
    if wd is None:
        s.solve_into(out, *args)
    else:
        s.solve_into(out, *args, wheel_dir=wd)
    torch.cuda.synchronize()
    nblk = nenv // 4
    buf = (ctypes.c_ulonglong * (nblk * len(NAMES)))()
    L = _lib.lib()
    L.osc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert L.osc_debug_stamps(ctypes.cast(buf, ctypes.c_void_p), nblk) == 0
    raw = np.frombuffer(buf, dtype=np.uint64).reshape(nblk, len(NAMES)).copy()
    rounds = (raw[:, 10] >> np.uint64(40)).astype(np.int64)   # refinement rounds per wave
    raw[:, 10] &= np.uint64((1 << 40) - 1)
    a = raw.astype(np.float64)
    it = out.iters.cpu().numpy().reshape(nblk, 4).max(axis=1) + 1   # + init pass
    tot = a.sum(axis=1)
    ipm = a[:, :10].sum(axis=1)
    per = {n: float(a[:, k].mean()) for k, n in enumerate(NAMES)}
    slow = int(np.argmax(tot))
    print(json.dumps({"robot": robot, "mean_cycles_per_wave": float(tot.mean()),
                      "mean_wave_iters": float(it.mean()),
                      "cycles_per_wave_iter": float((ipm / it).mean()),
                      "refine_rounds_hist": np.bincount(rounds).tolist(),
                      "slowest_wave": {"cycles": float(tot[slow]), "iters": int(it[slow]),
                                       "refine_rounds": int(rounds[slow]),
                                       "refine_cycles": float(a[slow, 10] + a[slow, 11])},
                      "refine_cycles_per_round": float((a[:, 10] + a[:, 11]).sum() /
                                                       max(rounds.sum(), 1)),
                      "share": {n: round(per[n] / tot.mean(), 3) for n in NAMES}}), flush=True)
