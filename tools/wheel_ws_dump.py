"""Diagnostic (GPU): the wheel model's assembled workspace (setup_env output) for a few envs, with
the inputs, to an npz for a CPU-side comparison against a numpy restatement.

    python tools/wheel_ws_dump.py [out.npz] [scenario] [seed] [nenv] [env,env,...]
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))

import torch  # noqa: E402

from osc_amd.robots import config_path  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, WALTER_WHEEL_DOFS, WHEEL_RADIUS, generate, wheel_directions  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wheel_ws.npz"
scen = sys.argv[2] if len(sys.argv) > 2 else "standing"
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 81
nenv = int(sys.argv[4]) if len(sys.argv) > 4 else 8
keep = [int(a) for a in sys.argv[5].split(",")] if len(sys.argv) > 5 else list(range(nenv))
YAML = os.path.join(os.path.dirname(config_path("walter_sr_wheels")), "walter_sr_wheels_noslip_config.yaml")
d = generate("walter_sr_wheels", nenv, SEED_BASE + seed, scen, "ones" if scen == "standing" else "bernoulli")
wd = wheel_directions("walter_sr_wheels", d, np.array(WALTER_WHEEL_DOFS), np.full(8, WHEEL_RADIUS),
                      SEED_BASE + seed + 1)
s = OSCBatchSolver("walter_sr_wheels", YAML)
args = s.prepare(**d)
res = s.alloc_outputs(nenv, want_x=True)
s.assemble_into(res, *args[:5], args[5], wheel_dir=torch.from_numpy(wd).cuda())
torch.cuda.synchronize()
WSD = res.workspace.numel() // nenv
def pick(wsv):
    return np.concatenate([wsv[e * WSD:(e + 1) * WSD] for e in keep])
ws_asm = pick(res.workspace.cpu().numpy())
s.solve_into(res, *args, wheel_dir=torch.from_numpy(wd).cuda())
torch.cuda.synchronize()
np.savez(out, keep=np.array(keep), ws_asm=ws_asm, ws=pick(res.workspace.cpu().numpy()),
         x=res.x.cpu().numpy()[keep], tau=res.tau.cpu().numpy()[keep],
         status=res.status.cpu().numpy()[keep], iters=res.iters.cpu().numpy()[keep], wd=wd[keep],
         **{k: np.asarray(v)[keep] for k, v in d.items()})
print("status", res.status.cpu().numpy()[keep].tolist(), "iters", res.iters.cpu().numpy()[keep].tolist())
