"""Diagnostic: run a synthetic batch on the GPU and save the inputs of every environment that
did not converge (status != 0) to gpurun_out/stalls_<robot>_<nenv>.npz."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
import numpy as np  # noqa: E402
from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402

robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 2
scenario = sys.argv[4] if len(sys.argv) > 4 else "standing"
mask = sys.argv[5] if len(sys.argv) > 5 else "ones"
tag = f"{robot}_{nenv}_{seed}_{scenario}_{mask}"
d = generate(robot, nenv, SEED_BASE + seed, scenario, mask)
s = OSCBatchSolver(robot)
r = s.solve(**d, want_x=True)
st = r.status.cpu().numpy()
it = r.iters.cpu().numpy()
bad = np.where((st != 0) | (it >= 20))[0]
print(tag, "mean_it", round(float(it.mean()), 2), "max_it", int(it.max()), "hard", len(bad), "unconverged", np.where(st != 0)[0].tolist(),
      flush=True)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", f"stalls_{tag}.npz"), idx=bad,
         x=r.x.cpu().numpy()[bad], **{k: v[bad] for k, v in d.items()})
