"""How much of the interior point's kernel time a faster SOLO iteration could save (VERDICT r5
#5): per-env interior-point iteration counts of a cold solve and of warm-started ticks (1 % random
walk), grouped four envs to a wavefront as the kernel does.  A wave costs max(iters) lockstep
iterations; the last max - second_max of them have one env left ("solo").  If a solo iteration ran
s times faster, the wave would cost second + (max - second) / s; the kernel is set by its slowest
wave.  Prints one JSON line per batch.  Diagnostic (GPU).

    python tools/solo_tail.py [robot] [nenv]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate, random_walk  # noqa: E402


def model(iters, label):
    it = np.asarray(iters, dtype=float)
    it = np.where(it > 1000, it - 1000, it)   # (fix-up passes: none expected)
    w = np.sort(it.reshape(-1, 4), axis=1)
    mx, second = w[:, 3], w[:, 2]
    out = {"batch": label, "envs": int(it.size), "mean_iters": float(it.mean()),
           "max_iters": float(mx.max()), "slowest_wave_second": float(second[np.argmax(mx)]),
           "mean_wave_max": float(mx.mean()), "mean_solo_iters": float((mx - second).mean())}
    for s in (1.5, 2.0, 3.0, 4.0):
        cost = second + (mx - second) / s
        out[f"kernel_iters_solo_x{s:g}"] = float(cost.max())
    out["kernel_iters_now"] = float(mx.max())
    return out


def main():
    robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
    nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    s = OSCBatchSolver(robot)
    d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    out = s.alloc_outputs(nenv)
    s.solve_into(out, *s.prepare(**d))
    torch.cuda.synchronize()
    print(json.dumps(model(out.iters.cpu().numpy(), "cold")), flush=True)
    rng = np.random.default_rng(SEED_BASE + 9)
    seq = [d]
    for _ in range(9):
        seq.append(random_walk(seq[-1], rng))
    warm = s.alloc_warm_state(nenv)
    order = list(range(10)) + list(range(8, 0, -1))
    for k in range(3 * len(order)):
        s.solve_warm_into(out, warm, *s.prepare(**seq[order[k % len(order)]]))
        if k >= 2 * len(order) and k % 6 == 0:
            torch.cuda.synchronize()
            print(json.dumps(model(out.iters.cpu().numpy(), f"warm tick {k}")), flush=True)


if __name__ == "__main__":
    main()
