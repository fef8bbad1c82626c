"""Throughput of one GPU's env shard split into G groups, each group's ticks in order on its own
stream (tick k+1 of a group after tick k of that group; groups independent), so one group's
assembly can fill the SIMDs another group's interior-point straggler tail leaves idle.

    python tools/stagger_probe.py [robot] [nenv] [steps]

Prints one JSON line per G in (1, 2, 4) and mode: "free" (each group's stream runs ahead: group
g's tick k+1 may overlap group h's tick k) or "joined" (every step forks from and joins one
stream: all envs of step k done before step k+1 starts -- the semantics of ONE call): ms per step
(every env solved once), solves/s, and whether each group's torques equal the single-call solve
of its envs (bitwise).  Diagnostic.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import torch  # noqa: E402

from osc_amd.solver import OSCBatchSolver  # noqa: E402
from osc_amd.synth import SEED_BASE, generate  # noqa: E402


def main():
    robot = sys.argv[1] if len(sys.argv) > 1 else "unitree_go2"
    nenv = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    s = OSCBatchSolver(robot)
    d = generate(robot, nenv, SEED_BASE + 2, "standing", "ones")
    full = s.prepare(**d)
    ref = s.alloc_outputs(nenv)
    s.solve_into(ref, *full)
    torch.cuda.synchronize()
    for G, mode in ((1, "free"), (2, "free"), (4, "free"), (2, "joined"), (4, "joined")):
        per = nenv // G
        groups = []
        for g in range(G):
            sl = slice(g * per, (g + 1) * per)
            inp = tuple(t[sl].contiguous() for t in full)
            groups.append((torch.cuda.Stream(), inp, s.alloc_outputs(per)))
        main = torch.cuda.current_stream()

        def step():
            for st, inp, out in groups:
                if mode == "joined":
                    st.wait_stream(main)
                s.solve_into(out, *inp, stream=st)
            if mode == "joined":
                for st, _, _ in groups:
                    main.wait_stream(st)

        for _ in range(20):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        same = all(torch.equal(out.tau, ref.tau[g * per:(g + 1) * per])
                   for g, (_, _, out) in enumerate(groups))
        print(json.dumps({"robot": robot, "nenv": nenv, "groups": G, "mode": mode, "ms_per_step": el / steps * 1e3,
                          "solves_per_s": nenv * steps / el, "bitwise_vs_one_call": same}),
              flush=True)


if __name__ == "__main__":
    main()
