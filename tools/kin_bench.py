"""Time the kinematics front end (osc_batch_kinematics) alone: HIP events over K launches.
    python tools/kin_bench.py [--steps 50]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "operational-space-control_amd"))
import torch  # noqa: E402

from osc_amd.kinematics import KinematicsBatch, load_tree, random_states  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    for robot, nenv in (("unitree_go2", 4096), ("unitree_go2", 65536), ("walter_sr", 4096),
                        ("walter_sr", 65536)):
        tree = load_tree(robot)
        kb = KinematicsBatch(tree=tree)
        q, v = random_states(tree, nenv, 1, joint_range=0.5)
        q, v = torch.from_numpy(q).cuda(), torch.from_numpy(v).cuda()
        out = kb.alloc(nenv)
        for _ in range(5):
            kb.compute_into(out, q, v)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(args.steps):
            kb.compute_into(out, q, v)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.steps
        nb = 8 * (kb.nq + kb.nv + kb.nv ** 2 + kb.nv + 6 * kb.ns * kb.nv + 6 * kb.ns)
        print(json.dumps({"robot": robot, "nenv": nenv, "ms": round(ms, 5),
                          "GBs": round(nb * nenv / ms / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
