"""Diagnostic (GPU): A/B of the joint-state tick (osc_batch_solve_qpos: kinematics + assembly +
interior point) between library builds -- e.g. the fused tick (kinematics in the assembly
kernel's prologue) against a -DOSC_NO_FUSED_TICK build (osc_batch_kinematics + osc_batch_solve).
Each library runs in its own child process (the ctypes binding loads one library per process),
rounds interleaved; HIP events over 30 ticks after 5.

    python tools/tick_ab.py lib1.so lib2.so ...      (TICK_CONFIGS="unitree_go2:4096,...",
                                                      TICK_ROUNDS=3)
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(configs):
    sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))
    import torch
    from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
    from osc_amd.solver import OSCBatchSolver
    from osc_amd.synth import generate
    for c in configs.split(","):
        robot, nenv = c.split(":")
        nenv = int(nenv)
        tree = load_tree(robot)
        kb, solver = KinematicsBatch(tree=tree), OSCBatchSolver(robot)
        q, v = random_states(tree, nenv, 11, joint_range=0.5)
        d = generate(robot, nenv, 11, "standing", "ones")
        q, v = torch.from_numpy(q).cuda(), torch.from_numpy(v).cuda()
        T, mask = torch.from_numpy(d["T"]).cuda(), torch.from_numpy(d["mask"]).cuda()
        out = solver.alloc_outputs(nenv)
        ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64,
                         device="cuda")
        for _ in range(5):
            kb.solve_into(solver, out, q, v, T, mask, ws)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(30):
            kb.solve_into(solver, out, q, v, T, mask, ws)
        e1.record(s)
        torch.cuda.synchronize()
        ok = int((out.status == 0).sum().item())
        print(json.dumps({"robot": robot, "nenv": nenv, "ms": round(e0.elapsed_time(e1) / 30, 5),
                          "ok": ok, "tau_sum": float(out.tau.sum().item())}), flush=True)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    configs = os.environ.get("TICK_CONFIGS", "unitree_go2:4096,unitree_go2:8192,"
                             "unitree_go2:65536,walter_sr:4096,walter_sr:65536")
    for r in range(int(os.environ.get("TICK_ROUNDS", "3"))):
        for lib in sys.argv[1:]:
            env = dict(os.environ, OSC_LIB_PATH=os.path.abspath(lib))
            out = subprocess.run([sys.executable, __file__, "--child", configs], env=env,
                                 capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(out.stderr[-2000:], file=sys.stderr)
                sys.exit(out.returncode)
            for line in out.stdout.splitlines():
                rec = json.loads(line)
                rec.update(lib=lib[-40:], round=r)
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
