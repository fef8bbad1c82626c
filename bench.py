#!/usr/bin/env python
"""Benchmark: batched OSC control steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W] [--robot unitree_go2] [--nenv-per-gpu 4096]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One "step" = one pass of the hot path over one batch: for every environment the QP assembly
+ QP solve + torque slice (the reference's update_optimization_data + update_optimization +
solve_optimization, operational_space_controller.h:457-573), from post-kinematics inputs that
are already resident in HBM when the timed region starts.  MuJoCo kinematics is excluded (as on
the CPU side).  Default workload = BASELINE configs[1]: Unitree Go2 (nv 18, nu 12, 4 feet),
4096 envs per GPU, synthetic seeded inputs (osc_amd.synth; no robot XML offline).  Environments
are independent: each rank solves its own shard, no collective on the data path
("scaling": "weak").  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "operational-space-control_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from osc_amd.robots import bytes_per_solve, dims  # noqa: E402
from osc_amd.synth import SEED_BASE, generate, random_walk  # noqa: E402

METRIC = "OSC control steps/sec (batched envs), Go2 18-DoF, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X spec sheet FP64 (vector = dense matrix); not in the guides


def algorithmic_flops(robot: str, iters: float) -> float:
    """F0 + K * F_it of the reference formulation (n = nv+nu+3nc, m = nv+4nc+n)."""
    d = dims(robot)
    s, nv, n, m, nc = d["s"], d["nv"], d["n"], d["m"], d["nc"]
    f0 = 2 * s * nv * nv + 2 * s * nv + n * n * nv + n ** 3 / 3
    fit = 2 * n * n + 4 * nv * n + 24 * nc + 10 * (n + m)
    return f0 + iters * fit


def cpu_baseline(robot: str, seconds: float) -> dict:
    """Reference CPU path restated (oracle/osc_ref_port.c: CasADi-equivalent assembly + OSQP
    0.6.3 ADMM, warm start) on ONE host core: a single environment ticking through a 1 %
    random walk of its inputs, no 500 Hz sleep."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    from ref_port import RefPort  # checker / baseline only
    rng = np.random.default_rng(SEED_BASE)
    d = generate(robot, 1, SEED_BASE + 1, "standing", "ones")
    ticks = [d]
    for _ in range(63):
        ticks.append(random_walk(ticks[-1], rng))
    inputs = [[t[k][0] for k in ("M", "C", "J", "b", "T", "mask")] for t in ticks]
    port = RefPort(robot)
    for a in inputs[:4]:
        port.step(*a)
    n, iters, t0 = 0, 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, it = port.step(*inputs[n % len(inputs)])
        iters += it
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"{robot} single env, {n} warm-started ticks over a 64-tick 1% random walk "
                      f"in {dt:.1f} s on 1 host core (mean {iters / max(n, 1):.0f} ADMM iters/tick)"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--robot", default="unitree_go2")
    ap.add_argument("--nenv-per-gpu", type=int, default=4096)
    ap.add_argument("--scenario", default="standing", choices=["standing", "tumbling"])
    ap.add_argument("--mask", default="ones", choices=["ones", "bernoulli"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    from osc_amd.solver import OSCBatchSolver
    nenv = args.nenv_per_gpu
    solver = OSCBatchSolver(args.robot)
    d = generate(args.robot, nenv, SEED_BASE + 2 + 1000 * rank, args.scenario, args.mask)
    inputs = solver.prepare(**d)
    out = solver.alloc_outputs(nenv)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        solver.solve_into(out, *inputs)
    torch.cuda.synchronize()

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        solver.solve_into(out, *inputs)
        ev[k][1].record(stream)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps

    st = out.status.cpu().numpy()
    mean_iters = float(out.iters.double().mean().item())
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])
        c = torch.tensor([float((st == 0).sum()), float(st.size)], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(c)
        converged = float(c[0] / c[1])
    else:
        converged = float((st == 0).mean())

    if rank == 0:
        total = nenv * world
        value = total * args.steps / elapsed
        bps = bytes_per_solve(args.robot)
        achieved = bps * nenv / (kernel_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            with open(args.traffic_json) as fh:
                tj = json.load(fh)
            if tj.get("robot") == args.robot and tj.get("nenv") == nenv:
                traffic = tj.get("bytes_per_launch")
        flops = algorithmic_flops(args.robot, mean_iters)
        tflops = flops * nenv / (kernel_ms * 1e-3) / 1e12
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded post-kinematics M, C, J, b, T, mask; osc_amd.synth)",
            "config": {"workload": f"{args.robot} {args.scenario} mask={args.mask}, "
                                   f"{nenv} envs per GPU (BASELINE configs[1])",
                       "robot": args.robot, "envs_per_gpu": nenv, "global_envs": total,
                       "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_solve": bps, "kernel_ms": kernel_ms},
            "roofline_fp64": {"achieved": tflops, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                              "frac": tflops / FP64_PEAK_TFLOPS,
                              "flops_per_solve": flops, "mean_ipm_iters": mean_iters},
            "converged_frac": converged,
        }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args.robot, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
