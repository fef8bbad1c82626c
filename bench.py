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

from osc_amd.dist import barrier as dist_barrier, job_value, rank_info, reduce_stats, shard_seed  # noqa: E402,E501
from osc_amd.robots import bytes_per_solve, dims  # noqa: E402
from osc_amd.synth import generate  # noqa: E402

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


def cpu_baseline(robot: str, seconds: float, cores: int) -> dict:
    """Reference CPU path restated (oracle/osc_ref_port.c: CasADi-equivalent assembly + OSQP
    0.6.3 ADMM, warm start): each worker process ticks ONE environment through a 1 % random
    walk of its inputs with no 500 Hz sleep (oracle/ref_port.py timed_ticks).  Run once on
    1 core, then `cores` independent workers at once."""
    import subprocess
    worker = [sys.executable, os.path.join(REPO, "oracle", "ref_port.py"), "--robot", robot,
              "--seconds", str(seconds)]

    def run(n):
        procs = [subprocess.Popen(worker + ["--seed", str(k)], stdout=subprocess.PIPE, text=True)
                 for k in range(n)]
        res = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in procs]
        if any(p.returncode != 0 for p in procs):
            raise RuntimeError("cpu baseline worker failed")
        return res

    one = run(1)[0]
    many = run(cores)
    rate1 = one["ticks"] / one["seconds"]
    rate = sum(r["ticks"] / r["seconds"] for r in many)
    iters = sum(r["admm_iters"] for r in many) / max(sum(r["ticks"] for r in many), 1)
    return {"value": rate, "unit": "solves/s", "cores": cores, "kind": "port",
            "single_core_value": rate1,
            "sample": f"{robot}: {cores} worker processes x 1 env each, warm-started ticks over a "
                      f"64-tick 1% random walk for {seconds:.0f} s (mean {iters:.0f} ADMM "
                      f"iters/tick); single core alone {rate1:.0f} solves/s"}


def front_end(robot: str, solver, nenv: int, steps: int, warmup: int, seed: int, stream) -> dict:
    """the GPU kinematics front end (osc_batch_kinematics: qpos/qvel ->
    M, C, J, b) and the whole tick from joint states (osc_batch_solve_qpos), timed with HIP
    events on the launch stream.  Not part of `value` (the headline excludes MuJoCo/kinematics
    on both sides)."""
    from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
    tree = load_tree(robot)
    kb = KinematicsBatch(tree=tree)
    qpos, qvel = random_states(tree, nenv, seed, joint_range=0.5)
    qpos = torch.from_numpy(qpos).cuda()
    qvel = torch.from_numpy(qvel).cuda()
    kout = kb.alloc(nenv)
    d = generate(robot, nenv, seed, "standing", "ones")
    T = torch.from_numpy(d["T"]).cuda()
    mask = torch.from_numpy(d["mask"]).cuda()
    out = solver.alloc_outputs(nenv)
    ws = torch.empty((kb.workspace_bytes(solver, nenv) // 8 + 2,), dtype=torch.float64,
                     device=qpos.device)

    def timed(fn):
        for _ in range(warmup):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    kin_ms = timed(lambda: kb.compute_into(kout, qpos, qvel))
    tick_ms = timed(lambda: kb.solve_into(solver, out, qpos, qvel, T, mask, ws))
    # the same QPs solved from their M, C, J, b (osc_batch_solve): the tick minus this is what the
    # kinematics front end adds -- joint-state QPs take more interior-point iterations than the
    # synthetic headline batch, so the headline's ms_per_step is not the comparison
    kq = kb.compute(qpos, qvel, want_sites=False)
    qargs = solver.prepare(kq.M, kq.C, kq.J, kq.b, T, mask)
    out_q = solver.alloc_outputs(nenv)
    solve_ms = timed(lambda: solver.solve_into(out_q, *qargs))
    # a control loop: 10 consecutive joint states (joint angles +-0.01 rad, velocities +-1 % per
    # step, base quaternion re-normalised), replayed ping-pong, warm state carried tick to tick
    g = torch.Generator(device=qpos.device).manual_seed(seed + 11)
    states = [(qpos, qvel)]
    for _ in range(9):
        q, v = states[-1]
        q = q + 0.01 * torch.randn(q.shape, generator=g, device=q.device, dtype=q.dtype)
        q[:, 3:7] = q[:, 3:7] / q[:, 3:7].norm(dim=1, keepdim=True)
        q[:, 0:3] = 0.0                                  # base position 0 (osc.h:358-359)
        v = v * (1.0 + 0.01 * torch.randn(v.shape, generator=g, device=v.device, dtype=v.dtype))
        states.append((q.contiguous(), v.contiguous()))
    order = list(range(10)) + list(range(8, 0, -1))
    warm = solver.alloc_warm_state(nenv)
    k = [0]

    def warm_tick():
        q, v = states[order[k[0] % len(order)]]
        kb.solve_warm_into(solver, out, warm, q, v, T, mask, ws)
        k[0] += 1
    for _ in range(len(order)):
        warm_tick()
    warm_ms = timed(warm_tick)
    nq, nv, ns = kb.nq, kb.nv, kb.ns
    kin_bytes = 8 * (nq + nv + nv * nv + nv + 6 * ns * nv + 6 * ns)
    gbs = kin_bytes * nenv / (kin_ms * 1e-3) / 1e9
    return {"kernel": "osc_kinematics_kernel", "tree": tree["name"], "envs": nenv,
            "kinematics_ms": kin_ms,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "bytes_per_env": kin_bytes},
            "tick_from_joint_states_ms": tick_ms,
            "tick_from_joint_states_solves_per_s": nenv / (tick_ms * 1e-3),
            "solve_same_qps_ms": solve_ms,
            "kinematics_added_ms": tick_ms - solve_ms,
            "tick_from_joint_states_warm_ms": warm_ms,
            "tick_from_joint_states_warm_solves_per_s": nenv / (warm_ms * 1e-3),
            "tick_from_joint_states_warm_mean_ipm_iters": float(out.iters.double().mean().item())}


def tumbling_pipeline(solver, nenv: int, steps: int, warmup: int, seed: int, stream) -> dict:
    """BASELINE configs[3] as ONE device pipeline per control tick (SURVEY.md §8(f) rows 1 + 3):
    joint states -> osc_batch_kinematics (M, C, J, b and the site positions) ->
    osc_tumbling_targets (walter_sr_true_tumbling_mjjoint.cc:622-1019: shin angle / thigh height /
    torso PD rows) -> osc_contact_mask_from_contacts (:473-558, a fresh synthetic contact list
    per tick through the example's geom -> site rule) -> osc_batch_solve.  No host round trip
    inside a tick.  The site positions stand in for the simulator's site_xpos the example reads.
    Timed with HIP events on the launch stream; reported beside the headline, not as it."""
    from osc_amd.kinematics import KinematicsBatch, load_tree, random_states
    from osc_amd.producers import contact_geom_table, contact_mask_into, tumbling_targets_into
    robot_tree = load_tree("walter_sr")
    kb = KinematicsBatch(tree=robot_tree)
    dev = solver.device
    q0, v0 = random_states(robot_tree, nenv, seed, joint_range=0.5)
    rng = np.random.default_rng(seed + 5)
    nticks = 8
    qs = [torch.from_numpy(q0 + 0.01 * (k + 1) * rng.standard_normal(q0.shape)).to(dev)
          for k in range(nticks)]
    for q in qs:
        q[:, 3:7] = q[:, 3:7] / q[:, 3:7].norm(dim=1, keepdim=True)
        q[:, 0:3] = 0.0
    vs = [torch.from_numpy(v0 * (1 + 0.01 * rng.standard_normal(v0.shape))).to(dev)
          for _ in range(nticks)]
    q0d, v0d = torch.from_numpy(q0).to(dev), torch.from_numpy(v0).to(dev)
    init = kb.compute(q0d, v0d, want_sites=True)               # the pre-loop snapshot (:363)
    t0 = torch.zeros(nenv, dtype=torch.float64, device=dev)
    ts = [torch.full((nenv,), 0.002 * (k + 1), dtype=torch.float64, device=dev)
          for k in range(nticks)]
    # contact lists: 20 geoms, geom g on body g, site s on body s: the example's id list marks
    # contact site k for geom ids[k] (osc_contact_geom_table)
    ids = (3, 4, 7, 8, 11, 12, 15, 16)
    table = torch.from_numpy(contact_geom_table(np.arange(20), np.arange(17), ids)).to(dev)
    max_con = 12
    ncons = [torch.from_numpy(rng.integers(0, max_con + 1, nenv).astype(np.int32)).to(dev)
             for _ in range(nticks)]
    pairs = [torch.from_numpy(np.stack([np.zeros((nenv, max_con), np.int32),
                                        rng.integers(0, 20, (nenv, max_con)).astype(np.int32)],
                                       axis=2)).to(dev) for _ in range(nticks)]
    kout = kb.alloc(nenv, want_sites=True)
    T = torch.empty((nenv, 17, 6), dtype=torch.float64, device=dev)
    mask = torch.empty((nenv, 8), dtype=torch.float64, device=dev)
    out = solver.alloc_outputs(nenv)
    k = [0]

    def tick():
        i = k[0] % nticks
        kb.compute_into(kout, qs[i], vs[i])
        tumbling_targets_into(T, qs[i], vs[i], kout.site_xpos, ts[i], t0, q0d, init.site_xpos)
        contact_mask_into(mask, ncons[i], pairs[i], table)
        solver.solve_into(out, kout.M, kout.C, kout.J, kout.b, T, mask)
        k[0] += 1

    for _ in range(warmup):
        tick()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        tick()
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    return {"stages": "osc_batch_kinematics -> osc_tumbling_targets -> "
                      "osc_contact_mask_from_contacts -> osc_batch_solve",
            "envs": nenv, "tick_ms": ms, "solves_per_s": nenv / (ms * 1e-3),
            "converged_frac": float((out.status == 0).double().mean().item()),
            "mean_ipm_iters": float(out.iters.double().mean().item()),
            "mean_contacts_active": float(mask.mean().item() * 8)}


def run_mixed(args, world, rank, dev, barrier, solver_cls=None, multi_fn=None,
              nenv=None) -> dict | None:
    """BASELINE configs[4]: mixed Go2 + WaLTER Sr.  Every rank solves its own shard of `nenv`
    Go2 envs AND `nenv` WaLTER envs (4,096 + 4,096 per GPU: 65,536 over 8 GPUs) in ONE
    osc_batch_solve_multi call: one assembly grid and one interior-point grid for both models,
    WaLTER's wavefronts first so Go2's fill the SIMDs its early finishers free (one
    kernel instantiation per model, no collective).  --mixed-mode streams / serial run the two
    models as two osc_batch_solve calls on two streams / one stream instead.  A step = both shards
    solved; value = all envs of all ranks / max-over-ranks time.  Returns the line on rank 0
    (the `mixed` object of the headline line, or the line of --robot mixed)."""
    if solver_cls is None:
        from osc_amd.solver import OSCBatchSolver as solver_cls
    if multi_fn is None:
        from osc_amd.solver import solve_multi_into as multi_fn
    nenv = args.nenv_per_gpu if nenv is None else nenv
    robots = ("unitree_go2", "walter_sr")
    clock = DeviceClock(dev)
    main = clock.stream()
    streams = [torch.cuda.Stream(dev) for _ in robots] if clock.cuda else [None, None]
    jobs = []
    for i, robot in enumerate(robots):
        solver = solver_cls(robot)
        d = generate(robot, nenv, shard_seed(rank) + 500 * i, args.scenario, args.mask)
        jobs.append((solver, solver.prepare(**d), solver.alloc_outputs(nenv)))
    multi_jobs = [(s, o, inp) for s, inp, o in jobs]

    def step():
        if args.mixed_mode == "multi":
            multi_fn(multi_jobs, stream=main)
        elif args.mixed_mode == "serial" or not clock.cuda:
            for solver, inputs, out in jobs:
                solver.solve_into(out, *inputs, stream=main)
        else:
            for st, (solver, inputs, out) in zip(streams, jobs):
                st.wait_stream(main)
                solver.solve_into(out, *inputs, stream=st)
            for st in streams:
                main.wait_stream(st)

    for _ in range(args.warmup):
        step()
    clock.sync()
    e0, e1 = clock.event(), clock.event()
    barrier()
    clock.sync()
    t0 = time.perf_counter()
    e0.record(main)
    for _ in range(args.steps):
        step()
    e1.record(main)
    clock.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / args.steps
    conv = sum(int((o.status == 0).sum().item()) for _, _, o in jobs)
    stats = reduce_stats(world, dev, 2 * nenv, elapsed, kernel_ms, 0.0, conv)
    if rank != 0:
        return None
    value = job_value(stats, args.steps)
    bps = (bytes_per_solve("unitree_go2") + bytes_per_solve("walter_sr")) * nenv
    achieved = bps / (stats.kernel_ms * 1e-3) / 1e9
    return {
        "metric": METRIC, "value": value, "unit": "solves/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": stats.elapsed_s / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded post-kinematics M, C, J, b, T, mask; osc_amd.synth)",
        "config": {"workload": f"mixed unitree_go2 + walter_sr {args.scenario} mask={args.mask}, "
                               f"{nenv} + {nenv} envs per GPU (BASELINE configs[4] at 8 GPUs)",
                   "robot": "mixed", "envs_per_gpu": 2 * nenv, "global_envs": stats.total_envs,
                   "parallelism": f"env-shard x{world}, 2 models per GPU ({args.mixed_mode})"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "kernel": ("osc_setup_pair_kernel + osc_ipm_pair_kernel"
                                if args.mixed_mode == "multi" else
                                f"osc_setup_kernel + osc_ipm_kernel x 2 models ({args.mixed_mode})"),
                     "kernel_ms": stats.kernel_ms},
        "converged_frac": stats.converged,
        **({"rehearsal": f"{os.environ['OSC_DIST_BACKEND']}: {world} ranks on "
                         f"{torch.cuda.device_count()} GPU(s), ranks sharing devices"}
           if world > 1 and os.environ.get("OSC_DIST_BACKEND", "nccl") != "nccl" else {})}


def run_north_star(args, world, rank, dev, barrier, solver_cls, clock) -> dict | None:
    """BASELINE.json north_star: Go2 at a GLOBAL batch of --north-star-envs (65,536) split over
    the N ranks (65,536 / N per GPU: strong scaling of that batch), the same timed-region rules as
    the headline (warmup, barrier, K cold solves, barrier, max over ranks).  Reported as the
    `north_star` object of the headline line; the target is >= 1M solves/s on 8 GPUs."""
    total = args.north_star_envs
    nenv = total // world + (1 if rank < total % world else 0)
    solver = solver_cls("unitree_go2")
    d = generate("unitree_go2", nenv, shard_seed(rank, 5), "standing", "ones")
    inputs = solver.prepare(**d)
    out = solver.alloc_outputs(nenv)
    stream = clock.stream()
    for _ in range(args.warmup):
        solver.solve_into(out, *inputs)
    clock.sync()
    e0, e1 = clock.event(), clock.event()
    barrier()
    clock.sync()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        solver.solve_into(out, *inputs)
    e1.record(stream)
    clock.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = e0.elapsed_time(e1) / args.steps
    conv = int((out.status == 0).sum().item())
    stats = reduce_stats(world, dev, nenv, elapsed, kernel_ms, 0.0, conv)
    if rank != 0:
        return None
    value = job_value(stats, args.steps)
    return {"workload": f"unitree_go2 standing, global batch {stats.total_envs} over {world} "
                        f"GPU(s) ({total // world} per GPU; BASELINE north_star at 8 GPUs)",
            "global_envs": stats.total_envs, "envs_per_gpu": total // world, "n_gpus": world,
            "value": value, "unit": "solves/s", "ms_per_step": stats.elapsed_s / args.steps * 1e3,
            "kernel_ms": stats.kernel_ms, "scaling": "strong (fixed global batch)",
            "target": 1e6, "meets_target": value >= 1e6, "converged_frac": stats.converged}


def warm_ticks(solver, inputs, nenv: int, steps: int, warmup: int, seed: int, stream) -> dict:
    """SURVEY.md §8d warm runs: a 10-step 1 % random walk of the inputs (M by an SPD-preserving
    congruence; made on the device before
    timing, replayed ping-pong so consecutive ticks always differ by one walk step), solved with
    the warm state carried from tick to tick (osc_batch_solve_warm; the reference's SetWarmStart,
    operational_space_controller.h:519-526).  Reported beside the cold headline, not as it."""
    g = torch.Generator(device=inputs[0].device).manual_seed(seed)
    nv = inputs[0].shape[1]
    eye = torch.eye(nv, dtype=torch.float64, device=inputs[0].device)
    seq = [inputs]
    for _ in range(9):
        new = []
        for i, t in enumerate(seq[-1]):
            if i == 5:                                   # contact mask: unchanged
                new.append(t)
                continue
            if i == 0:   # M: congruence A M A' keeps it SPD (osc_amd.synth.random_walk)
                A = eye + 0.01 / nv ** 0.5 * torch.randn(t.shape, generator=g, device=t.device,
                                                         dtype=t.dtype)
                w = A @ t @ A.transpose(1, 2)
                w = 0.5 * (w + w.transpose(1, 2))
            else:
                w = t * (1.0 + 0.01 * torch.randn(t.shape, generator=g, device=t.device,
                                                  dtype=t.dtype))
            new.append(w.contiguous())
        seq.append(tuple(new))
    order = list(range(10)) + list(range(8, 0, -1))
    warm = solver.alloc_warm_state(nenv)
    out = solver.alloc_outputs(nenv)
    k = 0
    for _ in range(warmup + len(order)):                 # settle, then one untimed cycle for iters
        solver.solve_warm_into(out, warm, *seq[order[k % len(order)]])
        k += 1
    torch.cuda.synchronize()
    iters = []
    for _ in range(len(order)):
        solver.solve_warm_into(out, warm, *seq[order[k % len(order)]])
        iters.append(out.iters.double().mean())
        k += 1
    mean_iters = float(torch.stack(iters).mean().item())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(stream)
    for _ in range(steps):
        solver.solve_warm_into(out, warm, *seq[order[k % len(order)]])
        k += 1
    e1.record(stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    conv = float((out.status == 0).double().mean().item())
    return {"value": nenv / (ms * 1e-3), "unit": "solves/s", "kernel_ms": ms,
            "mean_ipm_iters": mean_iters, "converged_frac": conv,
            "warm_state_bytes_per_env_rw": 2 * warm.numel() * 8 // max(nenv, 1),
            "workload": "same envs, 10-step 1 % random walk of M, C, J, b, T replayed "
                        "ping-pong, warm state carried between ticks"}


def host_fed(args, world, rank, dev, barrier, solver, feed_cls=None, kin_cls=None) -> dict | None:
    """SURVEY.md §8(e)'s data path: every tick's inputs start in PINNED HOST
    memory -- where the reference's control loop finds them (operational_space_controller.h:
    546-573) -- cross PCIe in one H2D copy, are solved, and tau / status / iters come back
    (include/osc_host_feed.h).  Depth 2: tick k's copy overlaps tick k-1's solve.  Two input forms:
    post-kinematics QP inputs (M, C, J, b, T, mask: 7,664 B per Go2 env) and joint states (qpos,
    qvel, T, mask through the GPU kinematics: 568 B).  Each rank runs its own feed (its own pinned
    buffers, its own host thread = the rank process); value = all ranks' envs x ticks / the slowest
    rank's time.  The producer's writes are not timed (the inputs of two ticks are written once
    into the two pinned slots, alternating); each tick still waits for its slot as a producer
    would.  Stage durations by HIP events on each stage's stream (the last ticks).  Reported
    beside the headline (whose inputs are HBM-resident), never as it."""
    if feed_cls is None:
        from osc_amd.host_feed import HostFeed as feed_cls
    if kin_cls is None:
        from osc_amd.kinematics import KinematicsBatch as kin_cls
    from osc_amd.kinematics import load_tree, random_states
    robot = solver.robot
    sizes = [int(s) for s in args.host_fed_envs.split(",") if s.strip()]
    res = {"robot": robot, "depth": args.host_fed_depth, "per_gpu": {}}
    tree = load_tree(robot)
    kin = kin_cls(tree=tree)
    steps, warmup = max(args.steps, 10), max(args.warmup, 4)
    for nenv in sizes:
        d = [generate(robot, nenv, shard_seed(rank) + 40 + k, args.scenario, args.mask)
             for k in range(2)]
        qs = [random_states(tree, nenv, shard_seed(rank) + 50 + k, joint_range=0.5)
              for k in range(2)]
        # the warm-started loop (the reference warm-starts every tick, osc.h:519-526): two joint
        # states one control step apart (joint angles +-0.01 rad, velocities +-1 %), alternating
        rng = np.random.default_rng(shard_seed(rank) + 60)
        q1, v1 = qs[0][0].copy(), qs[0][1] * (1.0 + 0.01 * rng.standard_normal(qs[0][1].shape))
        q1[:, 7:] += 0.01 * rng.standard_normal(q1[:, 7:].shape)
        qw = [qs[0], (q1, v1)]
        for key, form, warm in (("qp", "qp", False), ("joint_states", "joint_states", False),
                                ("joint_states_warm", "joint_states", True)):
            row = {}
            for depth in (args.host_fed_depth, 1):
                feed = feed_cls(solver, nenv, form, depth=depth, warm=warm,
                                kin=kin if form == "joint_states" else None)
                tick = [0]

                def step(fill=False):
                    k = tick[0]
                    v = feed.inputs(k)
                    if fill:
                        src = d[k % 2]
                        if form == "qp":
                            for a in ("M", "C", "J", "b"):
                                v[a][...] = src[a]
                        else:
                            v["qpos"][...], v["qvel"][...] = (qw if warm else qs)[k % 2]
                        tm = d[0] if warm else src
                        v["T"][...], v["mask"][...] = tm["T"], tm["mask"]
                    feed.submit(k)
                    if k >= depth - 1:
                        feed.wait(k - depth + 1)
                    tick[0] += 1

                for w in range(warmup):
                    step(fill=w < 2)
                barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    step()
                for j in range(tick[0] - depth + 1, tick[0]):   # drain the pipeline
                    feed.wait(j)
                elapsed = time.perf_counter() - t0
                barrier()
                last = tick[0] - 1
                tau, status, iters = feed.wait(last)
                conv = int((np.asarray(status) == 0).sum())
                tims = [feed.timing(j) for j in range(max(0, last - depth + 1), last + 1)]
                stats = reduce_stats(world, dev, nenv, elapsed, 0.0, 0.0, conv)
                h2d = float(np.mean([t["h2d_ms"] for t in tims]))
                sol = float(np.mean([t["solve_ms"] for t in tims]))
                d2h = float(np.mean([t["d2h_ms"] for t in tims]))
                kin_ms = float(np.mean([t.get("kin_ms", 0.0) for t in tims]))
                period = stats.elapsed_s / steps * 1e3
                serial = h2d + sol + d2h
                longest = max(h2d, sol, d2h)
                entry = {"value": job_value(stats, steps), "unit": "solves/s",
                         "ms_per_tick": period, "h2d_ms": h2d, "solve_ms": sol, "d2h_ms": d2h,
                         **({"kin_ms": kin_ms} if form == "joint_states" else {}),
                         "h2d_bytes": int(feed.in_bytes), "d2h_bytes": int(feed.out_bytes),
                         "h2d_GBps": feed.in_bytes / (h2d * 1e-3) / 1e9 if h2d > 0 else None,
                         "bytes_per_env_h2d": feed.in_bytes / nenv,
                         "converged_frac": stats.converged,
                         "mean_ipm_iters": float(np.asarray(iters).mean()),
                         "global_envs": stats.total_envs}
                if depth > 1:
                    entry["overlap_frac"] = ((serial - period) / (serial - longest)
                                             if serial > longest else None)
                    entry["bound"] = "h2d (PCIe)" if h2d >= sol else "solve"
                    row.update(entry)
                else:
                    row["serial_depth1"] = {k: entry[k] for k in ("value", "ms_per_tick")}
                feed.close()
            res["per_gpu"].setdefault(str(nenv), {})[key] = row
    res["note"] = ("overlap_frac = (h2d + solve + d2h - period) / (h2d + solve + d2h - longest "
                   "stage): 1 = every stage but the longest hidden; serial_depth1 = the same "
                   "ticks with one slot (copies and solve in series)")
    return res if rank == 0 else None


def staggered(args, solver, inputs, groups: int) -> dict:
    """The headline's batch as `groups` env groups, each group's ticks in order on its own stream
    (tick k+1 of a group after its tick k; groups independent) -- how a deployment whose env groups
    tick out of phase uses the GPU: one group's assembly fills the SIMDs another group's
    interior-point straggler tail leaves idle (tools/stagger_probe.py).  A step = every env solved
    once; reported beside the headline, not as it (the headline's step is ONE call over the whole
    batch: forking and joining streams inside a step measured slower, profiles/r06/
    stagger_probe.jsonl)."""
    nenv = inputs[0].shape[0]
    per = nenv // groups
    gs = []
    for g in range(groups):
        sl = slice(g * per, nenv if g == groups - 1 else (g + 1) * per)
        inp = tuple(t[sl].contiguous() for t in inputs)
        gs.append((torch.cuda.Stream(), inp, solver.alloc_outputs(inp[0].shape[0])))

    def step():
        for st, inp, out in gs:
            solver.solve_into(out, *inp, stream=st)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    conv = sum(int((out.status == 0).sum().item()) for _, _, out in gs)
    return {"groups": groups, "envs": nenv, "value": nenv * args.steps / el, "unit": "solves/s",
            "ms_per_step": el / args.steps * 1e3, "converged_frac": conv / nenv,
            "workload": f"the headline's {nenv} envs as {groups} groups of {per}, each group's "
                        f"ticks in order on its own stream, groups out of phase"}


def baseline_config_tag(args, nenv):
    """Which BASELINE.json config this workload is (configs[1]..[3] are single-GPU ones)."""
    tags = {("unitree_go2", "standing", "ones", 4096): 1,
            ("walter_sr", "standing", "ones", 4096): 2,
            ("walter_sr", "tumbling", "bernoulli", 8192): 3}
    c = tags.get((args.robot, args.scenario, args.mask, nenv))
    return f" (BASELINE configs[{c}])" if c is not None else ""


class DeviceClock:
    """HIP events on the launch stream on a GPU; host timestamps on the CPU (the gloo test of the
    multi-rank path, tests/test_dist.py, runs the same per-rank code without a device)."""

    class _HostEvent:
        def record(self, stream=None):
            self.t = time.perf_counter()

        def elapsed_time(self, other):
            return (other.t - self.t) * 1e3

    def __init__(self, dev: torch.device):
        self.cuda = dev.type == "cuda"
        self.dev = dev

    def event(self):
        return torch.cuda.Event(enable_timing=True) if self.cuda else self._HostEvent()

    def sync(self):
        if self.cuda:
            torch.cuda.synchronize()

    def stream(self):
        return torch.cuda.current_stream(self.dev) if self.cuda else None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--robot", default="unitree_go2")
    ap.add_argument("--nenv-per-gpu", type=int, default=4096)
    ap.add_argument("--scenario", default="standing", choices=["standing", "tumbling"])
    ap.add_argument("--mask", default="ones", choices=["ones", "bernoulli"])
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--cpu-cores", type=int, default=min(16, os.cpu_count() or 1),
                    help="CPU baseline worker processes (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-warm", action="store_true",
                    help="skip the warm-start (random-walk) timing reported beside the headline")
    ap.add_argument("--no-front-end", action="store_true",
                    help="skip the kinematics front-end timing (reported beside the headline)")
    ap.add_argument("--no-single-env", action="store_true",
                    help="skip the configs[0] single-env tick latency reported beside the headline")
    ap.add_argument("--single-env-ticks", type=int, default=2000)
    ap.add_argument("--no-pipeline", action="store_true",
                    help="walter_sr tumbling: skip the whole-tick device pipeline timing")
    ap.add_argument("--event-every", type=int, default=5,
                    help="HIP events around the two kernels on every N-th step of a sampled run "
                         "after the timed steps (kernel durations for the roofline objects); the "
                         "timed steps run bare")
    ap.add_argument("--mask-redraw", type=int, default=0,
                    help="cycle through this many Bernoulli masks, one per step (configs[3]: "
                         "contact-mode switching, walter_sr_true_tumbling_mjjoint.cc:554-614)")
    ap.add_argument("--mixed-mode", default="multi", choices=["multi", "streams", "serial"],
                    help="--robot mixed: one osc_batch_solve_multi call, or two solves on two "
                         "streams / on one stream")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "pmc_traffic.json"))
    ap.add_argument("--north-star-envs", type=int, default=65536,
                    help="global Go2 batch of the north_star object (split over the ranks)")
    ap.add_argument("--no-north-star", action="store_true")
    ap.add_argument("--mixed-envs", type=int, default=4096,
                    help="per-model envs per GPU of the mixed (configs[4]) object")
    ap.add_argument("--no-mixed", action="store_true")
    ap.add_argument("--hbm-batches", type=int, default=10,
                    help="roofline.hbm_inputs: rotate this many copies of the batch (> 256 MB of "
                         "inputs: past the Infinity Cache); 0 = off")
    ap.add_argument("--host-fed-envs", default="4096,8192",
                    help="per-GPU batches of the host_fed object (SURVEY.md §8(e): inputs from "
                         "pinned host memory every tick); empty = off")
    ap.add_argument("--host-fed-after", action="store_true",
                    help="run the host_fed object after the headline instead of before the "
                         "north_star / mixed lines (default: before -- like them it completes, "
                         "synced, before the headline's timed steps, which then start at the "
                         "clocks of a running loop: Go2 4,096 in the driver's 20 + 5 window 24.1-24.5 "
                         "vs 23.5-23.8 M solves/s after, profiles/r06/bench_order_ab.jsonl)")
    ap.add_argument("--host-fed-depth", type=int, default=2,
                    help="pipeline slots of the host-fed tick (2 = H2D of tick k overlaps the "
                         "solve of tick k-1)")
    ap.add_argument("--stagger-groups", type=int, default=0,
                    help="the `staggered` object beside the headline: its batch as this many env "
                         "groups ticking out of phase on their own streams; <= 1 = off (default: "
                         "off -- in a process that already holds more streams than the GPU's 4 "
                         "hardware queues the groups share queues and serialise; measured on its "
                         "own by tools/stagger_probe.py)")
    ap.add_argument("--hbm-only", action="store_true",
                    help="run only the HBM-input rotation (for rocprofv3 --pmc passes)")
    ap.add_argument("--hbm-traffic-json",
                    default=os.path.join(REPO, "profiles", "pmc_traffic_hbm.json"))
    return ap.parse_args(argv)


def launch_ranks(args, argv) -> int | None:
    """One process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process IS a rank
    and WORLD_SIZE must equal --gpus.  Otherwise --gpus N > 1 starts the N ranks itself: a
    torch.distributed.run child on 127.0.0.1 running this script with the same arguments, started
    before this process has touched the GPU; its exit code is returned."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def prepare_headline(args, rank: int, solver_cls):
    """The headline's model, device inputs and outputs (host-side generation: done before the
    GPU lines that precede the timed region, so no idle gap lets the clocks drop before it)."""
    solver = solver_cls(args.robot)
    d = generate(args.robot, args.nenv_per_gpu, shard_seed(rank), args.scenario, args.mask)
    inputs = solver.prepare(**d)
    return solver, inputs, solver.alloc_outputs(args.nenv_per_gpu)


def run_headline(args, world: int, rank: int, dev: torch.device, barrier, solver_cls,
                 clock: DeviceClock, prepared=None):
    """The timed region of one rank (BASELINE metric): warmup, barrier, K steps of assemble +
    interior point over this rank's shard, barrier, then the max-over-ranks reduction.  Returns
    (line, solver, inputs) on rank 0 and (None, solver, inputs) elsewhere."""
    nenv = args.nenv_per_gpu
    solver, inputs, out = prepared or prepare_headline(args, rank, solver_cls)
    stream = clock.stream()
    # per-step contact masks (mask switching): step k assembles and solves with masks[k % K]
    masks = [inputs[5]]
    if args.mask_redraw > 0:
        rng = np.random.default_rng(shard_seed(rank) + 1)
        nc = inputs[5].shape[1]
        masks = [torch.from_numpy((rng.uniform(size=(nenv, nc)) < 0.75).astype(np.float64))
                 .to(dev) for _ in range(args.mask_redraw)]

    for _ in range(args.warmup):
        solver.solve_into(out, *inputs)
    clock.sync()

    # Each step = osc_batch_assemble (setup kernel) + osc_batch_solve_assembled (interior-point
    # kernel), the two halves of osc_batch_solve.  The K timed steps run bare (no events: each
    # costs the stream ~3 us, tools/event_overhead.py); the per-kernel durations of the roofline
    # objects come from HIP events on the launch stream around each kernel over a separate sampled
    # run of the same steps right after the timed region (round 6: before, events on every 5-th
    # timed step made the split an upper bound of the step).
    barrier()
    clock.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        mask = masks[k % len(masks)]
        solver.assemble_into(out, *inputs[:5], mask)
        solver.solve_assembled_into(out, mask)
    clock.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    every = max(1, args.event_every)
    nsample = max(4, args.steps // every)
    ev = [[clock.event() for _ in range(3)] for _ in range(nsample)]
    for k in range(nsample):
        mask = masks[k % len(masks)]
        ev[k][0].record(stream)
        solver.assemble_into(out, *inputs[:5], mask)
        ev[k][1].record(stream)
        solver.solve_assembled_into(out, mask)
        ev[k][2].record(stream)
        if k + 1 < nsample:   # (bare steps between the sampled ones: the loop's steady state)
            for j in range(every - 1):
                mj = masks[(k + 1 + j) % len(masks)]
                solver.assemble_into(out, *inputs[:5], mj)
                solver.solve_assembled_into(out, mj)
    clock.sync()
    setup_ms = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev)
    ipm_ms = sum(e[1].elapsed_time(e[2]) for e in ev) / len(ev)

    st = out.status.cpu().numpy()
    mean_iters = float(out.iters.double().mean().item())
    stats = reduce_stats(world, dev, nenv, elapsed, setup_ms, ipm_ms, int((st == 0).sum()))
    elapsed, kernel_ms, setup_ms, ipm_ms = stats.elapsed_s, stats.kernel_ms, stats.setup_ms, stats.ipm_ms
    if rank != 0:
        return None, solver, inputs
    total = stats.total_envs
    value = job_value(stats, args.steps)
    bps = bytes_per_solve(args.robot)
    # dominant kernel = osc_ipm_kernel (~80 % of the solve): path bytes per launch over its
    # own event-timed duration; the setup + IPM pair is reported beside it
    achieved = bps * nenv / (ipm_ms * 1e-3) / 1e9
    achieved_pair = bps * nenv / (kernel_ms * 1e-3) / 1e9
    traffic = traffic_pair = None
    tpath = args.traffic_json
    if not os.path.exists(tpath) or json.load(open(tpath)).get("nenv") != nenv:
        # PMC passes at other batch sizes sit beside it (tools/pmc_summary.py)
        alt = os.path.join(os.path.dirname(tpath), f"pmc_traffic_{nenv}.json")
        tpath = alt if os.path.exists(alt) else tpath
    if os.path.exists(tpath):
        with open(tpath) as fh:
            tj = json.load(fh)
        if tj.get("robot") == args.robot and tj.get("nenv") == nenv:
            traffic_pair = tj.get("bytes_per_launch")
            traffic = tj.get("per_kernel", {}).get("osc_ipm_kernel")
    flops = algorithmic_flops(args.robot, mean_iters)
    tflops = flops * nenv / (kernel_ms * 1e-3) / 1e12
    ipm_name = ipm_kernel_name(args.robot, nenv, dev)
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
        "config": {"workload": f"{args.robot} {args.scenario} mask={args.mask}"
                               f"{f' redrawn per step ({args.mask_redraw} masks)' if args.mask_redraw else ''}, "
                               f"{nenv} envs per GPU{baseline_config_tag(args, nenv)}",
                   "robot": args.robot, "envs_per_gpu": nenv, "global_envs": total,
                   "parallelism": f"env-shard x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ipm_name, "kernel_ms": ipm_ms,
                     "kernel_ms_from": f"HIP events around the kernel on every "
                                       f"{max(1, args.event_every)}-th step of a sampled run right "
                                       f"after the (event-free) timed steps (the full-space "
                                       f"refinement runs inside it)",
                     "bytes_per_solve": bps,
                     "inputs": "cache-warm: the same batch every step (its 31 MB stays in the "
                               "256 MB Infinity Cache); the kernel is latency-bound; "
                               "hbm_inputs: the same QPs rotated through > 256 MB of buffers",
                     "solve_pair": {"kernel": f"osc_setup_kernel + {ipm_name}",
                                    "kernel_ms": kernel_ms, "achieved": achieved_pair,
                                    "frac": achieved_pair / HBM_PEAK_GBS,
                                    "traffic": traffic_pair,
                                    "kernel_ms_split": {"osc_setup_kernel": setup_ms,
                                                        ipm_name: ipm_ms}}},
        "roofline_fp64": {"kernel": f"osc_setup_kernel + {ipm_name}", "achieved": tflops,
                          "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": tflops / FP64_PEAK_TFLOPS,
                          "flops_per_solve": flops, "mean_ipm_iters": mean_iters},
        "converged_frac": stats.converged,
    }
    return line, solver, inputs


def hbm_inputs(args, solver, inputs, clock, traffic_json: str) -> dict:
    """roofline.hbm_inputs: the headline's step over inputs that come from HBM.
    The headline solves the same 31 MB batch every step, which stays in the 256 MB Infinity Cache
    (MALL).  Here `--hbm-batches` copies of that batch -- the same QPs, each copy's envs rotated
    by a different offset, in their own buffers (10 x 31.4 MB = 314 MB > 256 MB) -- are solved in
    turn, so every step's setup kernel reads inputs the previous steps have evicted.  Same QPs, so
    the iteration counts (and the interior point's work) equal the headline's: the difference is
    where the inputs come from.  Kernel times by HIP events as in the headline."""
    nb = args.hbm_batches
    nenv = inputs[0].shape[0]
    batches = [tuple(t.roll(shifts=(i * 1031) % nenv, dims=0).contiguous() for t in inputs)
               for i in range(nb)]
    out = solver.alloc_outputs(nenv)
    stream = clock.stream()
    steps = max(args.steps, 3 * nb)
    for k in range(max(args.warmup, nb)):
        solver.solve_into(out, *batches[k % nb])
    every = max(1, args.event_every)
    sampled = [k for k in range(steps) if k % every == every - 1] or [steps - 1]
    ev = {k: [clock.event() for _ in range(3)] for k in sampled}
    clock.sync()
    t0 = time.perf_counter()
    for k in range(steps):
        inp = batches[k % nb]
        e = ev.get(k)
        if e:
            e[0].record(stream)
        solver.assemble_into(out, *inp[:5], inp[5])
        if e:
            e[1].record(stream)
        solver.solve_assembled_into(out, inp[5])
        if e:
            e[2].record(stream)
    clock.sync()
    elapsed = time.perf_counter() - t0
    setup_ms = sum(e[0].elapsed_time(e[1]) for e in ev.values()) / len(ev)
    ipm_ms = sum(e[1].elapsed_time(e[2]) for e in ev.values()) / len(ev)
    bps = bytes_per_solve(args.robot)
    res = {"inputs": "hbm", "batches": nb,
           "input_bytes_resident": int(sum(t.numel() * t.element_size() for b in batches for t in b)),
           "steps": steps, "value": nenv * steps / elapsed, "unit": "solves/s",
           "ms_per_step": elapsed / steps * 1e3,
           "kernel": "osc_ipm_kernel", "kernel_ms": ipm_ms,
           "achieved": bps * nenv / (ipm_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit_bw": "GB/s",
           "frac": bps * nenv / (ipm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
           "solve_pair": {"kernel_ms": setup_ms + ipm_ms,
                          "kernel_ms_split": {"osc_setup_kernel": setup_ms, "osc_ipm_kernel": ipm_ms},
                          "achieved": bps * nenv / ((setup_ms + ipm_ms) * 1e-3) / 1e9,
                          "frac": bps * nenv / ((setup_ms + ipm_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS},
           "traffic": None, "solve_pair_traffic": None}
    if os.path.exists(traffic_json):
        tj = json.load(open(traffic_json))
        if tj.get("robot") == args.robot and tj.get("nenv") == nenv and tj.get("inputs") == "hbm":
            res["traffic"] = tj.get("per_kernel", {}).get("osc_ipm_kernel")
            res["solve_pair_traffic"] = tj.get("bytes_per_launch")
            res["traffic_source"] = tj.get("source")
    return res


def multi_gpu_objects(args, world, rank, dev, barrier, solver_cls, clock,
                      multi_fn=None) -> dict:
    """The BASELINE targets beside the headline (every rank takes part; rank 0 attaches them):
    `north_star` = Go2 at global batch 65,536 split over the ranks, `mixed` = configs[4]'s
    per-GPU shard (4,096 Go2 + 4,096 WaLTER per rank) through osc_batch_solve_multi.  They run
    BEFORE the headline's timed region: the headline's K steps then start at the clocks a running
    control loop sees, not from an idle GPU's ramp (at the driver's 5 warmup steps the ramp alone
    cost ~5 % of a Go2 4,096 step)."""
    out = {}
    if not args.no_north_star:
        out["north_star"] = run_north_star(args, world, rank, dev, barrier, solver_cls, clock)
    if not args.no_mixed:
        mx = run_mixed(args, world, rank, dev, barrier, solver_cls, multi_fn, args.mixed_envs)
        if mx is not None:
            out["mixed"] = {k: mx[k] for k in ("value", "unit", "ms_per_step", "converged_frac",
                                               "config", "roofline")}
    return out


def attach_multi_gpu_objects(args, world, rank, dev, barrier, solver_cls, clock, line,
                             multi_fn=None) -> None:
    """multi_gpu_objects, attached to `line` (rank 0)."""
    objs = multi_gpu_objects(args, world, rank, dev, barrier, solver_cls, clock, multi_fn)
    if line is not None:
        line.update(objs)


def single_env(robot: str, ticks: int) -> dict:
    """BASELINE configs[0]: one environment, one tick at a time through the controller
    (osc_amd/bin/osc_tick_latency: OperationalSpaceController::step() = State packing, H2D, GPU
    kinematics + QP, D2H), against the reference's 2,000 us control period (osc.h:108).
    Reported beside the CPU port's single-core rate; never part of `value`."""
    import subprocess
    exe = os.path.join(REPO, "operational-space-control_amd", "bin", "osc_tick_latency")
    xml = os.path.join(REPO, "operational-space-control_amd", "config",
                       f"{'unitree_go2' if robot == 'unitree_go2' else 'walter_sr'}.xml")
    if not os.path.exists(exe):
        return {"error": f"{exe} not built (__graft_entry__.build())"}
    r = subprocess.run([exe, robot, xml, str(ticks)], capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": f"osc_tick_latency exit {r.returncode}: {r.stderr.strip()[-300:]}"}
    res = json.loads(r.stdout.strip().splitlines()[-1])
    res["path"] = ("OperationalSpaceController::step(): State -> qpos/qvel, H2D, GPU kinematics "
                   "(MJCF tree) + reduced QP + interior point (warm), D2H; wall time per tick")
    res["reference_period_us"] = 2000
    return res


def ipm_kernel_name(robot: str, nenv: int, dev) -> str:
    """The interior-point kernel(s) one launch runs: past one resident wavefront per SIMD the
    cold WaLTER solve of at least four rounds of wavefronts runs the lockstep compaction's park and resume passes (csrc/osc_ipm.hpp,
    ParkArgs; the default park iteration, osc_model_tuning.park_it, is 16 for WaLTER, off for Go2)."""
    cus = (torch.cuda.get_device_properties(dev).multi_processor_count
           if torch.cuda.is_available() else 256)   # (CPU rehearsal of the rank path: MI355X)
    resident = 4 * 4 * cus
    if nenv >= 4 * resident and robot == "walter_sr":   # (kParkMinRounds)
        return "osc_ipm_compact_kernel (park + resume passes)"
    return "osc_ipm_kernel"


def main(argv=None) -> None:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    rc = launch_ranks(args, argv)
    if rc is not None:
        sys.exit(rc)

    ri = rank_info()
    world, rank, local = ri.world, ri.rank, ri.local
    # OSC_DIST_BACKEND=gloo: rehearsal of the N-rank path on a box with fewer GPUs than ranks
    # (ranks share the devices round-robin; barriers and the reduction over gloo on the host)
    backend = os.environ.get("OSC_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)   # RCCL; barriers + timing reduction only
        else:
            dist.init_process_group(backend)

    def barrier():
        dist_barrier(world)

    if args.robot == "mixed":
        line = run_mixed(args, world, rank, dev, barrier)
        if line is not None:
            print(json.dumps(line), flush=True)
        if world > 1:
            torch.distributed.destroy_process_group()
        return

    from osc_amd.solver import OSCBatchSolver
    clock = DeviceClock(dev)
    if args.hbm_only:   # (profiling aid: the rotation alone, nothing else on the GPU)
        solver = OSCBatchSolver(args.robot)
        d = generate(args.robot, args.nenv_per_gpu, shard_seed(rank), args.scenario, args.mask)
        print(json.dumps(hbm_inputs(args, solver, solver.prepare(**d), clock,
                                    args.hbm_traffic_json)), flush=True)
        return
    prepared = prepare_headline(args, rank, OSCBatchSolver)
    # SURVEY.md §8(e)'s host-fed tick: every rank its own pinned feed.  It completes (synced,
    # barriers) before or after the headline's timed region -- never overlapping it
    want_hf = bool(args.host_fed_envs.strip()) and args.robot != "mixed"
    hf = (host_fed(args, world, rank, dev, barrier, prepared[0])
          if want_hf and not args.host_fed_after else None)
    objs = multi_gpu_objects(args, world, rank, dev, barrier, OSCBatchSolver, clock)
    line, solver, inputs = run_headline(args, world, rank, dev, barrier, OSCBatchSolver, clock,
                                        prepared)
    if want_hf and args.host_fed_after:
        hf = host_fed(args, world, rank, dev, barrier, solver)
    if line is not None:
        line.update(objs)
        if hf is not None:
            line["host_fed"] = hf
        line["clocks"] = ("the headline's timed steps run after the host_fed / north_star / mixed "
                          "lines (GPU clocks at a running loop's level, not an idle GPU's ramp)")
    if line is not None:
        nenv = args.nenv_per_gpu
        stream = clock.stream()
        if world == 1 and args.hbm_batches > 0:
            line["roofline"]["hbm_inputs"] = hbm_inputs(args, solver, inputs, clock,
                                                         args.hbm_traffic_json)
        if world == 1 and args.stagger_groups > 1:
            line["staggered"] = staggered(args, solver, inputs, args.stagger_groups)
        if world == 1 and not args.no_warm:
            line["warm"] = warm_ticks(solver, inputs, nenv, args.steps, args.warmup,
                                      shard_seed(rank) + 7, stream)
        if world == 1 and not args.no_front_end:   # rank-local extra; N=1 only, like cpu_baseline
            line["front_end"] = front_end(args.robot, solver, nenv, args.steps, args.warmup,
                                          shard_seed(rank), stream)
        if world == 1 and args.robot == "walter_sr" and args.scenario == "tumbling" and \
                not args.no_pipeline:
            line["pipeline"] = tumbling_pipeline(solver, nenv, args.steps, args.warmup,
                                                 shard_seed(rank) + 13, stream)
        if world == 1 and not args.no_single_env:
            line["single_env"] = single_env(args.robot, args.single_env_ticks)
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(args.robot, args.cpu_seconds, args.cpu_cores)
        if backend != "nccl" and world > 1:   # not a multi-GPU measurement
            line["rehearsal"] = (f"{backend}: {world} ranks on {torch.cuda.device_count()} "
                                 f"GPU(s), ranks sharing devices")
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
