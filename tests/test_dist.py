"""Multi-GPU path of bench.py (osc_amd/dist.py) on CPU: world_size 2 over gloo on 127.0.0.1.
Each rank draws its own shard (weak scaling, no collective on the data path); the job's time is
the max over ranks and its convergence the sum -- the same functions bench.py calls over RCCL."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from osc_amd.dist import barrier, job_value, reduce_stats, shard_seed
from osc_amd.synth import generate


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        nenv = 8 + 4 * rank                                   # ranks may hold different shards
        d = generate("unitree_go2", nenv, shard_seed(rank), "standing", "ones")
        barrier(world)
        stats = reduce_stats(world, torch.device("cpu"), nenv, elapsed_s=1.0 + rank,
                             setup_ms=0.1 * (rank + 1), ipm_ms=0.5 + rank,
                             n_converged=nenv - rank)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), M0=d["M"][0], elapsed=stats.elapsed_s,
                 kernel=stats.kernel_ms, setup=stats.setup_ms, ipm=stats.ipm_ms,
                 conv=stats.converged, total=stats.total_envs, value=job_value(stats, 10))
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_bookkeeping(tmp_path):
    world, port = 2, _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    r = [np.load(tmp_path / f"r{k}.npz") for k in range(world)]
    assert not np.array_equal(r[0]["M0"], r[1]["M0"])     # independent shards
    for k in range(world):                                 # every rank sees the job totals
        assert float(r[k]["elapsed"]) == 2.0                # max over ranks
        assert float(r[k]["setup"]) == 0.2 and float(r[k]["ipm"]) == 1.5
        assert abs(float(r[k]["kernel"]) - (0.2 + 1.5)) < 1e-12   # max of the per-rank sums (1.7)
        assert int(r[k]["total"]) == 8 + 12
        assert abs(float(r[k]["conv"]) - (8 + 11) / 20) < 1e-12
        assert abs(float(r[k]["value"]) - 20 * 10 / 2.0) < 1e-9


# ---- bench.py's own per-rank path on two gloo ranks (the solve stubbed: no device here) ----

class _StubSolver:
    """Host stand-in for OSCBatchSolver with the calls bench.run_headline makes; every env
    "converges" in 10 iterations.  Only the device work is stubbed: shards, timing, barriers and
    the reduction are bench.py's own."""

    def __init__(self, robot):
        from osc_amd.robots import dims
        self.robot = robot
        self.nu = dims(robot)["nu"]

    def prepare(self, M, C, J, b, T, mask):
        return tuple(torch.from_numpy(x) for x in (M, C, J, b, T, mask))

    def alloc_outputs(self, nenv):
        import types
        return types.SimpleNamespace(tau=torch.zeros(nenv, self.nu, dtype=torch.float64),
                                     status=torch.zeros(nenv, dtype=torch.int32),
                                     iters=torch.full((nenv,), 10, dtype=torch.int32))

    def solve_into(self, out, *inputs, stream=None):
        out.tau.zero_()

    def assemble_into(self, out, M, C, J, b, T, mask):
        out.tau.copy_(M[:, :self.nu, 0])

    def solve_assembled_into(self, out, mask):
        out.status.zero_()


class _StubFeed:
    """Host stand-in for osc_amd.host_feed.HostFeed (pinned slots -> H2D -> solve -> D2H): the
    slot / tick bookkeeping of include/osc_host_feed.h on numpy buffers, no device."""

    def __init__(self, solver, nenv, form="qp", depth=2, warm=False, kin=None):
        from osc_amd.robots import dims
        d = dims(solver.robot)
        self.nenv, self.form, self.depth, self.next = nenv, form, depth, 0
        shapes = {"T": (nenv, d["ns"], 6), "mask": (nenv, d["nc"])}
        if form == "qp":
            shapes.update(M=(nenv, d["nv"], d["nv"]), C=(nenv, d["nv"]),
                          J=(nenv, d["s"], d["nv"]), b=(nenv, d["s"]))
        else:
            assert kin is not None
            shapes.update(qpos=(nenv, d["nv"] + 1), qvel=(nenv, d["nv"]))
        self.slots = [{k: np.zeros(v) for k, v in shapes.items()} for _ in range(depth)]
        self.in_bytes = sum(a.nbytes for a in self.slots[0].values())
        self.out_bytes = nenv * (d["nu"] * 8 + 8)
        self.done, self.nu = {}, d["nu"]

    def inputs(self, k):
        assert k == self.next
        return self.slots[k % self.depth]

    def submit(self, k):
        assert k == self.next
        src = self.slots[k % self.depth]
        first = src["M"][:, 0, :self.nu] if self.form == "qp" else src["qpos"][:, :self.nu]
        self.done[k] = (first.copy(), np.zeros(self.nenv, np.int32), np.full(self.nenv, 10, np.int32))
        self.next += 1

    def wait(self, k):
        assert self.next - self.depth <= k < self.next
        return self.done[k]

    def timing(self, k):
        return {"h2d_ms": 0.3, "solve_ms": 0.2, "d2h_ms": 0.01, "latency_ms": 0.6}

    def close(self):
        pass


class _StubKin:
    def __init__(self, tree=None):
        self.tree = tree


def _stub_multi(jobs, stream=None):
    for solver, out, inputs in jobs:
        solver.solve_into(out, *inputs)


def _bench_worker(rank, world, port, out_dir):
    import json
    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        args = bench.parse_args(["--gpus", str(world), "--steps", "3", "--warmup", "1",
                                 "--nenv-per-gpu", "24", "--traffic-json", "/nonexistent",
                                 "--north-star-envs", "50", "--mixed-envs", "8"])
        dev = torch.device("cpu")
        clock = bench.DeviceClock(dev)
        line, _, inputs = bench.run_headline(args, world, rank, dev, lambda: barrier(world),
                                             _StubSolver, clock)
        bench.attach_multi_gpu_objects(args, world, rank, dev, lambda: barrier(world), _StubSolver,
                                       clock, line, multi_fn=_stub_multi)
        np.save(os.path.join(out_dir, f"M{rank}.npy"), inputs[0].numpy())
        # every rank its own host feed (pinned slots, its own host thread)
        args.host_fed_envs = "16,32"
        hf = bench.host_fed(args, world, rank, dev, lambda: barrier(world), _StubSolver("unitree_go2"),
                            feed_cls=_StubFeed, kin_cls=_StubKin)
        if line is not None:
            line["host_fed"] = hf
        else:
            assert hf is None
        if rank == 0:
            with open(os.path.join(out_dir, "line.json"), "w") as fh:
                json.dump(line, fh)
        else:
            assert line is None
    finally:
        dist.destroy_process_group()


def test_bench_rank_path_two_gloo_ranks(tmp_path):
    import json
    world, port = 2, _free_port()
    mp.spawn(_bench_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    line = json.load(open(tmp_path / "line.json"))
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    assert line["config"]["envs_per_gpu"] == 24
    assert line["config"]["global_envs"] == 2 * 24
    assert line["config"]["parallelism"] == "env-shard x2"
    assert abs(line["value"] - 2 * 24 * 3 / (line["ms_per_step"] * 3 / 1e3)) <= 1e-6 * line["value"]
    assert line["converged_frac"] == 1.0
    # independent shards: each rank drew its own environments
    assert not np.array_equal(np.load(tmp_path / "M0.npy"), np.load(tmp_path / "M1.npy"))
    # BASELINE north_star: Go2 at a fixed GLOBAL batch split over the ranks (50 = 25 + 25)
    ns = line["north_star"]
    assert ns["global_envs"] == 50 and ns["envs_per_gpu"] == 25 and ns["n_gpus"] == 2
    assert ns["converged_frac"] == 1.0 and ns["target"] == 1e6
    assert abs(ns["value"] - 50 * 3 / (ns["ms_per_step"] * 3 / 1e3)) <= 1e-6 * ns["value"]
    # configs[4]: 8 Go2 + 8 WaLTER per rank through the multi-model call
    mx = line["mixed"]
    assert mx["config"]["global_envs"] == 2 * 2 * 8 and mx["config"]["envs_per_gpu"] == 16
    assert mx["converged_frac"] == 1.0
    # host-fed tick: per-GPU batches 16 and 32, both input forms, every rank's envs counted
    hf = line["host_fed"]
    assert hf["depth"] == 2 and set(hf["per_gpu"]) == {"16", "32"}
    for nenv in (16, 32):
        for form in ("qp", "joint_states", "joint_states_warm"):
            r = hf["per_gpu"][str(nenv)][form]
            assert r["global_envs"] == 2 * nenv and r["converged_frac"] == 1.0
            assert r["h2d_GBps"] > 0 and r["bound"] == "h2d (PCIe)"
            assert r["value"] > 0 and r["serial_depth1"]["value"] > 0
            assert r["bytes_per_env_h2d"] == (7664 - 96 if form == "qp" else (19 + 18 + 30 + 4) * 8)
            assert r["mean_ipm_iters"] == 10.0


def test_bench_launcher(monkeypatch):
    """--gpus N > 1 without WORLD_SIZE: bench.py starts N ranks through torch.distributed.run on
    127.0.0.1; WORLD_SIZE that disagrees with --gpus is refused."""
    import subprocess
    import bench
    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: seen.update(cmd=cmd, env=env) or 0)
    argv = ["--gpus", "4", "--steps", "7"]
    assert bench.launch_ranks(bench.parse_args(argv), argv) == 0
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert bench.launch_ranks(bench.parse_args(["--gpus", "1"]), ["--gpus", "1"]) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.launch_ranks(bench.parse_args(["--gpus", "4"]), ["--gpus", "4"]) == 2
    assert bench.launch_ranks(bench.parse_args(["--gpus", "2"]), ["--gpus", "2"]) is None
