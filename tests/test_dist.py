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
