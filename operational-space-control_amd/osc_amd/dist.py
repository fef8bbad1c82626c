"""Multi-GPU bookkeeping of the batched solve: one process per GPU, each rank
solves its own shard of independent environments; there is NO collective on the data path.
torch.distributed is used only for the start/stop barriers and for reducing the per-rank
timings (max) and convergence counts (sum) into the whole-job numbers.  Backend "nccl" (RCCL)
on the GPU box; "gloo" in the CPU tests, which run the same functions."""
from __future__ import annotations

import dataclasses
import os

import torch

from .synth import SEED_BASE


@dataclasses.dataclass
class RankInfo:
    rank: int
    world: int
    local: int


def rank_info() -> RankInfo:
    return RankInfo(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
                    int(os.environ.get("LOCAL_RANK", "0")))


def shard_seed(rank: int, config_seed: int = 2) -> int:
    """Each rank draws its own environments (weak scaling: per-GPU work is fixed)."""
    return SEED_BASE + config_seed + 1000 * rank


def barrier(world: int) -> None:
    if world > 1:
        torch.distributed.barrier()


@dataclasses.dataclass
class JobStats:
    elapsed_s: float          # max over ranks of the timed region
    kernel_ms: float          # max over ranks
    setup_ms: float
    ipm_ms: float
    converged: float          # fraction over all ranks' environments
    total_envs: int


def reduce_stats(world: int, device: torch.device, nenv: int, elapsed_s: float, setup_ms: float,
                 ipm_ms: float, n_converged: int) -> JobStats:
    """Max-over-ranks timing and summed convergence counts (one all_reduce each)."""
    if world > 1:
        if torch.distributed.get_backend() == "gloo":   # CPU tests / one-GPU rehearsal
            device = torch.device("cpu")
        t = torch.tensor([elapsed_s, setup_ms + ipm_ms, setup_ms, ipm_ms], device=device,
                         dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        c = torch.tensor([float(n_converged), float(nenv)], device=device, dtype=torch.float64)
        torch.distributed.all_reduce(c)
        elapsed_s, kernel_ms, setup_ms, ipm_ms = (float(v) for v in t)
        converged, total = float(c[0] / c[1]), int(c[1])
    else:
        kernel_ms = setup_ms + ipm_ms
        converged, total = n_converged / max(nenv, 1), nenv
    return JobStats(elapsed_s, kernel_ms, setup_ms, ipm_ms, converged, total)


def job_value(stats: JobStats, steps: int) -> float:
    """Whole-job throughput: every rank's environments x steps / the slowest rank's time."""
    return stats.total_envs * steps / stats.elapsed_s
