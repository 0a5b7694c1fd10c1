"""Multi-GPU plumbing of the rollout: envs shard by global env id, one process per
GPU, and the only collective on the path is the advantage-normalisation all-reduce.

Env ids: every env's root seed derives from its global id (SeedManager.derive_env_seed(base, worker,
global_id), base.py:377-431 of the reference), so an env's trajectory does not depend on the number
of GPUs and there is no env-state exchange. Two partitions of the ids (`shard`):
* weak: rank g owns E envs, ids [g*E, (g+1)*E); the per-GPU work is fixed as N grows;
* strong (BASELINE configs[3]): E_total envs in all, rank g owns ids [g*E_total/N, (g+1)*E_total/N).

Advantage normalisation: the GAE kernel accumulates [sum A, sum A^2, n] in f64 per rank (one row
per module: one for the shared policy, W when every agent has its own); these 24 B per module are
SUM-all-reduced (RCCL over xGMI on MI355X, gloo on CPU) once per rollout, and every
rank normalises with the global mean/std: (A - mean) / max(1e-4, std) (RLlib's standardisation).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int]:
    """(rank, world_size) of the default process group, (0, 1) when not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def env_index_offset(envs_per_rank: int, rank: Optional[int] = None) -> int:
    """First global env id of `rank` when every rank owns envs_per_rank consecutive ids (both
    partitions: weak with envs_per_rank = E, strong with E_total / N)."""
    r = world()[0] if rank is None else rank
    return r * envs_per_rank


def shard(n_envs: int, scaling: str = "weak", rank: Optional[int] = None,
          world_size: Optional[int] = None) -> Tuple[int, int]:
    """(envs of this rank, its first global env id). weak: every rank owns n_envs envs; strong:
    n_envs in total split evenly (n_envs must divide by the rank count)."""
    r, n = world()
    r = r if rank is None else rank
    n = n if world_size is None else world_size
    if scaling == "weak":
        return n_envs, env_index_offset(n_envs, r)
    if scaling != "strong":
        raise ValueError(f"scaling must be 'weak' or 'strong', got {scaling!r}")
    if n_envs % n:
        raise ValueError(f"{n_envs} envs do not split evenly over {n} ranks")
    per = n_envs // n
    return per, env_index_offset(per, r)


def ranks_per_device() -> int:
    """Processes of this node that share one GPU: 1 with one rank per GPU (torchrun on an N-GPU node),
    LOCAL_WORLD_SIZE / device count when ranks outnumber the visible GPUs (the gloo rehearsal on one
    card). Counting devices does not initialise the GPU."""
    import os
    local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    n_dev = max(1, torch.cuda.device_count())
    return max(1, -(-local // n_dev))


def ea_mem_fraction(default: float = 0.25) -> float:
    """Episode-ahead memory budget of one rank's env handle (msc_env_desc.ea_mem_fraction: a fraction
    of the device memory free at create time). Ranks that share a card create their handles at about
    the same time and each sees the same free memory, so the budget is split between them: together
    they take at most `default` of the card, as one rank alone would."""
    return default / ranks_per_device()


def allreduce_adv_stats(stats: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce of the f64 [sum, sum_sq, n] advantage statistics ([3], or [G, 3]
    with one row per module when every agent has its own policy)."""
    if stats.dtype != torch.float64 or stats.numel() % 3 != 0 or stats.numel() == 0 or stats.shape[-1] != 3:
        raise ValueError("advantage statistics must be a float64 tensor of shape [3] or [G, 3]")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(stats, op=dist.ReduceOp.SUM, group=group)
    return stats


def mean_std(stats: torch.Tensor):
    """Global mean and (population) std from reduced [sum, sum_sq, n]: floats for a [3] table,
    lists of G floats each for a [G, 3] one (one row per module)."""
    rows = stats.reshape(-1, 3).tolist()
    out = []
    for s, ss, n in rows:
        if n <= 0:
            raise ValueError("no advantages")
        mean = s / n
        out.append((mean, math.sqrt(max(ss / n - mean * mean, 0.0))))
    if stats.dim() == 1:
        return out[0]
    return [m for m, _ in out], [sd for _, sd in out]
