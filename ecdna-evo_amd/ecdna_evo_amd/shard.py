"""Replicate sharding across GPUs/processes and the single reduction step.

The reference's only parallelism is independent replicates (rayon over replicate ids,
src/main.rs:221-224; cluster array jobs with distinct --seed, src/main.rs:213). Here replicates
are split into contiguous global-id ranges, one per rank; because every replicate's RNG stream
is keyed by its GLOBAL id (include/ecdna_ssa.h), per-replicate results are identical for any
number of ranks, and the pooled histogram of a G-rank run is the sum of the shards' histograms —
one all-reduce (RCCL over xGMI on GPUs, gloo in CPU tests). Nothing else is exchanged.
"""
from __future__ import annotations

from typing import Tuple


def shard_range(rank: int, world: int, total: int) -> Tuple[int, int]:
    """Strong scaling: global ids [first, first + n) of `rank` when `total` replicates are split."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    first = rank * total // world
    last = (rank + 1) * total // world
    return first, last - first


def interleaved_range(rank: int, world: int, total: int) -> Tuple[int, int, int]:
    """Strong scaling, interleaved: `rank` runs global ids rank, rank + world, rank + 2 world, ... < total,
    as (first, n, stride) for RunSpec(first_replicate, n_replicates, replicate_stride). Every rank gets
    the same mix of parameter sets, so an ABC sweep whose sets differ in cost (C4: initial copy numbers
    1 .. 128) is balanced across GPUs; contiguous shards would hand each GPU one cost class."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    n = (total - rank + world - 1) // world if total > rank else 0
    return rank, n, world


def weak_range(rank: int, per_rank: int) -> Tuple[int, int]:
    """Weak scaling: every rank runs `per_rank` replicates; rank g owns [g*per_rank, (g+1)*per_rank)."""
    return rank * per_rank, per_rank


def reduce_outputs(hist, totals, group=None) -> None:
    """Sum the per-rank copy-number histograms and totals in place (int64 tensors: u64 counts stay
    far below 2^63). The histogram bins and totals words are plain integer sums, so the result is
    exact and independent of the reduction order."""
    import torch.distributed as dist

    dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)
