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


def k0_split(spec, k0_min: int, wide_kmax: int, caps: Tuple[int, int]):
    """A bin-store shard split by initial copy number ("C4 shard split"): the replicates whose
    parameter set starts with a cell of k0 >= k0_min copies run on a second context with K = wide_kmax, whose bins
    keep their cells in LDS (with K = 64 most of them sit in the large-k row in HBM), concurrently with the rest;
    caps = (max_workgroups of the rest, of the heavy part) so that the two persistent grids share the GPU. The
    heavy replicates must be a suffix of the shard's local order (the C4 sweep orders its sets by k0). Each
    replicate's results are those of a run at its part's K (bin_kmax orders the cells, so K is part of the draw
    mapping). Returns [(spec, local offset)] of the non-empty parts."""
    import dataclasses

    import numpy as np

    n, first, stride = spec.n_replicates, spec.first_replicate, spec.stride()
    if n == 0:
        return [(spec, 0)]
    if spec.init_per_set is None:
        k0s = [max(spec.init or {1: 1})] * len(spec.rates)
    else:
        k0s = [max(d) if d else 0 for d in spec.init_per_set]
    sets = (first + np.arange(n, dtype=np.int64) * stride) // int(spec.params().reps_per_set)
    heavy = np.asarray(k0s)[sets] >= k0_min
    i0 = int(np.argmax(heavy)) if heavy.any() else n
    if not np.all(heavy[i0:]):
        raise ValueError("k0_split: the heavy replicates are not a suffix of the shard")
    parts = []
    if i0 > 0:
        parts.append((dataclasses.replace(spec, n_replicates=i0, max_workgroups=caps[0], _keep=[]), 0))
    if i0 < n:
        parts.append((dataclasses.replace(spec, first_replicate=first + i0 * stride, n_replicates=n - i0,
                                          bin_kmax=wide_kmax, max_workgroups=caps[1], _keep=[]), i0))
    return parts


def reduce_outputs(hist, totals, group=None) -> None:
    """Sum the per-rank copy-number histograms and totals in place (int64 tensors: u64 counts stay
    far below 2^63). The histogram bins and totals words are plain integer sums, so the result is
    exact and independent of the reduction order."""
    import torch.distributed as dist

    dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(totals, op=dist.ReduceOp.SUM, group=group)


def rank_ids(rank: int, world: int, total: int, layout: str):
    """The global replicate ids a rank owns under `layout`, as a slice of range(total): "contiguous"
    (shard_range), "interleaved" (interleaved_range) or "weak" (weak_range with total // world each)."""
    if layout == "contiguous":
        first, n = shard_range(rank, world, total)
        return slice(first, first + n)
    if layout == "interleaved":
        first, n, stride = interleaved_range(rank, world, total)
        return slice(first, first + n * stride, stride)
    if layout == "weak":
        first, n = weak_range(rank, total // world)
        return slice(first, first + n)
    raise ValueError(f"unknown shard layout {layout!r}")


def gather_records(local, total: int, layout: str = "contiguous", group=None):
    """All-gather per-replicate records into global replicate order on every rank.

    `local` is a [n_local, W] tensor of this rank's records in its own order (row i = the i-th id of
    rank_ids), on the process group's device (CUDA for RCCL, CPU for gloo). The ABC sweep's rejection
    step (abc.md:38-55) needs every replicate's statistics in one place; this is the one exchange it
    adds beside the histogram all-reduce (a gather of R/G records per rank). Shards differ
    by at most one record, so each rank pads to the largest and one all_gather moves them."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ids = [range(total)[rank_ids(r, world, total, layout)] for r in range(world)]
    if local.shape[0] != len(ids[rank]):
        raise ValueError(f"rank {rank} holds {local.shape[0]} records, its shard has {len(ids[rank])}")
    width = tuple(local.shape[1:])
    cap = max(len(x) for x in ids)
    padded = torch.zeros((cap,) + width, dtype=local.dtype, device=local.device)
    padded[: local.shape[0]] = local
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    out = torch.empty((sum(len(x) for x in ids),) + width, dtype=local.dtype, device=local.device)
    for r in range(world):
        out[rank_ids(r, world, total, layout)] = parts[r][: len(ids[r])]
    return out


def gather_structured(arr, total: int, layout: str = "contiguous", device=None, group=None):
    """gather_records for a numpy structured array (ecdna_rep_summary_t or ecdna_rep_stats_t records as
    abi.SUMMARY_DTYPE / abi.STATS_DTYPE): the records travel as raw bytes, so every field comes back
    bit for bit. `device`: where the exchange buffers live ("cuda" under RCCL, None = CPU for gloo)."""
    import numpy as np
    import torch

    raw = np.ascontiguousarray(arr).view(np.uint8).reshape(len(arr), arr.dtype.itemsize)
    t = torch.from_numpy(raw.copy())
    if device is not None:
        t = t.to(device)
    g = gather_records(t, total, layout, group).cpu().numpy()
    return np.ascontiguousarray(g).view(arr.dtype).reshape(-1)
