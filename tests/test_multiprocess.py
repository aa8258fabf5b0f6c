"""Multi-process sharding on CPU (gloo, world_size 2): the N>1 path of bench.py restated with the
oracle as the per-rank engine. Each rank runs its contiguous global-id shard; one all-reduce sums
histograms and totals; the result must be bit-identical to a single-process run of all replicates
(the 1-GPU == N-GPU identity)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ecdna_evo_amd import abi, shard


def _spec(first, n, total, stride=1):
    return abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, segregation=abi.SEG_BINOMIAL,
                       rates=((1.0, 1.0, 0.1, 0.1), (1.0, 1.5, 0.3, 0.3), (1.0, 2.0, 0.5, 0.2)),
                       reps_per_set=total // 3, first_replicate=first, n_replicates=n, replicate_stride=stride,
                       max_cells=500, hist_bins=129, flags=abi.FLAG_EVENT_HASH)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, total, port, outdir, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "ecdna-evo_amd"), os.path.join(os.path.dirname(here), "oracle")]
    import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    stride = 1
    if mode == "strong":
        first, n = shard.shard_range(rank, world, total)
    elif mode == "interleaved":
        first, n, stride = shard.interleaved_range(rank, world, total)
    else:
        first, n = shard.weak_range(rank, total // world)
    r = oracle.run(_spec(first, n, total, stride), mode="philox", n_threads=2)
    hist = torch.from_numpy(r.hist.astype(np.int64).reshape(-1).copy())
    tot = torch.from_numpy(r.totals.view(np.uint64).astype(np.int64).reshape(-1).copy())
    shard.reduce_outputs(hist, tot)
    np.save(os.path.join(outdir, f"summ{rank}.npy"), r.summaries)
    # the ABC step's exchange: every replicate's record in global order on every rank
    layout = {"strong": "contiguous", "interleaved": "interleaved", "weak": "weak"}[mode]
    gathered = shard.gather_structured(r.summaries, total, layout)
    np.save(os.path.join(outdir, f"gathered{rank}.npy"), gathered)
    if rank == 0:
        np.save(os.path.join(outdir, "hist.npy"), hist.numpy())
        np.save(os.path.join(outdir, "tot.npy"), tot.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["strong", "weak", "interleaved"])
def test_two_rank_shards_reduce_to_single_run(oracle_mod, tmp_path, mode):
    world, total = 2, 600
    mp.spawn(_worker, args=(world, total, _free_port(), str(tmp_path), mode), nprocs=world, join=True)
    full = oracle_mod.run(_spec(0, total, total), mode="philox")
    np.testing.assert_array_equal(np.load(tmp_path / "hist.npy"), full.hist.astype(np.int64).reshape(-1))
    np.testing.assert_array_equal(np.load(tmp_path / "tot.npy"), full.totals.view(np.uint64).astype(np.int64).reshape(-1))
    parts = [np.load(tmp_path / f"summ{r}.npy") for r in range(world)]
    if mode == "interleaved":  # rank r's replicate i is global id r + i * world
        summ = np.empty_like(full.summaries)
        for r, part in enumerate(parts):
            summ[r::world] = part
    else:
        summ = np.concatenate(parts)
    for f in full.summaries.dtype.names:
        np.testing.assert_array_equal(summ[f], full.summaries[f])
    for r in range(world):  # shard.gather_structured: bit-identical records in global id order on each rank
        g = np.load(tmp_path / f"gathered{r}.npy")
        assert g.dtype == full.summaries.dtype and len(g) == total
        assert g.tobytes() == full.summaries.tobytes()


def test_interleaved_calls_equal_one_call_per_set(oracle_mod):
    """G interleaved calls (first_replicate = g, replicate_stride = G) run exactly the replicates of one
    contiguous call: per-replicate results by global id, per-set histograms and totals sum to it."""
    total, world = 96, 5
    full = oracle_mod.run(_spec(0, total, total), mode="philox")
    hist = np.zeros_like(full.hist.astype(np.int64))
    for g in range(world):
        first, n, stride = shard.interleaved_range(g, world, total)
        assert n == len(range(g, total, world))
        r = oracle_mod.run(_spec(first, n, total, stride), mode="philox")
        for f in full.summaries.dtype.names:
            np.testing.assert_array_equal(r.summaries[f], full.summaries[f][g::world])
        hist += r.hist.astype(np.int64)
    np.testing.assert_array_equal(hist, full.hist.astype(np.int64))


def test_interleaved_ranges_partition():
    for total in (1, 7, 1000, 2**20 + 3):
        for world in (1, 2, 3, 8):
            ids = np.sort(np.concatenate([abi.RunSpec(first_replicate=f, n_replicates=n, replicate_stride=s).replicate_ids()
                                          for f, n, s in (shard.interleaved_range(r, world, total) for r in range(world))]))
            np.testing.assert_array_equal(ids, np.arange(total, dtype=np.uint64))


def test_shard_ranges_partition():
    for total in (1, 7, 1000, 2**20):
        for world in (1, 2, 3, 8):
            rs = [shard.shard_range(r, world, total) for r in range(world)]
            assert rs[0][0] == 0
            for (f0, n0), (f1, _) in zip(rs, rs[1:]):
                assert f0 + n0 == f1
            assert sum(n for _, n in rs) == total


def _gather_worker(rank, world, total, port, outdir, layout):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = np.arange(total)[shard.rank_ids(rank, world, total, layout)]
    # records derived from the global id (f64, two columns), so the expected gather is known
    local = torch.from_numpy(np.stack([ids * 0.5, -ids.astype(np.float64)], axis=1))
    out = shard.gather_records(local, total, layout)
    np.save(os.path.join(outdir, f"g{rank}.npy"), out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("layout,total", [("contiguous", 7), ("interleaved", 7), ("interleaved", 2), ("weak", 6)])
def test_three_rank_gather_records_ragged(tmp_path, layout, total):
    """Ragged shards (7 records over 3 ranks; a rank with none when total < world) come back in global
    id order on every rank."""
    world = 3
    mp.spawn(_gather_worker, args=(world, total, _free_port(), str(tmp_path), layout), nprocs=world, join=True)
    ids = np.arange(total, dtype=np.float64)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"g{r}.npy"), np.stack([ids * 0.5, -ids], axis=1))


def test_rank_ids_partition():
    for layout in ("contiguous", "interleaved"):
        for total in (0, 1, 7, 1000):
            for world in (1, 2, 3, 8):
                ids = np.sort(np.concatenate([np.arange(total)[shard.rank_ids(r, world, total, layout)]
                                              for r in range(world)]))
                np.testing.assert_array_equal(ids, np.arange(total))
    with pytest.raises(ValueError):
        shard.rank_ids(0, 2, 10, "blocks")
