"""bench.py's workloads (BASELINE.json configs C2-C5) on the CPU: every rank's shard is a valid run of
the engine's ABI, the shards of a strong-scaling workload partition its total, C4's interleaved shards
give every rank every parameter set, and a few replicates of each workload run through the oracle with
the bookkeeping identities of the reference's events (tests/test_gpu_statistics.py runs them at full
size on the GPU)."""
import numpy as np
import pytest

import bench
from ecdna_evo_amd import abi, shard


@pytest.mark.parametrize("workload", sorted(bench.WORKLOADS))
@pytest.mark.parametrize("world", [1, 2, 8])
def test_workload_shards_partition_the_total(workload, world):
    total = bench.WORKLOADS[workload][0]
    if workload == "c3":
        total *= world  # weak scaling: 2^20 per rank
    ids = []
    for rank in range(world):
        if workload == "c3":
            first, n = shard.weak_range(rank, total // world)
            stride = 1
        else:
            first, n, stride = shard.interleaved_range(rank, world, total)
        spec = bench.workload_spec(first, n, total, workload=workload, stride=stride)
        p = spec.params()
        assert p.n_replicates == n and (p.replicate_stride or 1) == stride
        last = spec.last_replicate()
        assert last // p.reps_per_set < p.n_param_sets
        if workload == "c4":  # interleaved: every rank holds all 1024 sets, 4096 / world replicates each
            sets = np.bincount((spec.replicate_ids() // p.reps_per_set).astype(np.int64), minlength=1024)
            assert np.all(sets == 4096 // world)
        ids.append(spec.replicate_ids())
    ids = np.sort(np.concatenate(ids))
    np.testing.assert_array_equal(ids, np.arange(total, dtype=np.uint64))


@pytest.mark.parametrize("workload", sorted(bench.WORKLOADS))
def test_workload_sample_runs_on_the_oracle(oracle_mod, workload):
    total = bench.WORKLOADS[workload][0]
    n = 1 if workload == "c5" else 24
    stride = total // n if workload == "c4" else 1
    spec = bench.workload_spec(0, n, total, workload=workload, stride=stride)
    r = oracle_mod.run(spec, mode="philox", n_threads=4)
    s = r.summaries
    assert np.all(s["error"] == 0)
    ev = s["events_by_type"].astype(np.int64)
    np.testing.assert_array_equal(ev.sum(axis=1), s["iters"].astype(np.int64))
    assert int(r.totals["replicates"].sum()) == n
    if workload == "c2":  # pure birth: exactly max_cells - 1 events from one cell (or the time cap)
        full = s["stop_reason"] == abi.STOP_MAX_CELLS
        assert np.all(s["iters"][full] == 10_000 - 1)
    if workload == "c5":  # 1,000 initial cells; the run ends at 1e6 cells or extinction
        assert s["stop_reason"][0] in (abi.STOP_MAX_CELLS, abi.STOP_ABSORBING)


@pytest.mark.parametrize("workload,kmax", [("c2", 32), ("c3", 32), ("c4", 64), ("c5", 64)])
def test_workload_bin_kmax_defaults(workload, kmax):
    """bench.py's K per workload (K = 32 where the pick scan dominates, 64 where copy numbers
    spread); an explicit --bin-kmax overrides it; the row store has no K."""
    total = bench.WORKLOADS[workload][0]
    assert bench.workload_spec(0, 8, total, workload=workload).bin_kmax == kmax
    assert bench.workload_spec(0, 8, total, workload=workload, bin_kmax=256).bin_kmax == 256
    assert bench.workload_spec(0, 8, total, workload=workload, store="rows").bin_kmax == 0


def _kmax_by_id(workload, world, **kw):
    """{global replicate id: K it runs at} over every rank's contexts of a `world`-GPU bench run (bench.rank_parts)."""
    ids, ks = [], []
    for rank in range(world):
        rp = bench.rank_parts(workload, world, rank, **kw)
        assert sum(sp.n_replicates for sp, _ in rp.parts) == rp.spec.n_replicates
        for sp, _ in rp.parts:
            ids.append(sp.replicate_ids())
            ks.append(np.full(sp.n_replicates, sp.bin_kmax, dtype=np.uint16))
    ids, ks = np.concatenate(ids), np.concatenate(ks)
    order = np.argsort(ids, kind="stable")
    return ids[order], ks[order]


@pytest.mark.parametrize("workload,kw", [("c5", {}), ("c4", {}), ("c2", {}), ("c3", {"scaling": "strong"}),
                                         ("c4", {"k0_split": "off"}), ("c5", {"bin_kmax": 32})])
def test_every_gpu_count_runs_each_replicate_at_the_same_k(workload, kw):
    """K is part of the draw mapping, so a replicate's results depend on its id and
    the workload only if every GPU count runs it at the same K. For each fixed-total workload, every rank of every GPU
    count from 1 to 8 (and 16) together runs each id exactly once and at the K of the one-GPU run: C5 at K = 64 (round
    5 took K = 32 on one GPU only), C4's k0 = 128 sets at K = 256 under the k0 split at every count (round 5 split only
    at 1, 2, 4 and 8)."""
    ids1, k1 = _kmax_by_id(workload, 1, **kw)
    assert len(ids1) == bench.WORKLOADS[workload][0] if workload != "c3" else len(ids1) == 1 << 20
    for world in (2, 3, 4, 5, 6, 7, 8, 16):
        ids, k = _kmax_by_id(workload, world, **kw)
        np.testing.assert_array_equal(ids, ids1, err_msg=f"{workload} at {world} GPUs: ids")
        np.testing.assert_array_equal(k, k1, err_msg=f"{workload} at {world} GPUs: K per replicate")
    if workload == "c5":
        assert set(np.unique(k1)) == {kw.get("bin_kmax", 64)}
    if workload == "c4" and not kw:
        assert set(np.unique(k1)) == {64, bench.C4_SPLIT_KMAX} and np.count_nonzero(k1 == 256) == len(k1) // 8


def test_c4_split_caps_cover_every_gpu_count():
    """The k0 split's grid caps (speed only) for GPU counts without a measured entry: the nearest measured count
    below."""
    assert bench.c4_split_caps(3) == bench.C4_SPLIT_CAPS[2]
    assert bench.c4_split_caps(7) == bench.C4_SPLIT_CAPS[4]
    assert bench.c4_split_caps(16) == bench.C4_SPLIT_CAPS[8]
    for g, caps in bench.C4_SPLIT_CAPS.items():
        assert bench.c4_split_caps(g) == caps


@pytest.mark.parametrize("world", sorted(set(bench.C4_SPLIT_CAPS) | {3, 5}))
def test_c4_k0_split_parts_partition_each_shard(world):
    """shard.k0_split on bench's C4 shards: two parts that together hold the shard's replicates in
    local order, the second exactly those of the k0 = 128 sets (K = 256), the first the rest (K = 64), each with
    its workgroup cap from bench.c4_split_caps (at any GPU count)."""
    total = bench.WORKLOADS["c4"][0]
    caps = bench.c4_split_caps(world)
    for rank in sorted({0, world - 1}):
        first, n, stride = shard.interleaved_range(rank, world, total)
        spec = bench.workload_spec(first, n, total, workload="c4", stride=stride)
        parts = shard.k0_split(spec, bench.C4_SPLIT_K0, bench.C4_SPLIT_KMAX, caps)
        assert [off for _, off in parts] == [0, parts[0][0].n_replicates]
        ids = np.concatenate([sp.replicate_ids() for sp, _ in parts])
        np.testing.assert_array_equal(ids, spec.replicate_ids())
        (narrow, _), (heavy, _) = parts
        k0 = np.array([max(d) for d in spec.init_per_set])
        assert np.all(k0[heavy.replicate_ids() // spec.reps_per_set] == 128)
        assert np.all(k0[narrow.replicate_ids() // spec.reps_per_set] < 128)
        assert (narrow.bin_kmax, heavy.bin_kmax) == (64, bench.C4_SPLIT_KMAX)
        assert (narrow.max_workgroups, heavy.max_workgroups) == caps
        assert heavy.params().max_workgroups == caps[1] and heavy.params().reserved0 == 0


def test_k0_split_refuses_a_shard_whose_heavy_sets_are_not_a_suffix():
    spec = abi.RunSpec(n_replicates=8, reps_per_set=2, rates=[(1.0, 1.0, 0.0, 0.0)] * 4,
                       init_per_set=[{1: 1}, {128: 1}, {1: 1}, {128: 1}], flags=abi.FLAG_BIN_STORE, bin_kmax=64)
    with pytest.raises(ValueError):
        shard.k0_split(spec, 128, 256, (1, 1))
    whole = shard.k0_split(abi.RunSpec(n_replicates=4, flags=abi.FLAG_BIN_STORE, bin_kmax=64), 128, 256, (1, 1))
    assert len(whole) == 1 and whole[0][0].bin_kmax == 64  # no heavy replicate: one part
    empty = shard.k0_split(abi.RunSpec(n_replicates=0, flags=abi.FLAG_BIN_STORE, bin_kmax=64), 1, 256, (1, 1))
    assert len(empty) == 1 and empty[0][0].n_replicates == 0  # (an empty shard stays one context)
