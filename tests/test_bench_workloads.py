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


def test_c5_bin_kmax_by_replicates_per_gpu():
    """C5 takes K = 32 where a GPU holds more replicates than K = 64's grid has lanes (the whole run on one GPU), and
    K = 64 for the 8-, 4- and 2-GPU shards (profiles/r04s_c5_kmax.txt)."""
    total = bench.WORKLOADS["c5"][0]
    assert bench.workload_spec(0, total, total, workload="c5").bin_kmax == 32
    for gpus in (2, 4, 8):
        assert bench.workload_spec(0, total // gpus, total, workload="c5").bin_kmax == 64
    assert bench.workload_spec(0, total, total, workload="c5", bin_kmax=64).bin_kmax == 64
