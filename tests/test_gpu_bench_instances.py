"""The exact kernel instances the bench lines time, checked bit for bit at full size.

bench.py picks its instance per workload through ecdna_ssa_ctx_create's automatic rules (schedule, paired lanes,
rotation, K, the cost-ordered start): the C4 and C5 throughput claims rest on instances that the small parity
cases only cover in miniature. Each test below builds bench.py's own RunSpec (bench.workload_spec) for a
workload as the bench runs it — same flags (no event hash: the hash selects a different template instance),
same K, big_cap and cost hint, same shard layout — asserts the instance the context chose
(ecdna_ssa_ctx_instance, ABI v7), so the test fails if an automatic rule stops choosing it, then runs the whole
shard and compares a sample of its replicates with the philox oracle field by field (summaries incl. the f64 time
bits; the birth-death paths of src/main.rs:130-173)."""
import dataclasses
import os
import sys

import numpy as np
import pytest

from ecdna_evo_amd import abi, shard

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _bench():
    import importlib

    return importlib.import_module("bench")


def _run_with_instance(engine_mod, spec):
    with engine_mod.Context(spec) as ctx:
        ins = ctx.instance()
        ctx.launch()
        ctx.sync()
        return ins, ctx.download()


def _compare_sample(res, spec, oracle_mod, local, n, threads=8):
    """Local replicates local .. local + n - 1 of `res` against the oracle run of the same global ids."""
    stride = spec.stride()
    sub = dataclasses.replace(spec, first_replicate=spec.first_replicate + local * stride, n_replicates=n, _keep=[])
    c = oracle_mod.run(sub, mode="philox", n_threads=threads)
    for f in c.summaries.dtype.names:
        a, b = res.summaries[f][local:local + n], c.summaries[f]
        if f == "time":
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, err_msg=f"replicates {local}..{local + n - 1}: {f}")
    assert np.all(c.summaries["iters"] > 0)


@pytest.mark.gpu
def test_c5_bench_shard_instance_bit_exact(engine_mod, oracle_mod):
    """C5 8-GPU rank-0 shard as bench.py runs it (interleaved ids 0, 8, 16, ...; 32,768 replicates; K = 64 with u32
    counters; large-k row 2^16; f64 time, no hash): paired lanes under the max-ILP schedule; replicates 0..3 (about
    2e7 events each, to 1e6 cells) equal the oracle."""
    bench = _bench()
    first, n, stride = shard.interleaved_range(0, 8, 262_144)
    spec = bench.workload_spec(first, n, 262_144, workload="c5", stride=stride)
    assert spec.flags == abi.FLAG_BIN_STORE and spec.bin_kmax == 64 and spec.big_cap == 1 << 16
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 3, 1, 64, 1), ins
    assert ins["runtime_flags"] == 0 and ins["rotation"] == 0 and ins["n_chunks"] == 1, ins
    s = res.summaries
    assert np.all(s["error"] == 0)
    assert set(s["stop_reason"].tolist()) <= {abi.STOP_MAX_CELLS, abi.STOP_MAX_TIME, abi.STOP_ABSORBING}
    _compare_sample(res, spec, oracle_mod, 0, 4, threads=4)
    assert np.all(s["nminus"][:4] + s["nplus"][:4] == 1_000_000)  # these four reach the cap


@pytest.mark.gpu
def test_c4_bench_shard_instance_bit_exact(engine_mod, oracle_mod):
    """C4 8-GPU rank-3 shard as bench.py runs it (interleaved ids 3, 11, ...; 524,288 replicates over all 1024 sets;
    K = 64 / u16; costliest sets first from set_cost_hint): the max-ILP schedule without rotation; 64 replicates of
    set 1000 (k0 = 128: 256-bit binomials, cells beyond the bins) and 64 of set 37 (k0 = 1) equal the oracle."""
    bench = _bench()
    first, n, stride = shard.interleaved_range(3, 8, 4_194_304)
    spec = bench.workload_spec(first, n, 4_194_304, workload="c4", stride=stride)
    assert spec.set_cost_hint is not None and spec.bin_kmax == 64 and spec.flags == abi.FLAG_BIN_STORE
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 1, 0, 64, 0), ins
    assert ins["cost_order"] == 1 and ins["rotation"] == 0 and ins["runtime_flags"] == 0, ins
    assert np.all(res.summaries["error"] == 0) and np.all(res.totals["replicates"] == 512)
    for set_id in (1000, 37):
        m0 = (set_id * 4096 - first + stride - 1) // stride  # first local replicate of the set
        _compare_sample(res, spec, oracle_mod, m0, 64)


@pytest.mark.gpu
def test_c4_bench_shard_k0_split_bit_exact(engine_mod, oracle_mod):
    """C4 8-GPU rank-5 shard split as bench.py runs it (C4_SPLIT_CAPS[8]): the k0 = 128 sets' 65,536 replicates on a
    K = 256 context and the other 458,752 on K = 64, both launched concurrently on two streams with capped grids.
    Every replicate finishes without error; samples of set 1001 (heavy part, K = 256: its cells stay binned) and set
    200 (K = 64) equal the oracle at their part's K, and the concurrent run's summaries equal the parts run alone."""
    import torch

    bench = _bench()
    first, n, stride = shard.interleaved_range(5, 8, 4_194_304)
    spec = bench.workload_spec(first, n, 4_194_304, workload="c4", stride=stride)
    parts = shard.k0_split(spec, bench.C4_SPLIT_K0, bench.C4_SPLIT_KMAX, bench.C4_SPLIT_CAPS[8])
    assert [(sp.n_replicates, sp.bin_kmax, off) for sp, off in parts] == [(458_752, 64, 0), (65_536, 256, 458_752)]
    ctxs = [engine_mod.Context(sp) for sp, _ in parts]
    try:
        streams = [torch.cuda.Stream() for _ in ctxs]
        for c, st in zip(ctxs, streams):
            c.launch(st.cuda_stream)
        torch.cuda.synchronize()
        res = []
        for (sp, _), c in zip(parts, ctxs):
            c.sync()
            res.append(c.download())
            ins = c.instance()  # the grid respects the part's cap
            assert ins["bin_kmax"] == sp.bin_kmax and ins["grid_lanes"] <= sp.max_workgroups * ins["block_lanes"], ins
    finally:
        for c in ctxs:
            c.close()
    for r in res:
        assert np.all(r.summaries["error"] == 0)
    _compare_sample(res[1], parts[1][0], oracle_mod, (1001 * 4096 - parts[1][0].first_replicate + stride - 1) // stride, 48)
    _compare_sample(res[0], parts[0][0], oracle_mod, (200 * 4096 - first + stride - 1) // stride, 48)
    alone = engine_mod.run(parts[1][0])
    for f in ("nminus", "nplus", "iters", "event_hash"):
        np.testing.assert_array_equal(alone.summaries[f], res[1].summaries[f], err_msg=f)
    np.testing.assert_array_equal(alone.summaries["time"].view(np.uint64), res[1].summaries["time"].view(np.uint64))


@pytest.mark.gpu
def test_c4_bench_whole_instance_bit_exact(engine_mod, oracle_mod):
    """C4 on one GPU as `bench.py --workload c4` runs it (4,194,304 replicates, K = 64 / u16, cost-ordered starts,
    16 replicates per lane): the 128-VGPR occupancy build (schedule 2) with the drain control, no rotation (a cost
    hint is given); samples of sets 1023 (k0 = 128, the costliest), 512 and 0 equal the oracle."""
    bench = _bench()
    spec = bench.workload_spec(0, 4_194_304, 4_194_304, workload="c4")
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 2, 0, 64, 0), ins
    assert ins["cost_order"] == 1 and ins["rotation"] == 0 and ins["drain_control"] == 1, ins
    assert np.all(res.summaries["error"] == 0) and np.all(res.totals["replicates"] == 4096)
    for set_id in (1023, 512, 0):
        _compare_sample(res, spec, oracle_mod, set_id * 4096 + 1000, 48)


@pytest.mark.gpu
def test_c5_bench_whole_instance_bit_exact(engine_mod, oracle_mod):
    """C5 on one GPU as `bench.py --workload c5` runs it (262,144 replicates, K = 64 with u32 counters, the K of its
    shards since round 6: two workgroups per CU, two replicates per lane; large-k row 2^16): the max-ILP schedule,
    unpaired; replicates 0..3 and two from the end (about 2e7 events each, to 1e6 cells) equal the oracle."""
    bench = _bench()
    spec = bench.workload_spec(0, 262_144, 262_144, workload="c5")
    assert spec.flags == abi.FLAG_BIN_STORE and spec.bin_kmax == 64 and spec.big_cap == 1 << 16
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 1, 0, 64, 1), ins
    assert ins["blocks_per_cu"] == 2 and ins["runtime_flags"] == 0, ins
    s = res.summaries
    assert np.all(s["error"] == 0) and np.all(s["stop_reason"] == abi.STOP_MAX_CELLS)
    _compare_sample(res, spec, oracle_mod, 0, 4, threads=4)
    _compare_sample(res, spec, oracle_mod, 262_142, 2, threads=2)


@pytest.mark.gpu
def test_c3_bench_instance_bit_exact(engine_mod, oracle_mod):
    """C3, the metric's line (2^20 replicates, K = 32 / u32, rotation): the max-ILP schedule (since draw mapping v6 it
    keeps the occupancy-first build's four workgroups per CU) with rotation on; replicates spread over the id range
    equal the oracle."""
    bench = _bench()
    spec = bench.workload_spec(0, 1 << 20, 1 << 20, workload="c3")
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 1, 0, 32, 1), ins
    assert ins["rotation"] == 1 and ins["runtime_flags"] == 0 and ins["blocks_per_cu"] == 4, ins
    for local in (0, 333_333, (1 << 20) - 256):
        _compare_sample(res, spec, oracle_mod, local, 256)


@pytest.mark.gpu
def test_c3_strong_8gpu_shard_instance_bit_exact(engine_mod, oracle_mod):
    """The metric's fixed-total reading at 8 GPUs (bench.py --scaling strong --gpus 8): rank 7's contiguous 1/8 of 2^20
    replicates (131,072, ids 917,504 .. 2^20 - 1; K = 32 / u32): half a replicate per lane of the four-workgroup grid, so
    the launch is 512 workgroups (two per CU, grid_lanes = the replicates) under the max-ILP schedule (at most one wave
    of replicates per SIMD... two here: 256 replicates per CU), unpaired (birth-death with more than half a wave per
    SIMD), no rotation; samples equal the oracle."""
    bench = _bench()
    first, n = shard.shard_range(7, 8, 1 << 20)
    assert (first, n) == (917_504, 131_072)
    spec = bench.workload_spec(first, n, 1 << 20, workload="c3")
    assert spec.bin_kmax == 32 and spec.flags == abi.FLAG_BIN_STORE
    ins, res = _run_with_instance(engine_mod, spec)
    assert (ins["kernel"], ins["schedule"], ins["paired"], ins["bin_kmax"], ins["bin_c32"]) == (1, 1, 0, 32, 1), ins
    assert ins["rotation"] == 0 and ins["runtime_flags"] == 0 and ins["n_chunks"] == 1, ins
    assert ins["grid_lanes"] == 131_072 and ins["blocks_per_cu"] == 2, ins  # the launched grid
    assert np.all(res.summaries["error"] == 0) and int(res.totals["replicates"][0]) == n
    for local in (0, 65_536, n - 256):
        _compare_sample(res, spec, oracle_mod, local, 256)


@pytest.mark.gpu
def test_instance_reports_the_launched_grid_of_an_underfilled_paired_run(engine_mod):
    """the instance names the grid actually launched, not the occupancy cap. A C5-shaped paired run of 8,192
    replicates launches ceil(8192 / 128 owners) = 64 workgroups of 256 lanes; a 1,000-replicate unpaired pure-birth run
    4 workgroups; ECDNA_SSA_MAX_BLOCKS caps both."""
    spec = abi.RunSpec(seed=1, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), n_replicates=8192, max_cells=2000,
                       max_time=5.0, init={1: 1000}, flags=abi.FLAG_BIN_STORE, bin_kmax=64)
    with engine_mod.Context(spec) as ctx:
        ins = ctx.instance()
    assert ins["paired"] == 1 and ins["grid_lanes"] == 64 * 256 and ins["blocks_per_cu"] == 1, ins
    spec2 = abi.RunSpec(seed=1, n_replicates=1000, max_cells=100, flags=abi.FLAG_BIN_STORE, bin_kmax=32)
    with engine_mod.Context(spec2) as ctx:
        ins2 = ctx.instance()
    assert ins2["paired"] == 0 and ins2["grid_lanes"] == 4 * 256, ins2
    os.environ["ECDNA_SSA_MAX_BLOCKS"] = "16"
    try:
        with engine_mod.Context(spec) as ctx:
            ins3 = ctx.instance()
    finally:
        del os.environ["ECDNA_SSA_MAX_BLOCKS"]
    assert ins3["grid_lanes"] == 16 * 256, ins3


def _rank_summaries(engine_mod, workload, world, rank, **kw):
    """(global ids, summaries) of every context bench.py's rank `rank` of `world` launches (bench.rank_parts), run one
    after another on this GPU (results never depend on the grid, the stream or what else runs)."""
    bench = _bench()
    rp = bench.rank_parts(workload, world, rank, **kw)
    ids, summ = [], []
    for sp, _ in rp.parts:
        res = engine_mod.run(sp)
        assert np.all(res.summaries["error"] == 0)
        ids.append(sp.replicate_ids())
        summ.append(res.summaries)
    return np.concatenate(ids), np.concatenate(summ)


def _assert_same_replicates(ids_a, summ_a, ids_b, summ_b, what):
    """every replicate of b is in a, with the same summary bit for bit (the f64 time as bits)"""
    order = np.argsort(ids_a, kind="stable")
    idx = order[np.minimum(np.searchsorted(ids_a[order], ids_b), len(ids_a) - 1)]
    np.testing.assert_array_equal(ids_a[idx], ids_b, err_msg=f"{what}: ids")
    for f in summ_b.dtype.names:
        a, b = summ_a[f][idx], summ_b[f]
        if f == "time":
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, err_msg=f"{what}: {f}")


@pytest.mark.gpu
def test_c5_8gpu_shard_equals_the_one_gpu_run(engine_mod):
    """the C5 8-GPU rank-0 shard (32,768 replicates, paired lanes) and the same ids inside the one-GPU
    bench spec (262,144 replicates, unpaired max-ILP) give the same summaries bit for bit: one K (64) for every GPU
    count (round 5 ran the one-GPU C5 at K = 32, a different draw mapping). The real shard and whole-run replicate
    counts, so the real instances; the cell cap 1e5 instead of 1e6 (u32 counters as at 1e6) keeps the test short."""
    ids1, s1 = _rank_summaries(engine_mod, "c5", 1, 0, max_cells=100_000)
    ids8, s8 = _rank_summaries(engine_mod, "c5", 8, 0, max_cells=100_000)
    assert len(ids1) == 262_144 and len(ids8) == 32_768
    _assert_same_replicates(ids1, s1, ids8, s8, "C5 8-GPU rank 0 vs 1 GPU")
    assert np.all(s8["stop_reason"] == abi.STOP_MAX_CELLS)


@pytest.mark.gpu
def test_c4_3gpu_shard_equals_the_one_gpu_run(engine_mod):
    """a C4 shard at a GPU count without measured split caps (3: rank 1's 1,398,101 interleaved
    replicates, split by k0 with the caps of 2 GPUs) against the one-GPU bench run of all 4,194,304 (split with the
    caps of 1 GPU): the same summaries bit for bit, the k0 = 128 replicates at K = 256 on both sides (round 5 split
    only at 1, 2, 4 and 8 GPUs, so a 3-GPU shard ran them at K = 64)."""
    ids1, s1 = _rank_summaries(engine_mod, "c4", 1, 0)
    ids3, s3 = _rank_summaries(engine_mod, "c4", 3, 1)
    assert len(ids1) == 4_194_304 and len(ids3) == 1_398_101
    _assert_same_replicates(ids1, s1, ids3, s3, "C4 3-GPU rank 1 vs 1 GPU")


@pytest.mark.gpu
def test_c3_fixed_total_8gpu_shard_equals_the_one_gpu_run(engine_mod):
    """The metric's fixed-total reading (bench.py --scaling strong): the 8-GPU rank-7 shard (131,072 contiguous ids,
    two waves per SIMD) equals the same ids of the one-GPU run (2^20 replicates, rotation) bit for bit."""
    ids1, s1 = _rank_summaries(engine_mod, "c3", 1, 0, scaling="strong")
    ids8, s8 = _rank_summaries(engine_mod, "c3", 8, 7, scaling="strong")
    assert len(ids1) == 1 << 20 and len(ids8) == 1 << 17
    _assert_same_replicates(ids1, s1, ids8, s8, "C3 fixed total, 8-GPU rank 7 vs 1 GPU")
