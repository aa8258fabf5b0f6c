"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle (philox mode), bit for bit.

For every case in tests/cases.py the per-replicate summaries (final n-/n+, iterations, per-type
event counts, uneven count, final time, event hash, stop reason, error), the final N+ rows in
swap_remove order, the pooled copy-number histograms and the per-set totals must be identical.
"""
import numpy as np
import pytest

from cases import bin_cases, cases
from ecdna_evo_amd import abi

H = abi.FLAG_EVENT_HASH

CASES = cases()
BIN_CASES = bin_cases()


def _compare(gpu, cpu, name):
    gs, cs = gpu.summaries, cpu.summaries
    for f in gs.dtype.names:
        if f == "time":
            np.testing.assert_array_equal(gs[f].view(np.uint64), cs[f].view(np.uint64), err_msg=f"{name}: {f}")
        else:
            np.testing.assert_array_equal(gs[f], cs[f], err_msg=f"{name}: {f}")
    for i in range(len(gs)):
        np.testing.assert_array_equal(gpu.row(i), cpu.row(i), err_msg=f"{name}: row {i}")
    np.testing.assert_array_equal(gpu.hist, cpu.hist, err_msg=f"{name}: hist")
    for f in gpu.totals.dtype.names:
        np.testing.assert_array_equal(gpu.totals[f], cpu.totals[f], err_msg=f"{name}: totals.{f}")
    if cpu.snapshots is not None:
        for f in ("nminus", "nplus", "taken"):
            np.testing.assert_array_equal(gpu.snapshots[f], cpu.snapshots[f], err_msg=f"{name}: snapshots.{f}")
        np.testing.assert_array_equal(gpu.snapshots["time"].view(np.uint64), cpu.snapshots["time"].view(np.uint64))
        if cpu.snapshot_rows is not None:
            for i in range(len(gs)):
                for s in range(cpu.snapshots.shape[1]):
                    np.testing.assert_array_equal(gpu.snapshot_row(i, s), cpu.snapshot_row(i, s),
                                                  err_msg=f"{name}: snapshot row {i}/{s}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_matches_oracle(name, engine_mod, oracle_mod):
    spec = CASES[name]
    gpu = engine_mod.run(spec, want_rows=True)
    cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
    _compare(gpu, cpu, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(BIN_CASES))
def test_gpu_bin_store_matches_oracle(name, engine_mod, oracle_mod):
    """The bin store (ECDNA_FLAG_BIN_STORE) against the oracle's restatement of it, bit for bit; rows
    in canonical order."""
    spec = BIN_CASES[name]
    gpu = engine_mod.run(spec, want_rows=True)
    cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
    _compare(gpu, cpu, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(n for n, c in BIN_CASES.items() if not c.flags & 0x1))
def test_gpu_bin_store_fast_variant_matches_oracle(name, engine_mod, oracle_mod):
    """The bin store's compile-time variant for f64 time without the event hash (the bench's kernel):
    every case with the hash switched off, all outputs but the (zero) hash bit for bit."""
    import dataclasses

    from ecdna_evo_amd import abi

    spec = dataclasses.replace(BIN_CASES[name], flags=BIN_CASES[name].flags & ~abi.FLAG_EVENT_HASH, _keep=[])
    _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True), name)


@pytest.mark.gpu
def test_gpu_stop_reasons_and_errors_exercised(engine_mod):
    """The case list really reaches every stop reason and error code."""
    from ecdna_evo_amd import abi

    seen_stop, seen_err = set(), set()
    for name, spec in CASES.items():
        r = engine_mod.run(spec)
        seen_stop |= set(r.summaries["stop_reason"].tolist())
        seen_err |= set(r.summaries["error"].tolist())
    assert {abi.STOP_MAX_CELLS, abi.STOP_MAX_TIME, abi.STOP_MAX_ITER, abi.STOP_ABSORBING, abi.STOP_ERROR} <= seen_stop
    assert {abi.REP_ERR_OVERFLOW, abi.REP_ERR_EMPTY, abi.REP_ERR_CELL_CAP} <= seen_err


@pytest.mark.gpu
def test_gpu_chunked_run_matches_single_chunk(engine_mod, monkeypatch):
    """Chunking by HBM capacity (forced tiny here) does not change any result."""
    spec = CASES["bd_binomial"]
    whole = engine_mod.run(spec)
    monkeypatch.setenv("ECDNA_SSA_MAX_CHUNK", "7")
    chunked = engine_mod.run(spec)
    for f in whole.summaries.dtype.names:
        np.testing.assert_array_equal(whole.summaries[f], chunked.summaries[f])
    np.testing.assert_array_equal(whole.hist, chunked.hist)


@pytest.mark.gpu
def test_gpu_grid_size_does_not_change_results(engine_mod, monkeypatch):
    """Results depend on replicate ids only, not on which lane ran them (persistent refill)."""
    from ecdna_evo_amd import abi

    spec = abi.RunSpec(seed=31, process=abi.BIRTH_DEATH, rates=((1.0, 1.2, 0.8, 0.8),), n_replicates=3000,
                       max_cells=300, init={1: 2}, flags=abi.FLAG_EVENT_HASH)
    a = engine_mod.run(spec)
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", "1")  # 256 lanes refill ~12 times each
    b = engine_mod.run(spec)
    np.testing.assert_array_equal(a.summaries["event_hash"], b.summaries["event_hash"])
    np.testing.assert_array_equal(a.hist, b.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("kmax", [64, 256])
def test_gpu_bin_store_grid_and_chunks_do_not_change_results(kmax, engine_mod, monkeypatch):
    """Bin store: results depend on replicate ids only (lane refill, chunking)."""
    from ecdna_evo_amd import abi

    spec = abi.RunSpec(seed=31, process=abi.BIRTH_DEATH, rates=((1.0, 1.2, 0.8, 0.8),), n_replicates=3000,
                       max_cells=300, init={1: 2, 70: 1}, bin_kmax=kmax,
                       flags=abi.FLAG_EVENT_HASH | abi.FLAG_BIN_STORE)
    a = engine_mod.run(spec)
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", "1")
    b = engine_mod.run(spec)
    monkeypatch.setenv("ECDNA_SSA_MAX_CHUNK", "101")
    c = engine_mod.run(spec)
    for r in (b, c):
        np.testing.assert_array_equal(a.summaries["event_hash"], r.summaries["event_hash"])
        np.testing.assert_array_equal(a.hist, r.hist)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pb_binomial_c1", "bd_binomial", "bd_shrink", "bd_turnover", "big_copies", "abc_sets"])
def test_gpu_hbm_only_variant_matches_oracle(name, engine_mod, oracle_mod, monkeypatch):
    """The A/B reference variant without the LDS tail window (ECDNA_SSA_WINDOW=0) is exact too."""
    monkeypatch.setenv("ECDNA_SSA_WINDOW", "0")
    spec = CASES[name]
    _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True), name)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [H, H | abi.FLAG_BIN_STORE])
def test_gpu_edge_sizes_match_oracle(flags, engine_mod, oracle_mod):
    """Zero replicates, one replicate, and global ids at the top of the u64 range (Philox counter words
    rid_hi = 0xffffffff, interleaved with a stride) against the oracle."""
    empty = abi.RunSpec(seed=3, n_replicates=0, reps_per_set=1, max_cells=100, flags=flags)
    r = engine_mod.run(empty)
    assert len(r.summaries) == 0 and int(r.hist.sum()) == 0 and int(r.totals["replicates"].sum()) == 0
    top = 2**64 - 1
    for spec in (abi.RunSpec(seed=4, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=1,
                             max_cells=2000, flags=flags),
                 abi.RunSpec(seed=5, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),),
                             first_replicate=top - 1 - 3 * 36, n_replicates=37, replicate_stride=3, reps_per_set=top,
                             max_cells=800, flags=flags)):
        gpu = engine_mod.run(spec, want_rows=True)
        cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
        _compare(gpu, cpu, f"edge/{spec.n_replicates}")


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [H, H | abi.FLAG_BIN_STORE])
def test_gpu_extreme_rates_match_oracle(flags, engine_mod, oracle_mod):
    """Rates at the ends of the allowed range (2^-60 and 2^60, ABI v8) and mixtures of them: the f32 time step
    soft_log / a0 spans its whole range (the division without the compiler's range handling must
    still equal the IEEE quotient), bit for bit against the oracle's C division."""
    lo, hi = 2.0**-60, 2.0**60
    for i, rates in enumerate([(lo, lo, 0.0, lo), (hi, hi, hi / 3, hi / 2), (lo, hi, lo, 0.0), (1.1 * lo, 1.5, 0.3, 7 * lo),
                               (hi, 1e-12, 0.0, 3.3e11)]):
        spec = abi.RunSpec(seed=70 + i, process=abi.BIRTH_DEATH, rates=(rates,), n_replicates=300,
                           max_cells=400, init={1: 2, 40: 1}, max_time=float("inf"), flags=flags)
        _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True),
                 f"rates {rates}")


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["0", "1", "3"])
@pytest.mark.parametrize("name", sorted(BIN_CASES))
def test_gpu_bin_store_both_schedules_match_oracle(name, sched, engine_mod, oracle_mod, monkeypatch):
    """The bin stepper's instruction schedules (ECDNA_SSA_SCHED: 0 = occupancy-first, the large-run
    default; 1 = max-ILP, taken automatically for at most one wave of replicates per SIMD, i.e. for every
    case here; 3 = the 128-VGPR build of the K = 64 / u16 kernel, taken automatically at four or more
    replicates per lane, the default elsewhere) are the same kernels: each bit for bit against the oracle."""
    monkeypatch.setenv("ECDNA_SSA_SCHED", sched)
    spec = BIN_CASES[name]
    _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True), name)


@pytest.mark.gpu
@pytest.mark.parametrize("blocks", ["0", "2"])
@pytest.mark.parametrize("name", sorted(BIN_CASES))
def test_gpu_bin_store_paired_lanes_match_oracle(name, blocks, engine_mod, oracle_mod, monkeypatch):
    """Paired lanes forced (ECDNA_SSA_PAIR = 1; DESIGN.md §5: in the N- fast-forward lane l < 32 runs events
    e and e + 1, lane l + 32 forms the Philox block and soft log of e + 1) on every bin-store case, bit for bit
    against the oracle; on the default grid and squeezed onto two workgroups (owners refill many times). The
    kernels without a paired instance (pure birth, K = 256, snapshots) run unpaired and must match all the same."""
    monkeypatch.setenv("ECDNA_SSA_PAIR", "1")
    if blocks != "0":
        monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", blocks)
    spec = BIN_CASES[name]
    _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True), name)


def _no_uneven_small_specs():
    """The no-uneven rule's redraws at small copy numbers (n = 2k <= 32: a draw is rejected with probability
    2^(1-n), so k = 1 cells redraw about once per division and reach the spares and then Philox blocks):
    both processes, both stores, K = 32 and 64, spares refilled by N- and death events."""
    out = {}
    for i, (proc, rates, init) in enumerate([
            (abi.PURE_BIRTH, (1.0, 1.0, 0.0, 0.0), {1: 1}),
            (abi.BIRTH_DEATH, (1.0, 1.5, 0.3, 0.3), {1: 3, 2: 2, 16: 1}),
            (abi.BIRTH_DEATH, (1.4, 1.0, 0.6, 0.2), {1: 4, 0: 3}),
    ]):
        for store, kmax in (("rows", 0), ("bins", 32), ("bins", 64)):
            flags = H | (abi.FLAG_BIN_STORE if store == "bins" else 0)
            out[f"nu{i}_{store}{kmax or ''}"] = abi.RunSpec(
                seed=110 + i, process=proc, segregation=abi.SEG_BINOMIAL_NO_UNEVEN, rates=(rates,), init=init,
                n_replicates=300, max_cells=1200, bin_kmax=kmax, flags=flags)
    return out


NU_SPECS = _no_uneven_small_specs()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(NU_SPECS))
def test_gpu_no_uneven_small_redraws_match_oracle(name, engine_mod, oracle_mod):
    """ssa_device.hpp's redraw_even_small (the accepted word found branch-free over the base words, then four
    at a time over Philox blocks) against the oracle's try-by-try loop, bit for bit."""
    spec = NU_SPECS[name]
    _compare(engine_mod.run(spec, want_rows=True), oracle_mod.run(spec, mode="philox", want_rows=True), name)


def _nminus_heavy_specs():
    """Populations that become mostly N- (N- fitter than N+; uneven splits of k = 1 cells feed it), so the
    N- fast-forward runs most events; stops that land inside it (max_iter, max_time,
    cells); both processes, K = 32 / 64 / 256, f32 time, the event hash on and off."""
    out = {}
    for i, (proc, rates, extra) in enumerate([
            (abi.BIRTH_DEATH, (1.6, 1.0, 0.3, 0.3), dict(max_cells=3000)),
            (abi.BIRTH_DEATH, (1.0, 1.0, 0.9, 0.9), dict(max_cells=5000, init={1: 40})),
            (abi.PURE_BIRTH, (2.0, 1.0, 0.0, 0.0), dict(max_cells=2500)),
            (abi.BIRTH_DEATH, (1.6, 1.0, 0.3, 0.3), dict(max_cells=100_000, max_iter=900)),
            (abi.BIRTH_DEATH, (1.6, 1.0, 0.3, 0.3), dict(max_cells=100_000, max_time=4.5)),
            (abi.BIRTH_DEATH, (1.6, 1.0, 0.3, 0.3), dict(max_cells=3000, flags_extra=abi.FLAG_TIME_F32)),
    ]):
        for kmax in (32, 64, 256):
            for hash_ in (0, H):
                d = dict(extra)
                fx = d.pop("flags_extra", 0)
                d.setdefault("init", {1: 3})
                out[f"ff{i}_k{kmax}_h{int(bool(hash_))}"] = abi.RunSpec(
                    seed=90 + i, process=proc, rates=(rates,), n_replicates=700, bin_kmax=kmax,
                    flags=abi.FLAG_BIN_STORE | hash_ | fx, **d)
    return out


FF_SPECS = _nminus_heavy_specs()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FF_SPECS))
def test_gpu_nminus_fast_forward_matches_oracle(name, engine_mod, oracle_mod, monkeypatch):
    """The bin stepper's N- fast-forward (birth-death runs) against the oracle, bit for bit,
    on N--dominated runs, under both instruction schedules. (The pure-birth case has no fast-forward.)"""
    spec = FF_SPECS[name]
    cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
    for sched in ("1", "0", "3"):
        monkeypatch.setenv("ECDNA_SSA_SCHED", sched)
        _compare(engine_mod.run(spec, want_rows=True), cpu, f"{name}/sched{sched}")
    # paired lanes: the default here (auto: at most half a wave of replicates per SIMD), and forced
    # onto two workgroups so that every owner lane runs several replicates one after another
    monkeypatch.setenv("ECDNA_SSA_SCHED", "2")
    _compare(engine_mod.run(spec, want_rows=True), cpu, f"{name}/auto")
    monkeypatch.setenv("ECDNA_SSA_PAIR", "1")
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", "2")
    _compare(engine_mod.run(spec, want_rows=True), cpu, f"{name}/pair-refill")
    s = cpu.summaries
    ev = s["events_by_type"].astype(np.int64)
    nminus_share = (ev[:, 0] + ev[:, 2]).sum() / ev.sum()
    assert nminus_share > 0.6, nminus_share  # the fast-forward's regime


@pytest.mark.gpu
@pytest.mark.parametrize("flags,kmax", [(0, 0), (abi.FLAG_BIN_STORE, 32), (abi.FLAG_BIN_STORE, 64)])
def test_gpu_empty_replicates_stop_with_their_error_at_every_limit(flags, kmax, engine_mod, oracle_mod):
    """An empty initial distribution stops with ECDNA_REP_ERR_EMPTY and ECDNA_STOP_ERROR whatever other limit would
    hold at its first stop test (round 6: the bin stepper records the error at the claim and stops the replicate at
    that iteration's stop test, whose reason follows the error), mixed with non-empty sets in one launch; bit for bit
    against the oracle. max_iter 0 and a cell limit of 1 make every other stop condition true at the first test."""
    for max_iter, max_cells in ((0, 100), (50, 1), (50, 100)):
        spec = abi.RunSpec(seed=9, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),) * 2, n_replicates=16,
                           reps_per_set=8, max_cells=max_cells, max_iter=max_iter,
                           init_per_set=[{}, {1: 2, 3: 1}], flags=abi.FLAG_EVENT_HASH | flags, bin_kmax=kmax)
        gpu = engine_mod.run(spec, want_rows=True)
        cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
        _compare(gpu, cpu, f"empty/{flags}/{kmax}/{max_iter}/{max_cells}")
        s = gpu.summaries
        empty = np.arange(16) < 8
        assert (s["error"][empty] == abi.REP_ERR_EMPTY).all() and (s["stop_reason"][empty] == abi.STOP_ERROR).all()
        assert (s["iters"][empty] == 0).all()
        assert (s["error"][~empty] == 0).all()
