"""GPU tests at BASELINE.json's full sizes, through size-independent properties, plus the
reference-semantics KS comparison (BASELINE.json north_star: KS < 0.01).
"""
import os

import numpy as np
import pytest

from ecdna_evo_amd import abi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KS_TOL = 0.01  # north_star: KS distance < 0.01 on the final copy-number histogram
# both cell stores: rows (u16 per cell, swap_remove order) and bins (copy-number counters in LDS)
STORES = {"rows": 0, "bins": abi.FLAG_BIN_STORE}


def _ks(h1, h2):
    c1 = np.cumsum(h1.astype(np.float64)) / h1.sum()
    c2 = np.cumsum(h2.astype(np.float64)) / h2.sum()
    return float(np.abs(c1 - c2).max())


def c2_spec(**kw):
    d = dict(seed=42, n_replicates=65536, max_cells=10_000, hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


def c3_spec(first=0, n=1 << 20, **kw):
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), reps_per_set=1 << 20,
             first_replicate=first, n_replicates=n, max_cells=10_000, hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


def _invariants(res, spec):
    s, h, t = res.summaries, res.hist, res.totals
    assert h[:, 0].sum() == s["nminus"].sum()
    assert h[:, 1:].sum() == s["nplus"].sum()
    assert np.all(s["iters"] == s["events_by_type"].sum(axis=1))
    assert int(t["events"].sum()) == int(s["iters"].sum())
    assert int(t["replicates"].sum()) == len(s)
    assert np.all(s["error"] == 0)
    assert np.all(np.bincount(s["stop_reason"], minlength=6) == t["stop_reasons"].sum(axis=0))


def _balance(res, init_nplus, init_nminus=0):
    """Population bookkeeping per replicate under Binomial segregation (src/proliferation.rs:81-117,
    125-140): every ProliferateNMinus adds an N- cell, every uneven split (IsUneven::True) turns one
    N+ cell into an N+ and an N- cell, every even split adds one N+ cell, deaths remove one."""
    s = res.summaries
    ev = s["events_by_type"].astype(np.int64)
    un = s["uneven"].astype(np.int64)
    np.testing.assert_array_equal(s["nminus"].astype(np.int64), init_nminus + ev[:, 0] - ev[:, 2] + un)
    np.testing.assert_array_equal(s["nplus"].astype(np.int64), init_nplus + ev[:, 1] - un - ev[:, 3])


def c4_shard_spec(rank=0, gpus=8, **kw):
    """C4 (BASELINE.json configs[3]): 1024 (b1, d, k0) parameter sets x 4096 replicates over 8 GPUs;
    this is rank `rank`'s shard of 128 whole sets."""
    rates, inits = [], []
    for i in range(1024):
        sel = 1.0 + 1.5 * (i % 16) / 15.0
        d = 0.7 * ((i // 16) % 8) / 7.0
        rates.append((1.0, sel, d, d))
        inits.append({1 << (i // 128): 1})
    n = 1024 * 4096 // gpus
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=rates, reps_per_set=4096, first_replicate=rank * n,
             n_replicates=n, max_cells=10_000, init_per_set=inits, hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


def c5_shard_spec(rank=0, gpus=8, **kw):
    """C5 (BASELINE.json configs[4]): 262,144 turnover replicates from 1,000 cells to 1e6 cells or
    t = 1000 over 8 GPUs; this is rank `rank`'s shard of 32,768 replicates."""
    n = 262_144 // gpus
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), reps_per_set=262_144,
             first_replicate=rank * n, n_replicates=n, max_cells=1_000_000, max_time=1000.0, init={1: 1000},
             hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c2_ks_against_reference_semantics(engine_mod, store):
    """C2 shape (65,536 replicates, pure birth + binomial to 1e4 cells, seed 42) on the GPU vs the
    committed reference-semantics fixture (ChaCha8 + first-reaction + BTPE, tests/golden/)."""
    g = np.load(os.path.join(GOLDEN, "c2_compat_seed42.npz"))
    r = engine_mod.run(c2_spec(flags=STORES[store]))
    _invariants(r, c2_spec())
    _balance(r, 1)
    ks = _ks(r.hist[0], g["hist"])
    assert ks < KS_TOL, ks
    # per-replicate law of the N- fraction (two-sample KS on replicates, not cells)
    from scipy import stats

    fa = r.summaries["nminus"] / (r.summaries["nminus"] + r.summaries["nplus"])
    fb = g["nminus"] / (g["nminus"] + g["nplus"]).astype(np.float64)
    assert stats.ks_2samp(fa, fb).pvalue > 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c2_pure_birth_exact_event_counts(engine_mod, store):
    r = engine_mod.run(c2_spec(flags=STORES[store]))
    s = r.summaries
    full = s["stop_reason"] == abi.STOP_MAX_CELLS
    assert full.mean() > 0.99
    assert np.all(s["iters"][full] == 10_000 - 1)
    assert np.all(s["stop_reason"][~full] == abi.STOP_MAX_TIME)


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c3_full_size_properties_and_shard_identity(engine_mod, store):
    """C3 at 2^20 replicates: invariants, and the two halves run as separate shards (global ids)
    reproduce the full run's summaries and histogram bit for bit (the 1-GPU == N-GPU identity)."""
    fl = STORES[store]
    full = engine_mod.run(c3_spec(flags=fl))
    _invariants(full, c3_spec())
    _balance(full, 1)
    half = 1 << 19
    a = engine_mod.run(c3_spec(0, half, flags=fl))
    b = engine_mod.run(c3_spec(half, half, flags=fl))
    for f in full.summaries.dtype.names:
        np.testing.assert_array_equal(np.concatenate([a.summaries[f], b.summaries[f]]), full.summaries[f])
    np.testing.assert_array_equal(a.hist + b.hist, full.hist)
    # extinction probability of a birth-death process from one N+ cell ~ d1/b1 = 0.2 (k=1 start
    # loses its ecDNA only by uneven division, whose N- daughters then die out with prob d0/b0)
    ext = np.mean(full.summaries["stop_reason"] == abi.STOP_ABSORBING)
    assert 0.15 < ext < 0.35


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c3_matches_oracle_on_a_sample(engine_mod, oracle_mod, store):
    """Replicates 0..4095 of the C3 run, checked against the oracle bit for bit (hash on)."""
    spec = c3_spec(0, 4096, flags=abi.FLAG_EVENT_HASH | STORES[store])
    g = engine_mod.run(spec)
    c = oracle_mod.run(spec, mode="philox")
    for f in g.summaries.dtype.names:
        np.testing.assert_array_equal(g.summaries[f], c.summaries[f], err_msg=f)
    np.testing.assert_array_equal(g.hist, c.hist)


@pytest.mark.gpu
def test_engine_reproduces_parity_fixture(engine_mod):
    """The GPU reproduces the committed oracle fixtures without running the oracle."""
    import make_golden
    from cases import bin_cases, cases

    fx = np.load(os.path.join(GOLDEN, "parity_cases.npz"))
    for name, spec in sorted({**cases(), **bin_cases()}.items()):
        r = engine_mod.run(spec, want_rows=True)
        want = fx[f"{name}__summaries"]
        for f in want.dtype.names:
            np.testing.assert_array_equal(r.summaries[f], want[f], err_msg=f"{name}: {f}")
        np.testing.assert_array_equal(r.hist, fx[f"{name}__hist"], err_msg=name)
        assert make_golden.rows_digest(r) == str(fx[f"{name}__rows_sha256"]), name
        if f"{name}__snapshots" in fx:
            np.testing.assert_array_equal(r.snapshots, fx[f"{name}__snapshots"], err_msg=name)
            assert make_golden.snapshot_digest(r) == str(fx[f"{name}__snapshot_rows_sha256"]), name


@pytest.mark.gpu
def test_abc_sweep_shape_small(engine_mod, oracle_mod):
    """C4 shape scaled down: 64 parameter sets x 32 replicates, per-set rates; every set's histogram
    matches the oracle, and each set's totals count its own replicates only."""
    rates, inits = [], []
    for i in range(64):
        s = 1.0 + 1.5 * (i % 16) / 15
        d = 0.7 * (i // 16) / 3
        rates.append((1.0, s, d, d))
        inits.append({1 << (i % 4): 1})
    spec = abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=rates, reps_per_set=32, n_replicates=64 * 32,
                       max_cells=1000, hist_bins=513, init_per_set=inits, flags=abi.FLAG_EVENT_HASH)
    g = engine_mod.run(spec)
    c = oracle_mod.run(spec)
    np.testing.assert_array_equal(g.hist, c.hist)
    np.testing.assert_array_equal(g.summaries["event_hash"], c.summaries["event_hash"])
    assert np.all(g.totals["replicates"] == 32)


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c4_shard_full_size_properties(engine_mod, oracle_mod, store):
    """C4 rank-0 shard at full size (524,288 replicates, 128 parameter sets with per-set rates and
    initial copy numbers): invariants, bookkeeping, per-set replicate counts, and 256 replicates of a
    birth-death set with initial k = 1 against the oracle bit for bit (event hash)."""
    spec = c4_shard_spec(flags=abi.FLAG_EVENT_HASH | STORES[store])
    r = engine_mod.run(spec)
    _invariants(r, spec)
    _balance(r, 1)
    assert np.all(r.totals["replicates"][:128] == 4096) and np.all(r.totals["replicates"][128:] == 0)
    first = 37 * 4096  # set 37: b1 = 1.2, d = 0.2, k0 = 1
    c = oracle_mod.run(c4_shard_spec(first_replicate=first, n_replicates=256,
                                     flags=abi.FLAG_EVENT_HASH | STORES[store]), mode="philox")
    for f in c.summaries.dtype.names:
        np.testing.assert_array_equal(r.summaries[f][first:first + 256], c.summaries[f], err_msg=f)


@pytest.mark.gpu
def test_c4_interleaved_shard_full_size(engine_mod, oracle_mod):
    """C4 rank-3 shard of 8, interleaved (global ids 3, 11, 19, ...; the layout that balances the ABC
    grid across GPUs): every one of the 1024 sets gets 512 replicates, invariants hold,
    and 64 replicates of set 1000 (initial k = 128: 256-bit binomials through the block-wise popcount,
    cells beyond the LDS bins) match the oracle bit for bit."""
    from ecdna_evo_amd import shard

    first, n, stride = shard.interleaved_range(3, 8, 1024 * 4096)
    spec = c4_shard_spec(first_replicate=first, n_replicates=n, replicate_stride=stride,
                         flags=abi.FLAG_EVENT_HASH | abi.FLAG_BIN_STORE, bin_kmax=32)
    r = engine_mod.run(spec)
    _invariants(r, spec)
    assert np.all(r.totals["replicates"] == 512)
    m0 = (1000 * 4096 - first + stride - 1) // stride  # first local replicate in set 1000
    sub = c4_shard_spec(first_replicate=first + m0 * stride, n_replicates=64, replicate_stride=stride,
                        flags=abi.FLAG_EVENT_HASH | abi.FLAG_BIN_STORE, bin_kmax=32)
    assert (sub.first_replicate // 4096) == 1000
    c = oracle_mod.run(sub, mode="philox", n_threads=4)
    for f in c.summaries.dtype.names:
        np.testing.assert_array_equal(r.summaries[f][m0:m0 + 64], c.summaries[f], err_msg=f)


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(STORES))
def test_c5_shard_full_size_properties(engine_mod, oracle_mod, store):
    """C5 rank-0 shard at full size (32,768 replicates, rows up to 1e6 cells = 2 MB, 65 GB of rows):
    invariants, bookkeeping, the stop law of a critical-ish turnover process, and replicates 0..3
    (about 2e7 events each) against the oracle bit for bit (event hash). The bin store runs its
    256-bin, u32-counter variant here (cell_cap 1e6 > 65535) with a large-k row of 2^14 cells."""
    kw = dict(flags=abi.FLAG_EVENT_HASH | STORES[store], bin_kmax=256 if store == "bins" else 0,
              big_cap=(1 << 14) if store == "bins" else 0)  # bins: a bounded large-k row (k > 256 is rare)
    spec = c5_shard_spec(**kw)
    r = engine_mod.run(spec)
    _invariants(r, spec)
    _balance(r, 1000)
    stops = set(r.summaries["stop_reason"].tolist())
    assert stops <= {abi.STOP_MAX_CELLS, abi.STOP_MAX_TIME, abi.STOP_ABSORBING}, stops  # (no row-capacity errors)
    c = oracle_mod.run(c5_shard_spec(n_replicates=4, **kw), mode="philox", n_threads=4)
    for f in c.summaries.dtype.names:
        np.testing.assert_array_equal(r.summaries[f][:4], c.summaries[f], err_msg=f)


@pytest.mark.gpu
def test_c3_bin_store_and_row_store_agree_in_law(engine_mod):
    """The two cell stores simulate the same process (a uniform cell pick is invariant under the
    arrangement of the cells): at C3 size their pooled copy-number histograms are
    within the north-star KS tolerance and per-replicate laws (final size, N- fraction, events) agree."""
    from scipy import stats

    a = engine_mod.run(c3_spec(n=1 << 18))
    b = engine_mod.run(c3_spec(n=1 << 18, flags=abi.FLAG_BIN_STORE, seed=4242))
    assert _ks(a.hist[0], b.hist[0]) < KS_TOL
    for f in ("iters", "nplus", "nminus"):
        assert stats.ks_2samp(a.summaries[f], b.summaries[f]).pvalue > 1e-4, f
    ma = (np.arange(1025) * a.hist[0]).sum() / a.hist[0].sum()
    mb = (np.arange(1025) * b.hist[0]).sum() / b.hist[0].sum()
    assert abs(ma - mb) / ma < 0.01


# ---- the north star's KS clause on the birth-death configurations (BASELINE.json configs[2..4]): the engine's
# philox mapping, in the bench's own settings, against committed reference-semantics fixtures (ChaCha8 +
# first-reaction + rand_distr samplers + f32 time: tests/golden/make_golden.py, oracle compat mode), and the
# engine's reference-draws mode against the same fixtures seed for seed.


def _fixture(name):
    return np.load(os.path.join(GOLDEN, f"{name}_compat_seed42.npz"))


def _per_replicate_laws(s, g, p_min):
    """Two-sample KS on per-replicate statistics (replicates are independent; cells within one are not): final
    N- and N+ counts, events, and the N- fraction of the surviving replicates."""
    from scipy import stats

    for f in ("nminus", "nplus", "iters"):
        p = stats.ks_2samp(s[f].astype(np.float64), g[f].astype(np.float64)).pvalue
        assert p > p_min, (f, p)
    ca, cb = s["nminus"] + s["nplus"], g["nminus"].astype(np.int64) + g["nplus"]
    fa = s["nminus"][ca > 0] / ca[ca > 0]
    fb = g["nminus"][cb > 0] / cb[cb > 0]
    assert stats.ks_2samp(fa, fb).pvalue > p_min


def _ks_crit(n, m, alpha):
    """Two-sample KS critical value (asymptotic) at level alpha for sample sizes n, m."""
    return float(np.sqrt(-0.5 * np.log(alpha / 2.0)) * np.sqrt((n + m) / (n * m)))


BENCH_STORES = {"bins": dict(flags=abi.FLAG_BIN_STORE), "rows": dict(flags=0)}


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(BENCH_STORES))
def test_c3_ks_against_reference_semantics(engine_mod, store):
    """C3 (2^20 replicates, the metric's configuration, bench settings: f64 time, bin store K = 32 or the row
    store) against the reference-semantics C3 fixture (65,536 replicates): pooled copy-number histogram KS
    < 0.01 (CPU null with a second philox seed: 5e-5) and per-replicate laws."""
    import make_golden

    g = _fixture("c3")
    kw = dict(BENCH_STORES[store], bin_kmax=32 if store == "bins" else 0)
    r = engine_mod.run(make_golden.c3_spec(n=1 << 20, **kw))
    _invariants(r, make_golden.c3_spec())
    ks = _ks(r.hist[0], g["hist"][0])
    assert ks < KS_TOL, ks
    _per_replicate_laws(r.summaries, g, 1e-4)
    ext_a = np.mean(r.summaries["stop_reason"] == abi.STOP_ABSORBING)
    ext_b = np.mean(g["stop_reason"] == abi.STOP_ABSORBING)
    assert abs(ext_a - ext_b) < 5 * np.sqrt(ext_b * (1 - ext_b) / len(g["stop_reason"]))


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(BENCH_STORES))
def test_c4_subset_ks_against_reference_semantics(engine_mod, store):
    """16 sets of the C4 ABC sweep spanning s in [1, 2.5], d in [0, 0.7] and k0 in {1, 16, 128} (bench settings:
    bin store K = 64), 65,536 replicates per set against the fixture's 16,384. ABC rejection is per parameter set
    (abc.md:38-55), so EACH set is held to the north star's KS < 0.01 on its own pooled copy-number histogram (the
    old 4,096-replicate fixture only allowed the alpha = 1e-4 critical value per set, 0.039), plus per-replicate
    laws per set and the pooled KS over all sets."""
    import make_golden

    g = _fixture("c4_subset")
    m = make_golden.C4_REPS
    n = 65536
    kw = dict(BENCH_STORES[store], bin_kmax=64 if store == "bins" else 0)
    r = engine_mod.run(make_golden.c4_subset_spec(reps_per_set=n, **kw))
    assert np.all(r.summaries["error"] == 0)
    gh = g["hist"].reshape(16, -1)
    assert _ks(r.hist.sum(axis=0), gh.sum(axis=0)) < KS_TOL
    worst = 0.0
    for i in range(16):
        ks = _ks(r.hist[i], gh[i])
        worst = max(worst, ks)
        assert ks < KS_TOL, (i, make_golden.C4_SETS[i], ks)
        sa = r.summaries[i * n:(i + 1) * n]
        sb = {f: g[f][i * m:(i + 1) * m] for f in ("nminus", "nplus", "iters")}
        _per_replicate_laws(sa, sb, 1e-5)
    print(f"C4 subset ({store}): worst per-set KS {worst:.5f}")


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(BENCH_STORES))
def test_c3_halved_cap_ks_against_reference_semantics(engine_mod, store):
    """The other plausible reading of sosa's cell cap: the reference's BirthDeath
    duplicates its population vector [n-, n+, n-, n+] (src/process.rs:339-344), so a cap tested against its sum
    stops at n- + n+ >= max_cells / 2. Under ECDNA_FLAG_BD_CAP_COMPAT the engine (bench settings otherwise: C3 at
    2^20 replicates, f64 time) matches the reference-semantics fixture made under the same reading: pooled KS
    < 0.01 and per-replicate laws."""
    import make_golden

    g = _fixture("c3cap")
    kw = dict(BENCH_STORES[store], bin_kmax=32 if store == "bins" else 0)
    kw["flags"] |= abi.FLAG_BD_CAP_COMPAT
    r = engine_mod.run(make_golden.c3_spec(n=1 << 20, **kw))
    _invariants(r, make_golden.c3_spec())
    full = r.summaries["stop_reason"] == abi.STOP_MAX_CELLS
    assert np.all((r.summaries["nminus"] + r.summaries["nplus"])[full] == 5_000)
    assert _ks(r.hist[0], g["hist"][0]) < KS_TOL
    _per_replicate_laws(r.summaries, g, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("store", sorted(BENCH_STORES))
def test_c5_shaped_ks_against_reference_semantics(engine_mod, store):
    """C5's turnover process (b = 1, d = 0.9, {1: 1000}) to 2e4 cells with f32 time like the reference's
    process.time (bench settings otherwise: bin store K = 64), 32,768 replicates against the fixture's 4,096:
    pooled KS < 0.01 (CPU null 2e-4) and per-replicate laws."""
    import make_golden

    g = _fixture("c5_shaped")
    kw = dict(flags=BENCH_STORES[store]["flags"] | abi.FLAG_TIME_F32, bin_kmax=64 if store == "bins" else 0)
    r = engine_mod.run(make_golden.c5_shaped_spec(n=32768, **kw))
    assert np.all(r.summaries["error"] == 0)
    assert _ks(r.hist[0], g["hist"][0]) < KS_TOL
    _per_replicate_laws(r.summaries, g, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["c3", "c4_subset", "c5_shaped", "c3cap"])
def test_reference_draws_reproduce_bd_fixtures_seed_for_seed(engine_mod, name):
    """ECDNA_FLAG_REFERENCE_DRAWS (the Rust reference's draw structure) on the fixtures' exact configurations
    and replicate ids: every replicate's final n-, n+, events and stop reason, and the pooled histograms,
    equal the reference-semantics CPU run's (the fixture) — seed for seed, not just in law."""
    import make_golden

    spec = {"c3": make_golden.c3_spec, "c4_subset": make_golden.c4_subset_spec,
            "c5_shaped": make_golden.c5_shaped_spec,
            "c3cap": lambda **kw: make_golden.c3_spec(**{**kw, "flags": kw["flags"] | abi.FLAG_BD_CAP_COMPAT})}[name](
        flags=abi.FLAG_REFERENCE_DRAWS)
    g = _fixture(name)
    r = engine_mod.run(spec)
    np.testing.assert_array_equal(r.hist.reshape(-1), g["hist"].reshape(-1))
    for f in ("nminus", "nplus", "iters", "stop_reason"):
        np.testing.assert_array_equal(r.summaries[f].astype(np.int64), g[f].astype(np.int64), err_msg=f)
