"""Analytic known answers for the hot path (CPU oracle, both draw mappings) — SURVEY.md §8c (iii).

The reference has no golden vectors, so these pin the oracle's semantics to mathematics:
  * pure birth adds exactly one cell per event under Binomial/Deterministic/NoUneven
    (src/proliferation.rs:81-100, 113-117), so a run to max_cells takes max_cells - N0 events;
  * Deterministic segregation keeps every N+ cell at its initial copy number;
  * NoUneven never creates an N- cell;
  * with b0 = b1 = b the total population is a Yule process: P(T_N <= t) = (1 - e^{-bt})^{N-1}
    from one cell;
  * the first division of {k=1} yields an N- cell with probability exactly 1/2 (Binomial);
  * k1 ~ Binomial(2k, 1/2);
  * the philox mapping and the reference-semantics mapping (ChaCha8 + first-reaction + BTPE)
    give the same law of the final state.
"""
import numpy as np
import pytest
from scipy import stats

from ecdna_evo_amd import abi

MODES = ["philox", "compat"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seg", [abi.SEG_BINOMIAL, abi.SEG_DETERMINISTIC, abi.SEG_BINOMIAL_NO_UNEVEN])
def test_pure_birth_event_count_is_exact(oracle_mod, mode, seg):
    spec = abi.RunSpec(seed=5, segregation=seg, n_replicates=64, max_cells=700, init={1: 2, 3: 1}, flags=0)
    s = oracle_mod.run(spec, mode=mode).summaries
    ok = s["stop_reason"] == abi.STOP_MAX_CELLS
    assert ok.mean() > 0.95
    assert np.all(s["iters"][ok] == 700 - 3)
    assert np.all(s["nminus"][ok] + s["nplus"][ok] == 700)


@pytest.mark.parametrize("mode", MODES)
def test_deterministic_keeps_copy_numbers(oracle_mod, mode):
    spec = abi.RunSpec(seed=9, segregation=abi.SEG_DETERMINISTIC, n_replicates=16, max_cells=500,
                       init={3: 1, 7: 2}, hist_bins=16, flags=0)
    r = oracle_mod.run(spec, mode=mode)
    assert r.hist[0, 0] == 0  # n- never grows from 0
    assert set(np.nonzero(r.hist[0])[0].tolist()) <= {3, 7}


@pytest.mark.parametrize("mode", MODES)
def test_no_uneven_never_creates_nminus(oracle_mod, mode):
    spec = abi.RunSpec(seed=12, process=abi.BIRTH_DEATH, rates=((1.0, 1.3, 0.2, 0.2),),
                       segregation=abi.SEG_BINOMIAL_NO_UNEVEN, n_replicates=64, max_cells=400, flags=0)
    s = oracle_mod.run(spec, mode=mode).summaries
    assert np.all(s["nminus"] == 0) and np.all(s["uneven"] == 0)


@pytest.mark.parametrize("mode", MODES)
def test_yule_hitting_time_law(oracle_mod, mode):
    """b0 = b1 = 1, from one cell to N = 64: P(T <= t) = (1 - e^-t)^(N-1). KS test."""
    N = 64
    spec = abi.RunSpec(seed=77, segregation=abi.SEG_BINOMIAL, n_replicates=6000, max_cells=N, max_time=1e9,
                       flags=0)
    t = oracle_mod.run(spec, mode=mode).summaries["time"]
    cdf = lambda x: (1.0 - np.exp(-x)) ** (N - 1)  # noqa: E731
    assert stats.kstest(t, cdf).pvalue > 1e-3
    # mean = H_{N-1}
    assert abs(t.mean() - np.sum(1.0 / np.arange(1, N))) < 4 * np.sqrt(np.sum(1.0 / np.arange(1, N) ** 2) / len(t))


@pytest.mark.parametrize("mode", MODES)
def test_first_division_of_k1_is_uneven_half_the_time(oracle_mod, mode):
    spec = abi.RunSpec(seed=3, n_replicates=20000, max_cells=2, flags=0)
    s = oracle_mod.run(spec, mode=mode).summaries
    assert np.all(s["iters"] == 1)
    x = int(s["nminus"].sum())
    assert stats.binomtest(x, len(s), 0.5).pvalue > 1e-3


@pytest.mark.parametrize("k", [1, 3, 16, 17, 40, 300])
def test_segregation_law_chi2(oracle_mod, k):
    """k1 of the philox mapping ~ Binomial(2k, 1/2) (popcount of 2k fair bits; multi-block for 2k > 32)."""
    n = 2 * k
    x = np.array([oracle_mod.segregate(abi.SEG_BINOMIAL, n, 99, rid, e)[1]
                  for rid in range(40) for e in range(500)])
    lo, hi = max(0, int(k - 4 * np.sqrt(n) / 2)), min(n, int(k + 4 * np.sqrt(n) / 2))
    obs = np.bincount(np.clip(x, lo, hi) - lo, minlength=hi - lo + 1)
    pmf = stats.binom.pmf(np.arange(lo, hi + 1), n, 0.5)
    pmf[0] += stats.binom.cdf(lo - 1, n, 0.5)
    pmf[-1] += stats.binom.sf(hi, n, 0.5)
    exp = pmf * len(x)
    keep = exp > 5
    chi = ((obs[keep] - exp[keep]) ** 2 / exp[keep]).sum()
    assert stats.chi2.sf(chi, keep.sum() - 1) > 1e-4


@pytest.mark.parametrize("mode", MODES)
def test_snapshot_rule_pops_front_on_any_match(oracle_mod, mode):
    """src/process.rs:122-145: while ANY remaining snapshot equals n- + n+, pop the FRONT one and save.
    From 50 initial cells with snapshots [1, 40, 51, ...], 1 and 40 are never reached but are popped
    (and saved) together with 51; the last snapshot (= max_cells) is never saved by advance_step
    because the run stops first."""
    spec = abi.RunSpec(seed=8, n_replicates=32, max_cells=300, init={1: 50}, snapshots=[1, 40, 51, 60, 200, 300],
                       flags=abi.FLAG_SNAPSHOT_ROWS)
    r = oracle_mod.run(spec, mode=mode, want_rows=True)
    m = r.snapshots
    assert np.all(m["taken"][:, :5] == 1) and np.all(m["taken"][:, 5] == 0)
    tot = m["nminus"] + m["nplus"]
    assert np.all(tot[:, :3] == 51) and np.all(tot[:, 3] == 60) and np.all(tot[:, 4] == 200)
    assert np.all(m["time"][:, 0] == m["time"][:, 2]) and np.all(m["time"][:, 2] < m["time"][:, 3])
    for i in range(4):
        assert np.array_equal(r.snapshot_row(i, 0), r.snapshot_row(i, 2))
        assert len(r.snapshot_row(i, 4)) == m["nplus"][i, 4]


def test_default_snapshots_match_clap_app():
    """build_snapshots_from_cells(11, cells) (src/clap_app.rs:121-134)."""
    assert abi.default_snapshots(1000) == [1, 101, 201, 301, 401, 501, 601, 701, 801, 901, 1000]
    assert abi.default_snapshots(10) == [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 10]


def _ks_pooled(h1, h2):
    c1, c2 = np.cumsum(h1) / h1.sum(), np.cumsum(h2) / h2.sum()
    return float(np.abs(c1 - c2).max())


def test_philox_and_reference_semantics_agree_in_law(oracle_mod):
    """The engine's draw mapping vs the reference's samplers on a birth-death run (C3 rates, 300 cells, 40,000
    replicates per side): per-replicate statistics (two-sample KS) and the pooled copy-number histogram within
    the north star's KS tolerance, 0.01 (measured: 0.0012; two philox seeds: 0.0005)."""
    base = dict(process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=40_000, max_cells=300,
                hist_bins=257, flags=0)
    a = oracle_mod.run(abi.RunSpec(seed=1, **base), mode="philox")
    b = oracle_mod.run(abi.RunSpec(seed=2, **base), mode="compat")
    sa, sb = a.summaries, b.summaries
    for f in ("nminus", "nplus", "iters", "uneven"):
        assert stats.ks_2samp(sa[f], sb[f]).pvalue > 1e-3, f
    ext_a = np.mean(sa["stop_reason"] == abi.STOP_ABSORBING)
    ext_b = np.mean(sb["stop_reason"] == abi.STOP_ABSORBING)
    assert abs(ext_a - ext_b) < 0.015
    assert _ks_pooled(a.hist[0].astype(float), b.hist[0].astype(float)) < 0.01
