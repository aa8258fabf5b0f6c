"""Fused per-replicate ABC statistics (abc.md:38-55) on the GPU against the numpy
restatement (oracle/abc_stats.py) applied to the oracle's final rows. Floating-point tolerance: 1e-12
relative (sums are reduced in a different order on the GPU; log is ocml's vs numpy's)."""
import numpy as np
import pytest

from ecdna_evo_amd import abi

RTOL, ATOL = 1e-12, 1e-14


def _target(bins):
    rng = np.random.default_rng(5)
    t = np.zeros(bins, np.uint64)
    t[0] = 400
    t[1:40] = rng.integers(0, 90, 39)
    t[bins - 1] = 3
    return t


@pytest.mark.gpu
@pytest.mark.parametrize("store,kmax", [("rows", 0), ("bins", 32), ("bins", 64), ("bins", 256)])
@pytest.mark.parametrize("with_target", [False, True])
def test_rep_stats_match_restatement(engine_mod, oracle_mod, with_target, store, kmax):
    """Both cell stores (the bin store's statistics read its counters and its large-k row: the initial
    300-copy cell lies above every K)."""
    import abc_stats

    bins = 257
    tgt = _target(bins) if with_target else None
    flags = abi.FLAG_REP_STATS | abi.FLAG_EVENT_HASH | (abi.FLAG_BIN_STORE if store == "bins" else 0)
    spec = abi.RunSpec(seed=4, process=abi.BIRTH_DEATH, rates=((1.0, 1.4, 0.3, 0.3), (1.0, 2.0, 0.5, 0.2)),
                       reps_per_set=300, n_replicates=600, max_cells=2000, hist_bins=bins, init={1: 3, 300: 1},
                       stats_target=tgt, flags=flags, bin_kmax=kmax)
    g = engine_mod.run(spec)
    c = oracle_mod.run(spec, want_rows=True)
    np.testing.assert_array_equal(g.summaries["event_hash"], c.summaries["event_hash"])
    np.testing.assert_array_equal(g.hist, c.hist)
    for i in range(spec.n_replicates):
        want = abc_stats.rep_stats(c.summaries[i]["nminus"], c.row(i), bins, tgt)
        got = g.stats[i]
        assert int(got["cells"]) == want["cells"]
        for f in ("mean", "entropy", "frequency", "ks", "mean_rel", "entropy_rel", "frequency_diff"):
            np.testing.assert_allclose(got[f], want[f], rtol=RTOL, atol=ATOL, err_msg=f"replicate {i}: {f}")


@pytest.mark.gpu
def test_rep_stats_do_not_change_histogram(engine_mod):
    spec = dict(seed=9, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=4096, max_cells=1000,
                hist_bins=1025)
    a = engine_mod.run(abi.RunSpec(**spec, flags=0))
    b = engine_mod.run(abi.RunSpec(**spec, flags=abi.FLAG_REP_STATS, stats_target=_target(1025)))
    np.testing.assert_array_equal(a.hist, b.hist)
    for f in a.totals.dtype.names:
        np.testing.assert_array_equal(a.totals[f], b.totals[f])
    ext = a.summaries["nminus"] + a.summaries["nplus"] == 0
    assert np.all(b.stats["ks"][ext] == 1.0) and np.all(b.stats["cells"][~ext] > 0)
