"""The reference's unit tests, restated against the oracle's event kernels (CPU only).

The reference pins only count invariants, with quickcheck generators
(src/lib.rs:47-128). hypothesis plays quickcheck's role here; the generators mirror
NonEmptyDistribtionWithNPlusCells (src/lib.rs:58-75: up to 500 distinct even copy numbers in
[2, 254], 1-255 cells each, plus 1-255 N- cells) and DNACopySegregatingGreatherThanOne
(src/lib.rs:76-90: even values in [2, 254], odd values and 1 coerced to 2).
"""
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from ecdna_evo_amd import abi

SEGS = [abi.SEG_DETERMINISTIC, abi.SEG_BINOMIAL, abi.SEG_BINOMIAL_NO_UNEVEN, abi.SEG_BINOMIAL_NO_NMINUS]
FALSE, TRUE, TRUE_NO_NMINUS = 0, 1, 2


@st.composite
def distributions(draw):
    """NonEmptyDistribtionWithNPlusCells (src/lib.rs:58-75)."""
    entries = draw(st.dictionaries(st.integers(1, 127).map(lambda x: 2 * x), st.integers(1, 255),
                                   min_size=1, max_size=500))
    nminus = draw(st.integers(1, 255))
    cells = []
    for k in sorted(entries):
        cells += [k] * entries[k]
    return cells, nminus


def copies_segregating():
    """DNACopySegregatingGreatherThanOne (src/lib.rs:76-90)."""
    return st.integers(1, 255).map(lambda c: 2 if (c == 1 or c % 2 == 1) else c)


seeds = st.integers(0, 2**64 - 1)
rids = st.integers(0, 2**40)
events = st.integers(0, 2**32 - 1)


@settings(max_examples=150, deadline=None)
@given(distributions(), st.sampled_from(SEGS), seeds, rids, events)
def test_increase_nplus(oracle_mod, distr, seg, seed, rid, e):
    """increase_nplus_test (src/proliferation.rs:159-242)."""
    cells, nminus = distr
    d = oracle_mod.Distribution(cells, nminus)
    nplus0, nminus0 = d.nplus, d.nminus
    rc, k1, k2, un = d.increase_nplus(seg, seed, rid, e)
    assert rc == 0
    if seg == abi.SEG_DETERMINISTIC:
        assert un == FALSE and d.nplus == nplus0 + 1 and d.nminus == nminus0
    if seg == abi.SEG_BINOMIAL_NO_UNEVEN:
        assert un == FALSE
    if un == FALSE:
        assert d.nplus == nplus0 + 1 and d.nminus == nminus0
    elif un == TRUE:
        assert d.nplus == nplus0 and d.nminus == nminus0 + 1
    else:
        assert d.nplus == nplus0 and d.nminus == nminus0
    # copies are conserved: the picked cell's k doubled into k1 + k2
    before, after = np.sort(np.asarray(cells, np.int64)), np.sort(d.cells().astype(np.int64))
    assert after.sum() - before.sum() == (k1 + k2) // 2
    assert k1 + k2 == 2 * ((k1 + k2) // 2)


@settings(max_examples=100, deadline=None)
@given(distributions())
def test_increase_nminus(oracle_mod, distr):
    """increase_nminus_test (src/proliferation.rs:244-256)."""
    cells, nminus = distr
    d = oracle_mod.Distribution(cells, nminus)
    d.increase_nminus()
    assert d.nminus == nminus + 1 and d.nplus == len(cells)


@settings(max_examples=100, deadline=None)
@given(distributions(), seeds, rids, events)
def test_decrease_nplus(oracle_mod, distr, seed, rid, e):
    """decrease_nplus_test (src/proliferation.rs:258-272): n+ - 1, n- unchanged; one cell removed."""
    cells, nminus = distr
    d = oracle_mod.Distribution(cells, nminus)
    assert d.decrease_nplus(seed, rid, e) == 0
    assert d.nminus == nminus and d.nplus == len(cells) - 1
    b, a = np.sort(cells), np.sort(d.cells())
    removed = np.setdiff1d(np.unique(b), []).tolist()
    assert len(a) == len(b) - 1 and any(np.array_equal(np.sort(np.delete(b, np.searchsorted(b, k))), a)
                                        for k in removed)


@settings(max_examples=100, deadline=None)
@given(distributions())
def test_decrease_nminus(oracle_mod, distr):
    """decrease_nminus_test (src/proliferation.rs:274-286)."""
    cells, nminus = distr
    d = oracle_mod.Distribution(cells, nminus)
    assert d.decrease_nminus() == 0
    assert d.nminus == nminus - 1 and d.nplus == len(cells)


def test_try_from_dna_copy_rejects_0_1_3(oracle_mod):
    """try_from_dna_copy_{0,1,3}_test (src/segregation.rs:223-239; the '3' test there really checks 1)."""
    for n in (0, 1, 3, 5, 65535):
        assert oracle_mod.segregate(abi.SEG_BINOMIAL, n, 1, 2, 3)[0] == -1


@settings(max_examples=200, deadline=None)
@given(copies_segregating(), seeds, rids, events)
def test_segregate_deterministic(oracle_mod, n, seed, rid, e):
    """segregate_deterministic_test (src/segregation.rs:248-260)."""
    rc, k1, k2, un = oracle_mod.segregate(abi.SEG_DETERMINISTIC, n, seed, rid, e)
    assert rc == 0 and k1 == k2 and 2 * k1 == n and un == FALSE


@settings(max_examples=300, deadline=None)
@given(copies_segregating(), seeds, rids, events)
def test_segregate_random_binomial(oracle_mod, n, seed, rid, e):
    """segregate_random_binomial_test (src/segregation.rs:262-278)."""
    rc, k1, k2, un = oracle_mod.segregate(abi.SEG_BINOMIAL, n, seed, rid, e)
    assert rc == 0 and k1 + k2 == n
    assert (un != FALSE) == (k1 == 0 or k2 == 0)


@settings(max_examples=300, deadline=None)
@given(copies_segregating(), seeds, rids, events)
def test_segregate_no_uneven(oracle_mod, n, seed, rid, e):
    """segregate_random_binomial_no_nminus_test (src/segregation.rs:280-291; tests BinomialNoUneven)."""
    rc, k1, k2, un = oracle_mod.segregate(abi.SEG_BINOMIAL_NO_UNEVEN, n, seed, rid, e)
    assert rc == 0 and k1 + k2 == n and un == FALSE and k1 > 0 and k2 > 0


@settings(max_examples=200, deadline=None)
@given(copies_segregating(), seeds, rids, events)
def test_segregate_no_nminus_relabels(oracle_mod, n, seed, rid, e):
    """BinomialNoNminus (src/segregation.rs:176-194): same draw as Binomial, uneven relabelled."""
    a = oracle_mod.segregate(abi.SEG_BINOMIAL, n, seed, rid, e)
    b = oracle_mod.segregate(abi.SEG_BINOMIAL_NO_NMINUS, n, seed, rid, e)
    assert a[1:3] == b[1:3]
    assert b[3] == (TRUE_NO_NMINUS if a[3] == TRUE else FALSE)


@settings(max_examples=60, deadline=None)
@given(distributions(), st.integers(0, 25).map(lambda t: t / 10.0))
def test_create_process_preserves_state(oracle_mod, distr, _time):
    """create_birth_death_process_test (src/process.rs:356-384): a process that takes no step keeps
    n+, n-, time and mean. Here: max_cells <= initial cells, so the run stops before any event."""
    cells, nminus = distr
    hist = {0: nminus}
    for k in cells:
        hist[k] = hist.get(k, 0) + 1
    spec = abi.RunSpec(process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.5, 0.5),), n_replicates=1,
                       max_cells=len(cells) + nminus, init=hist, flags=abi.FLAG_EVENT_HASH)
    r = oracle_mod.run(spec, want_rows=True)
    s = r.summaries[0]
    assert s["iters"] == 0 and s["nplus"] == len(cells) and s["nminus"] == nminus and s["time"] == 0.0
    assert s["stop_reason"] == abi.STOP_MAX_CELLS
    assert np.array_equal(r.row(0), np.asarray(sorted(cells), np.uint16))


def test_nplus_events_on_an_empty_nplus_set_return_the_internal_error(oracle_mod):
    """pick_remove_random_nplus errors on an empty N+ set (src/proliferation.rs:55-57). The oracle's event kernels
    return ECDNA_REP_ERR_INTERNAL there, the code the engine's guard stops such a replicate with (ABI v11), and leave
    the distribution unchanged."""
    d = oracle_mod.Distribution([], 5)
    rc, _, _, _ = d.increase_nplus(abi.SEG_BINOMIAL, 42, 0, 0)
    assert rc == abi.REP_ERR_INTERNAL == 5
    assert d.decrease_nplus(42, 0, 0) == abi.REP_ERR_INTERNAL
    assert d.nplus == 0 and d.nminus == 5
