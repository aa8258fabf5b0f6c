"""The oracle reproduces its committed fixtures (tests/golden/, made by tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from cases import bin_cases, cases

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = {**cases(), **bin_cases()}


@pytest.fixture(scope="module")
def parity():
    return np.load(os.path.join(GOLDEN, "parity_cases.npz"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_parity_fixture(oracle_mod, parity, name):
    import make_golden  # noqa: F401  (tests/golden is on sys.path via conftest)

    r = oracle_mod.run(CASES[name], mode="philox", want_rows=True)
    want = parity[f"{name}__summaries"]
    for f in want.dtype.names:
        np.testing.assert_array_equal(r.summaries[f], want[f], err_msg=f"{name}: {f}")
    np.testing.assert_array_equal(r.hist, parity[f"{name}__hist"])
    assert make_golden.rows_digest(r) == str(parity[f"{name}__rows_sha256"])
    if f"{name}__snapshots" in parity:
        np.testing.assert_array_equal(r.snapshots, parity[f"{name}__snapshots"])
        assert make_golden.snapshot_digest(r) == str(parity[f"{name}__snapshot_rows_sha256"])


def test_oracle_reproduces_c2_compat_fixture(oracle_mod):
    import make_golden

    g = np.load(os.path.join(GOLDEN, "c2_compat_seed42.npz"))
    r = oracle_mod.run(make_golden.c2_spec(), mode="compat")
    np.testing.assert_array_equal(r.hist[0], g["hist"])
    np.testing.assert_array_equal(r.summaries["nminus"], g["nminus"])
    np.testing.assert_array_equal(r.summaries["nplus"], g["nplus"])


@pytest.mark.parametrize("name", ["c3", "c3cap", "c4_subset", "c5_shaped"])
def test_oracle_reproduces_bd_compat_fixture_heads(oracle_mod, name):
    """The committed birth-death reference-semantics fixtures are the compat oracle's output: the first
    replicates of every fixture (of every parameter set for the C4 subset) are recomputed and compared."""
    import make_golden
    from ecdna_evo_amd import abi

    g = np.load(os.path.join(GOLDEN, f"{name}_compat_seed42.npz"))
    if name == "c4_subset":
        m = make_golden.C4_REPS
        for i in range(16):
            spec = make_golden.c4_subset_spec(first_replicate=i * m, n_replicates=16)
            r = oracle_mod.run(spec, mode="compat", n_threads=8)
            for f in ("nminus", "nplus", "iters", "stop_reason"):
                np.testing.assert_array_equal(r.summaries[f].astype(np.int64),
                                              g[f][i * m:i * m + 16].astype(np.int64), err_msg=f"set {i}: {f}")
        return
    mk = {"c3": make_golden.c3_spec, "c5_shaped": make_golden.c5_shaped_spec,
          "c3cap": lambda **kw: make_golden.c3_spec(flags=abi.FLAG_BD_CAP_COMPAT, **kw)}[name]
    n = 16 if name == "c5_shaped" else 256
    r = oracle_mod.run(mk(n=n), mode="compat", n_threads=8)
    for f in ("nminus", "nplus", "iters", "stop_reason"):
        np.testing.assert_array_equal(r.summaries[f].astype(np.int64), g[f][:n].astype(np.int64), err_msg=f)
    if name == "c3cap":
        s = r.summaries
        full = s["stop_reason"] == abi.STOP_MAX_CELLS
        assert full.any() and np.all((s["nminus"] + s["nplus"])[full] == 5_000)
