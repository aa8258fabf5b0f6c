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
