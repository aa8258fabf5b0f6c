#!/usr/bin/env python3
"""Generates the committed fixtures in tests/golden/ from the CPU oracle (oracle/).

The reference (Rust; crates not vendored, no toolchain here) holds no golden vectors and cannot be
run, so these fixtures are regression pins of the oracle itself:

  parity_cases.npz     philox-mode outputs (summaries, histogram, sha256 of the final rows) of every
                       case in tests/cases.py (row store: cases(); bin store: bin_cases()). CPU tests
                       require the oracle to reproduce them; GPU tests require the engine to
                       reproduce them.
  c2_compat_seed42.npz reference-semantics run (ChaCha8 streams seed*10+i, first-reaction, BTPE) of
                       the C2 shape: 65,536 replicates, pure birth + binomial to 1e4 cells, seed 42:
                       pooled copy-number histogram + per-replicate final n-/n+. The GPU KS test
                       compares the engine's histogram against it (target KS < 0.01).

Usage: python tests/golden/make_golden.py [--only parity|c2]
"""
import argparse
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "ecdna-evo_amd"), os.path.join(REPO, "oracle"), os.path.dirname(HERE)]

import oracle  # noqa: E402
from cases import bin_cases, cases  # noqa: E402
from ecdna_evo_amd import abi  # noqa: E402


def rows_digest(res) -> str:
    h = hashlib.sha256()
    for i in range(len(res.summaries)):
        h.update(res.row(i).tobytes())
        h.update(b"|")
    return h.hexdigest()


def snapshot_digest(res) -> str:
    h = hashlib.sha256()
    if res.snapshot_rows is None:
        return ""
    for i in range(res.snapshots.shape[0]):
        for s in range(res.snapshots.shape[1]):
            h.update(res.snapshot_row(i, s).tobytes())
            h.update(b"|")
    return h.hexdigest()


def c2_spec():
    return abi.RunSpec(seed=42, n_replicates=65536, max_cells=10_000, hist_bins=1025, flags=0)


def make_parity():
    out = {}
    for name, spec in sorted({**cases(), **bin_cases()}.items()):
        r = oracle.run(spec, mode="philox", want_rows=True)
        out[f"{name}__summaries"] = r.summaries
        out[f"{name}__hist"] = r.hist
        out[f"{name}__rows_sha256"] = np.array(rows_digest(r))
        if r.snapshots is not None:
            out[f"{name}__snapshots"] = r.snapshots
            out[f"{name}__snapshot_rows_sha256"] = np.array(snapshot_digest(r))
    np.savez_compressed(os.path.join(HERE, "parity_cases.npz"), **out)


def make_c2():
    r = oracle.run(c2_spec(), mode="compat")
    np.savez_compressed(os.path.join(HERE, "c2_compat_seed42.npz"), hist=r.hist[0],
                        nminus=r.summaries["nminus"].astype(np.uint32),
                        nplus=r.summaries["nplus"].astype(np.uint32),
                        stop_reason=r.summaries["stop_reason"].astype(np.uint8))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["parity", "c2"])
    a = ap.parse_args()
    oracle.build()
    if a.only in (None, "parity"):
        make_parity()
    if a.only in (None, "c2"):
        make_c2()
