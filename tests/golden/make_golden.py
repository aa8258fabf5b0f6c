#!/usr/bin/env python3
"""Generates the committed fixtures in tests/golden/ from the CPU oracle (oracle/).

The reference (Rust; crates not vendored, no toolchain here) holds no golden vectors and cannot be
run, so these fixtures are regression pins of the oracle itself:

  parity_cases.npz     philox-mode outputs (summaries, histogram, sha256 of the final rows) of every
                       case in tests/cases.py (row store: cases(); bin store: bin_cases()). CPU tests
                       require the oracle to reproduce them; GPU tests require the engine to
                       reproduce them.
  refdraws_cases.npz   compat-mode outputs (the reference's draw structure) of every row-store case, which
                       the engine's ECDNA_FLAG_REFERENCE_DRAWS mode must reproduce bit for bit.
  c3_compat_seed42.npz, c4_subset_compat_seed42.npz, c5_shaped_compat_seed42.npz
                       reference-semantics runs of the birth-death configurations: C3 (65,536 replicates),
                       16 sets of the C4 sweep x 16,384 replicates (ABC rejects per set, abc.md:38-55, so each
                       set's law is held to KS < 0.01 on its own), C5's turnover process to 2e4 cells (4,096
                       replicates): pooled histograms + per-replicate final n-, n+, events, stop reason.
  c3cap_compat_seed42.npz
                       C3 under the other plausible reading of sosa's cell cap: the
                       cap tested against the sum of BirthDeath's duplicated population vector [n-, n+, n-, n+]
                       (src/process.rs:339-344), i.e. a stop at n- + n+ >= max_cells / 2
                       (ECDNA_FLAG_BD_CAP_COMPAT); 65,536 replicates.
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


def make_refdraws():
    """The compat oracle (the reference's draw structure) on every row-store parity case: the engine's
    ECDNA_FLAG_REFERENCE_DRAWS mode must reproduce it (tests/test_gpu_refdraws.py)."""
    from test_gpu_refdraws import refdraws_cases

    out = {}
    for name, spec in sorted(refdraws_cases().items()):
        r = oracle.run(spec, mode="compat", want_rows=True)
        out[f"{name}__summaries"] = r.summaries
        out[f"{name}__hist"] = r.hist
        out[f"{name}__rows_sha256"] = np.array(rows_digest(r))
    np.savez_compressed(os.path.join(HERE, "refdraws_cases.npz"), **out)


# --- reference-semantics fixtures of the birth-death configurations (BASELINE.json configs[2..4]); the GPU
# KS tests (tests/test_gpu_statistics.py) compare the engine's philox mapping with them in law

C3_REPS = 65_536


def c3_spec(n=C3_REPS, **kw):
    """C3: birth-death b0 = 1, b1 = 1.5, d0 = d1 = 0.3 (b1 != b0: the reference's fitness lever,
    src/main.rs:130-173, src/process.rs:259-345), binomial segregation, {1: 1}, 1e4 cells or t = 17, seed 42."""
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), reps_per_set=1 << 20,
             n_replicates=n, max_cells=10_000, hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


# C4 subset: 16 of the sweep's 1024 (b1 = s, d0 = d1 = d, k0) sets spanning s in [1, 2.5], d in [0, 0.7] and
# k0 in {1, 16, 128} (bench.py workload_spec("c4") grid: set i has s = 1 + 1.5 (i % 16) / 15,
# d = 0.7 ((i // 16) % 8) / 7, k0 = 2^(i // 128))
C4_SETS = [0, 21, 42, 63, 85, 112, 527, 533, 550, 567, 585, 620, 903, 920, 938, 1023]
C4_REPS = 16384


def c4_subset_spec(reps_per_set=C4_REPS, **kw):
    rates, inits = [], []
    for i in C4_SETS:
        sel, dd = 1.0 + 1.5 * (i % 16) / 15.0, 0.7 * ((i // 16) % 8) / 7.0
        rates.append((1.0, sel, dd, dd))
        inits.append({1 << (i // 128): 1})
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=rates, reps_per_set=reps_per_set,
             n_replicates=reps_per_set * len(C4_SETS), max_cells=10_000, init_per_set=inits, hist_bins=1025,
             flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


C5_REPS = 4096


def c5_shaped_spec(n=C5_REPS, **kw):
    """C5's turnover process (b0 = b1 = 1, d0 = d1 = 0.9, {1: 1000}) to 2e4 cells: a horizon (t ~ 30) where the
    reference's f32 process.time still advances (tau ~ 2.6e-5 against ulp(30) = 1.9e-6; C5's 1e6 cells would
    freeze it). The GPU side runs with f32 time (ECDNA_FLAG_TIME_F32) like the reference."""
    d = dict(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), reps_per_set=262_144,
             n_replicates=n, max_cells=20_000, max_time=1000.0, init={1: 1000}, hist_bins=1025, flags=0)
    d.update(kw)
    return abi.RunSpec(**d)


def _per_replicate(r):
    s = r.summaries
    return dict(hist=r.hist, nminus=s["nminus"].astype(np.uint32), nplus=s["nplus"].astype(np.uint32),
                iters=s["iters"].astype(np.uint32), stop_reason=s["stop_reason"].astype(np.uint8))


def make_bd_compat(only=None):
    for name, spec in (("c3_compat_seed42", c3_spec()), ("c4_subset_compat_seed42", c4_subset_spec()),
                       ("c5_shaped_compat_seed42", c5_shaped_spec()),
                       ("c3cap_compat_seed42", c3_spec(flags=abi.FLAG_BD_CAP_COMPAT))):
        if only and not name.startswith(only + "_"):
            continue
        r = oracle.run(spec, mode="compat")
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **_per_replicate(r))


def make_c2():
    r = oracle.run(c2_spec(), mode="compat")
    np.savez_compressed(os.path.join(HERE, "c2_compat_seed42.npz"), hist=r.hist[0],
                        nminus=r.summaries["nminus"].astype(np.uint32),
                        nplus=r.summaries["nplus"].astype(np.uint32),
                        stop_reason=r.summaries["stop_reason"].astype(np.uint8))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["parity", "c2", "refdraws", "bd"])
    ap.add_argument("--bd", choices=["c3", "c4_subset", "c5_shaped", "c3cap"], help="with --only bd: one fixture")
    a = ap.parse_args()
    oracle.build()
    if a.only in (None, "parity"):
        make_parity()
    if a.only in (None, "c2"):
        make_c2()
    if a.only in (None, "refdraws"):
        make_refdraws()
    if a.only in (None, "bd"):
        make_bd_compat(a.bd)
