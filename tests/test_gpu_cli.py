"""The ecdna-dynamics CLI on the GPU against the oracle: every JSON file the reference would write
(snapshots, end-of-run distribution, subsamples; src/main.rs:100-123, src/process.rs:31-55,
122-145) exists at the same path with the same histogram, and no other file is written."""
import json
import os
import subprocess

import numpy as np
import pytest

from ecdna_evo_amd import abi
from test_host import subsample_py

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "ecdna-evo_amd", "bin", "ecdna-dynamics")


def rate_str(x):
    return np.format_float_positional(np.float32(x), trim="-").replace(".", "dot")


def timepoint(t):
    return ("%.1f" % float(np.float32(t))).replace(".", "dot") + "years"


def hist_json(nminus, cells):
    h = {"0": int(nminus)}
    for k, c in zip(*np.unique(np.asarray(cells, np.int64), return_counts=True)):
        h[str(int(k))] = int(c)
    return h


def expected_files(spec, res, b, subsamples, reference=False):
    """reference: --draws reference, whose subsamples continue each replicate's ChaCha8 stream where the run left it
    (res.rng_words), chained over the subsample sizes (src/main.rs:110-123; oracle.compat_subsample)."""
    out = {}
    bd = spec.process == abi.BIRTH_DEATH
    for i in range(spec.n_replicates):
        idx = spec.seed * 10 + i
        fn = (f"{rate_str(b[0])}b0_{rate_str(b[1])}b1_{rate_str(b[2])}d0_{rate_str(b[3])}d1_{idx}idx" if bd
              else f"{rate_str(b[0])}b0_{rate_str(b[1])}b1_0d0_0d1_{idx}idx")

        def put(nm, cells, t):
            n = int(nm) + len(cells)
            out[f"{n}cells/ecdna/{timepoint(t)}/{fn}.json"] = hist_json(nm, cells)

        for s in range(res.snapshots.shape[1]):
            m = res.snapshots[i, s]
            if m["taken"]:
                put(m["nminus"], res.snapshot_row(i, s), m["time"])
        s = res.summaries[i]
        row = res.row(i)
        put(s["nminus"], row, s["time"])
        word = int(res.rng_words[i]) if reference else 0
        for k, nb in enumerate(subsamples):
            if reference:
                cells, word = oracle_compat_subsample(row, int(s["nminus"]), nb, spec.seed, idx, word)
                p, m = [int(c) for c in cells if c], int(np.sum(cells == 0))
            else:
                p, m = subsample_py(row.tolist(), int(s["nminus"]), nb, spec.seed, i, k)
            put(m, p, s["time"])
    return out


def oracle_compat_subsample(*a):
    import oracle

    return oracle.compat_subsample(*a)


def written_files(root):
    got = {}
    for d, _, files in os.walk(root):
        for f in files:
            p = os.path.join(d, f)
            got[os.path.relpath(p, root)] = json.load(open(p))
    return got


CASES = {
    "pb_defaults": (["--runs", "6", "--seed", "42", "--subsamples=10,100"], dict(process=abi.PURE_BIRTH, cells=1000,
                                                                                rates=(1, 1, 0, 0), subs=[10, 100])),
    "bd_c3_shape": (["--runs", "5", "--seed", "7", "--b1", "1.5", "--d0", "0.3", "--d1", "0.3", "-c", "800",
                     "--snapshots=5,50,400", "--subsamples=20"],
                    dict(process=abi.BIRTH_DEATH, cells=800, rates=(1, 1.5, 0.3, 0.3), subs=[20], snaps=[5, 50, 400])),
}


@pytest.mark.gpu
@pytest.mark.parametrize("store", ["bins", "rows", "reference"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_cli_writes_what_the_reference_writes(name, store, engine_mod, oracle_mod, tmp_path):
    """store "reference": --draws reference, the Rust binary's own draw structure (ChaCha8 + rand_distr), so
    every snapshot and end-of-run file equals the compat oracle's seed for seed, and the subsample files continue
    each replicate's own ChaCha8 stream as the reference's `into_subsampled(n, &mut rng)` does (src/main.rs:110-123;
    ecdna-lib's into_subsampled reconstructed, parity unpinned: DESIGN.md §10)."""
    args, c = CASES[name]
    extra = ["--draws", "reference"] if store == "reference" else ["--cell-store", store]
    out = subprocess.run([CLI, *args, *extra, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    runs = int(args[args.index("--runs") + 1])
    seed = int(args[args.index("--seed") + 1])
    snaps = c.get("snaps") or abi.default_snapshots(c["cells"])
    spec = abi.RunSpec(process=c["process"], rates=(c["rates"],), seed=seed, n_replicates=runs, max_cells=c["cells"],
                       snapshots=snaps, bin_kmax=64 if store == "bins" else 0,
                       flags=abi.FLAG_TIME_F32 | abi.FLAG_SNAPSHOT_ROWS | (abi.FLAG_BIN_STORE if store == "bins" else 0))
    res = oracle_mod.run(spec, mode="compat" if store == "reference" else "philox", want_rows=True)
    want = expected_files(spec, res, c["rates"], c["subs"], reference=store == "reference")
    got = written_files(tmp_path)
    assert set(got) == set(want)
    for k in want:
        assert got[k] == want[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("store", ["bins", "rows"])
def test_cli_pooled_histogram_is_the_reduced_run(store, engine_mod, tmp_path):
    """--pooled: the run's histogram and totals all-reduced over the GPUs' shards with RCCL
    (ecdna_ssa_comm_init_all + ecdna_ssa_ctx_reduce; one device on this box): equal to one engine run of all
    replicates."""
    pooled = tmp_path / "pooled.json"
    args = ["--runs", "64", "--seed", "42", "--b1", "1.5", "--d0", "0.3", "--d1", "0.3", "-c", "900",
            "--cell-store", store, "--pooled", str(pooled)]
    out = subprocess.run([CLI, *args, str(tmp_path / "out")], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    got = json.load(open(pooled))
    spec = abi.RunSpec(process=abi.BIRTH_DEATH, rates=((1, 1.5, 0.3, 0.3),), seed=42, n_replicates=64, max_cells=900,
                       snapshots=abi.default_snapshots(900), bin_kmax=64 if store == "bins" else 0,
                       flags=abi.FLAG_TIME_F32 | abi.FLAG_SNAPSHOT_ROWS | (abi.FLAG_BIN_STORE if store == "bins" else 0))
    r = engine_mod.run(spec)
    want = {str(b): int(v) for b, v in enumerate(r.hist[0]) if v}
    assert got["histogram"] == want
    t = r.totals[0]
    assert (got["replicates"], got["events"], got["nminus"], got["nplus"], got["errors"]) == \
        (64, int(t["events"]), int(t["nminus"]), int(t["nplus"]), 0)
    assert got["stop_reasons"] == [int(x) for x in t["stop_reasons"]]


@pytest.mark.gpu
def test_cli_pooled_with_zero_runs_writes_an_empty_pool(engine_mod, tmp_path):
    """--pooled with --runs 0 writes an empty pooled histogram (no replicate ran) instead of no file."""
    pooled = tmp_path / "pooled.json"
    out = subprocess.run([CLI, "--runs", "0", "--pooled", str(pooled), str(tmp_path / "out")], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.load(open(pooled))
    assert got["histogram"] == {} and got["replicates"] == 0 and got["events"] == 0
