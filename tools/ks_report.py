"""The north star's KS clause, measured: the engine (philox mapping, bench settings) against the committed
reference-semantics fixtures of C2..C5 (tests/golden/), printed as one JSON document (pooled copy-number
histogram KS, per-replicate two-sample KS p-values, extinction fractions) — the numbers DESIGN.md §4.2 quotes;
tests/test_gpu_statistics.py asserts the bounds. Usage: python tools/ks_report.py > out.json"""
import json
import os
import sys

import numpy as np
from scipy import stats

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "ecdna-evo_amd"), os.path.join(REPO, "tests", "golden"), os.path.join(REPO, "tests")]
from ecdna_evo_amd import abi, engine  # noqa: E402
import make_golden  # noqa: E402


def ks(h1, h2):
    c1 = np.cumsum(h1.astype(np.float64)) / h1.sum()
    c2 = np.cumsum(h2.astype(np.float64)) / h2.sum()
    return float(np.abs(c1 - c2).max())


def per_rep(s, g):
    out = {}
    for f in ("nminus", "nplus", "iters"):
        out[f] = float(stats.ks_2samp(s[f].astype(np.float64), g[f].astype(np.float64)).pvalue)
    return out


def main():
    rep = {}
    stores = {"bins": abi.FLAG_BIN_STORE, "rows": 0}
    for name, mk, n, kmax, extra in (("c3", make_golden.c3_spec, dict(n=1 << 20), 32, 0),
                                     ("c4_subset", make_golden.c4_subset_spec, dict(reps_per_set=16384), 64, 0),
                                     ("c5_shaped", make_golden.c5_shaped_spec, dict(n=32768), 64, abi.FLAG_TIME_F32)):
        g = np.load(os.path.join(REPO, "tests", "golden", f"{name}_compat_seed42.npz"))
        gh = g["hist"].reshape(-1, 1025)
        for store, fl in stores.items():
            r = engine.run(mk(flags=fl | extra, bin_kmax=kmax if store == "bins" else 0, **n))
            d = {"pooled_ks": ks(r.hist.sum(axis=0), gh.sum(axis=0)), "replicates_gpu": len(r.summaries),
                 "replicates_fixture": len(g["iters"])}
            if name == "c4_subset":
                d["per_set_ks_max"] = max(ks(r.hist[i], gh[i]) for i in range(16))
            else:
                d["per_replicate_ks_pvalues"] = per_rep(r.summaries, g)
                d["extinct_gpu"] = float(np.mean(r.summaries["stop_reason"] == abi.STOP_ABSORBING))
                d["extinct_fixture"] = float(np.mean(g["stop_reason"] == abi.STOP_ABSORBING))
            rep[f"{name}/{store}"] = d
        rr = engine.run(mk(flags=abi.FLAG_REFERENCE_DRAWS))
        same = bool(np.array_equal(rr.hist.reshape(-1), g["hist"].reshape(-1)) and
                    all(np.array_equal(rr.summaries[f].astype(np.int64), g[f].astype(np.int64))
                        for f in ("nminus", "nplus", "iters", "stop_reason")))
        rep[f"{name}/reference_draws_seed_for_seed"] = same
    g = np.load(os.path.join(REPO, "tests", "golden", "c2_compat_seed42.npz"))
    for store, fl in stores.items():
        r = engine.run(abi.RunSpec(seed=42, n_replicates=65536, max_cells=10_000, hist_bins=1025, flags=fl,
                                   bin_kmax=32 if store == "bins" else 0))
        rep[f"c2/{store}"] = {"pooled_ks": ks(r.hist[0], g["hist"])}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
