"""TEST INFRASTRUCTURE ONLY — numpy restatement of the per-replicate ABC summary statistics
(abc.md:38-55: "ecdna" = KS distance between the ecDNA distributions, "mean" = relative difference of
the means, "entropy" = relative difference of the entropies, "frequency" of N+ cells). The statistics
live in the external ecdna-lib 3.0.2 (Cargo.lock:423-438, not vendored) and are unpinned; the engine
defines them as in include/ecdna_ssa.h (ecdna_rep_stats_t) and this module restates that definition.
"""
import numpy as np


def target_summary(target_hist):
    t = np.asarray(target_hist, dtype=np.float64)
    tot = t.sum()
    p = t / tot
    cdf = np.cumsum(p)
    mean = float((np.arange(len(t)) * t).sum() / tot)
    nz = p[p > 0]
    ent = float(-(nz * np.log(nz)).sum())
    freq = float(1.0 - t[0] / tot)
    return cdf, mean, ent, freq


def rep_stats(nminus, row, bins, target_hist=None):
    """Statistics of one replicate's final distribution: n- N- cells and the N+ copy numbers `row`."""
    row = np.asarray(row, dtype=np.int64)
    cells = int(nminus) + len(row)
    h = np.bincount(np.minimum(row, bins - 1), minlength=bins).astype(np.float64)
    h[0] += nminus
    out = dict(cells=cells, mean=0.0, entropy=0.0, frequency=0.0, ks=0.0, mean_rel=0.0, entropy_rel=0.0,
               frequency_diff=0.0)
    if cells:
        p = h / cells
        nz = p[p > 0]
        out["mean"] = float(row.sum() / cells)
        out["entropy"] = float(-(nz * np.log(nz)).sum())
        out["frequency"] = len(row) / cells
    if target_hist is not None:
        cdf_t, mean_t, ent_t, freq_t = target_summary(target_hist)
        out["ks"] = float(np.abs(np.cumsum(h / cells) - cdf_t).max()) if cells else 1.0
        dm, de = abs(out["mean"] - mean_t), abs(out["entropy"] - ent_t)
        out["mean_rel"] = dm / mean_t if mean_t > 0 else dm
        out["entropy_rel"] = de / ent_t if ent_t > 0 else de
        out["frequency_diff"] = abs(out["frequency"] - freq_t)
    return out
