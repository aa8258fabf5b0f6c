"""TEST INFRASTRUCTURE ONLY — ctypes loader for the CPU oracle (oracle/_build/libecdna_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and only
as the checker / the timed CPU baseline. The product (ecdna-evo_amd/) never loads it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "ecdna-evo_amd"))

from ecdna_evo_amd import abi  # noqa: E402

LIB_PATH = os.path.join(HERE, "_build", "libecdna_oracle.so")


def build(quiet: bool = True) -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError(f"oracle build failed:\n{out.stdout}\n{out.stderr}")
    if not quiet:
        print(out.stdout)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    L.oracle_philox4x32_10.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
    L.oracle_philox4x32_10.restype = None
    L.oracle_softlog_neg.argtypes = [C.c_uint32]
    L.oracle_softlog_neg.restype = C.c_float
    L.oracle_channel.argtypes = [P(C.c_float), C.c_uint64, C.c_uint64, C.c_int, C.c_uint32]
    L.oracle_channel.restype = C.c_int
    L.oracle_softlog_many.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p]
    L.oracle_softlog_many.restype = None
    for fn in (L.oracle_run_philox, L.oracle_run_compat):
        fn.argtypes = [P(abi.Params), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
        fn.restype = C.c_int
    L.oracle_increase_nplus.argtypes = [C.c_void_p, C.c_int, C.c_uint64, C.c_uint64, C.c_uint32,
                                        P(C.c_uint32), P(C.c_uint32), P(C.c_int)]
    L.oracle_increase_nplus.restype = C.c_int
    L.oracle_decrease_nplus.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32]
    L.oracle_decrease_nplus.restype = C.c_int
    L.oracle_set_snapshot_outputs.argtypes = [C.c_void_p, C.c_void_p]
    L.oracle_set_snapshot_outputs.restype = None
    L.oracle_set_rng_words_output.argtypes = [C.c_void_p]
    L.oracle_set_rng_words_output.restype = None
    L.oracle_compat_subsample.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                          P(C.c_uint64), C.c_void_p]
    L.oracle_compat_subsample.restype = C.c_int64
    L.oracle_increase_nminus.argtypes = [C.c_void_p]
    L.oracle_increase_nminus.restype = C.c_int
    L.oracle_decrease_nminus.argtypes = [C.c_void_p]
    L.oracle_decrease_nminus.restype = C.c_int
    L.oracle_segregate.argtypes = [C.c_int, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32,
                                   P(C.c_uint32), P(C.c_uint32), P(C.c_int)]
    L.oracle_segregate.restype = C.c_int
    L.oracle_chacha_block.argtypes = [P(C.c_uint32), P(C.c_uint32), C.c_int]
    L.oracle_chacha_block.restype = None
    L.oracle_chacha_seed_from_u64.argtypes = [C.c_uint64, P(C.c_uint32)]
    L.oracle_chacha_seed_from_u64.restype = None
    L.oracle_chacha_new.argtypes = [C.c_uint64, C.c_uint64]
    L.oracle_chacha_new.restype = C.c_void_p
    L.oracle_chacha_free.argtypes = [C.c_void_p]
    L.oracle_chacha_free.restype = None
    L.oracle_chacha_next_u32.argtypes = [C.c_void_p]
    L.oracle_chacha_next_u32.restype = C.c_uint32
    L.oracle_chacha_next_u64.argtypes = [C.c_void_p]
    L.oracle_chacha_next_u64.restype = C.c_uint64
    L.oracle_compat_gen_range.argtypes = [C.c_void_p, C.c_uint64]
    L.oracle_compat_gen_range.restype = C.c_uint64
    L.oracle_compat_exp1.argtypes = [C.c_void_p]
    L.oracle_compat_exp1.restype = C.c_double
    L.oracle_compat_binomial.argtypes = [C.c_void_p, C.c_uint64, C.c_double]
    L.oracle_compat_binomial.restype = C.c_uint64
    L.oracle_compat_log.argtypes = [C.c_double]
    L.oracle_compat_log.restype = C.c_double
    L.oracle_compat_exp.argtypes = [C.c_double]
    L.oracle_compat_exp.restype = C.c_double
    L.oracle_compat_exp_approx.argtypes = [C.c_double]
    L.oracle_compat_exp_approx.restype = C.c_double
    L.oracle_compat_log_approx.argtypes = [C.c_double]
    L.oracle_compat_log_approx.restype = C.c_double
    _lib = L
    return L


def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def channel(rates, nminus: int, nplus: int, birth_death: bool, w1: int) -> int:
    """The channel the engine's direct method draws with word w1 from (n-, n+) (draw mapping v7): 0 ProliferateNMinus,
    1 ProliferateNPlus, 2 DeathNMinus, 3 DeathNPlus, -1 absorbing."""
    r = (C.c_float * 4)(*[float(x) for x in rates])
    return lib().oracle_channel(r, nminus, nplus, 1 if birth_death else 0, w1)


def softlog_many(words) -> np.ndarray:
    """oracle_softlog_neg over an array of u32 words (f32 results)."""
    w = np.ascontiguousarray(words, dtype=np.uint32)
    out = np.empty(len(w), dtype=np.float32)
    lib().oracle_softlog_many(w.ctypes.data, len(w), out.ctypes.data)
    return out


def softlog_neg(w: int) -> float:
    return lib().oracle_softlog_neg(w)


class OracleResult:
    def __init__(self, summaries, hist, totals, rows, row_stride):
        self.summaries = summaries
        self.hist = hist
        self.totals = totals
        self.rows = rows
        self.row_stride = row_stride

    def row(self, i: int) -> np.ndarray:
        n = int(self.summaries[i]["nplus"])
        return self.rows[i, :n]

    def snapshot_row(self, i: int, s: int) -> np.ndarray:
        return self.snapshot_rows[i, s, : int(self.snapshots[i, s]["nplus"])]


def run(spec: "abi.RunSpec", mode: str = "philox", n_threads: int = 0, want_rows: bool = False) -> OracleResult:
    p = spec.params()
    n = p.n_replicates
    summ = abi.summaries_array(n)
    hist = np.zeros(p.n_param_sets * p.hist_bins, dtype=np.uint64)
    tot = abi.totals_array(p.n_param_sets)
    stride = int(p.cell_cap)
    rows = np.zeros((n, stride), dtype=np.uint16) if want_rows else None
    fn = lib().oracle_run_philox if mode == "philox" else lib().oracle_run_compat
    S = p.n_snapshots
    meta = np.zeros((n, S), dtype=abi.SNAPSHOT_DTYPE) if S else None
    srows = np.zeros((n, S, p.cell_cap), dtype=np.uint16) if (S and p.flags & abi.FLAG_SNAPSHOT_ROWS) else None
    lib().oracle_set_snapshot_outputs(meta.ctypes.data if meta is not None else None,
                                      srows.ctypes.data if srows is not None else None)
    words = np.zeros(n, dtype=np.uint64) if mode == "compat" else None
    lib().oracle_set_rng_words_output(words.ctypes.data if words is not None else None)
    try:
        rc = fn(C.byref(p), summ.ctypes.data, hist.ctypes.data, tot.ctypes.data,
                rows.ctypes.data if rows is not None else None, stride, n_threads)
    finally:
        lib().oracle_set_snapshot_outputs(None, None)
        lib().oracle_set_rng_words_output(None)
    if rc != 0:
        raise ValueError(f"oracle run failed: {rc}")
    res = OracleResult(summ, hist.reshape(p.n_param_sets, p.hist_bins), tot, rows, stride)
    res.snapshots, res.snapshot_rows = meta, srows
    res.rng_words = words  # compat: ChaCha8 words each replicate's stream handed out
    return res


def compat_subsample(nplus_cells, nminus: int, nb_cells: int, seed: int, stream: int, word_pos: int):
    """ecdna-lib into_subsampled as reconstructed (oracle_compat_subsample): the chosen cells' copy numbers
    (0 = N-) in index-vector order, and the stream's word position after it."""
    cells = np.ascontiguousarray(np.asarray(nplus_cells, dtype=np.uint16))
    total = len(cells) + int(nminus)
    out = np.zeros(max(1, min(int(nb_cells), total)), dtype=np.uint16)
    wp = C.c_uint64(int(word_pos))
    k = lib().oracle_compat_subsample(cells.ctypes.data if len(cells) else None, len(cells), int(nminus),
                                      int(nb_cells), int(seed), int(stream), C.byref(wp), out.ctypes.data)
    if k < 0:
        raise ValueError("oracle_compat_subsample failed")
    return out[:k], wp.value


class Distr(C.Structure):
    """oracle_distr_t — EcDNADistribution restated (n- plus one u16 per N+ cell)."""

    _fields_ = [("cells", C.POINTER(C.c_uint16)), ("len", C.c_uint64), ("cap", C.c_uint64), ("nminus", C.c_uint64)]


class Distribution:
    def __init__(self, cells, nminus: int, cap: Optional[int] = None):
        cells = np.asarray(cells, dtype=np.uint16)
        cap = cap if cap is not None else len(cells) + 2
        self.buf = np.zeros(max(cap, 1), dtype=np.uint16)
        self.buf[: len(cells)] = cells
        self.d = Distr(self.buf.ctypes.data_as(C.POINTER(C.c_uint16)), len(cells), cap, nminus)

    @property
    def nplus(self) -> int:
        return int(self.d.len)

    @property
    def nminus(self) -> int:
        return int(self.d.nminus)

    def cells(self) -> np.ndarray:
        return self.buf[: self.d.len].copy()

    def increase_nplus(self, seg: int, seed: int, rid: int, e: int):
        k1, k2, un = C.c_uint32(), C.c_uint32(), C.c_int()
        rc = lib().oracle_increase_nplus(C.byref(self.d), seg, seed, rid, e, C.byref(k1), C.byref(k2), C.byref(un))
        return rc, k1.value, k2.value, un.value

    def decrease_nplus(self, seed: int, rid: int, e: int) -> int:
        return lib().oracle_decrease_nplus(C.byref(self.d), seed, rid, e)

    def increase_nminus(self) -> int:
        return lib().oracle_increase_nminus(C.byref(self.d))

    def decrease_nminus(self) -> int:
        return lib().oracle_decrease_nminus(C.byref(self.d))

    def mean(self) -> float:
        # EcDNADistribution::compute_mean: mean copy number over all cells, N- included
        total = self.nminus + self.nplus
        return float(self.cells().astype(np.float64).sum() / total) if total else float("nan")


def segregate(seg: int, n: int, seed: int, rid: int, e: int):
    k1, k2, un = C.c_uint32(), C.c_uint32(), C.c_int()
    rc = lib().oracle_segregate(seg, n, seed, rid, e, C.byref(k1), C.byref(k2), C.byref(un))
    return rc, k1.value, k2.value, un.value


class ChaCha:
    def __init__(self, seed: int, stream: int):
        self.h = lib().oracle_chacha_new(seed, stream)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_chacha_free(self.h)
            self.h = None

    def next_u32(self) -> int:
        return lib().oracle_chacha_next_u32(self.h)

    def next_u64(self) -> int:
        return lib().oracle_chacha_next_u64(self.h)

    def gen_range(self, n: int) -> int:
        return lib().oracle_compat_gen_range(self.h, n)

    def exp1(self) -> float:
        return lib().oracle_compat_exp1(self.h)

    def binomial(self, n: int, p: float) -> int:
        return lib().oracle_compat_binomial(self.h, n, p)


def compat_log(x: float) -> float:
    return lib().oracle_compat_log(x)


def compat_exp(x: float) -> float:
    return lib().oracle_compat_exp(x)


def compat_exp_approx(x: float) -> float:
    """csrc/refdraws.hpp exp_approx restated (the wedge-test filter; tests only)."""
    return lib().oracle_compat_exp_approx(x)


def compat_log_approx(x: float) -> float:
    """csrc/refdraws.hpp log_approx restated (BTPE's region-3/4 filter; tests only)."""
    return lib().oracle_compat_log_approx(x)


def chacha_block(state, rounds: int):
    i = (C.c_uint32 * 16)(*state)
    o = (C.c_uint32 * 16)()
    lib().oracle_chacha_block(i, o, rounds)
    return list(o)


def chacha_key_from_u64(seed: int):
    k = (C.c_uint32 * 8)()
    lib().oracle_chacha_seed_from_u64(seed, k)
    return list(k)
