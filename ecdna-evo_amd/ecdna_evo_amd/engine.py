"""ctypes bindings of libecdna_ssa.so (include/ecdna_ssa.h) — the product's host-side entry points.

`run()` is the batched replacement of the reference's per-replicate `sosa::simulate` calls
(src/main.rs:92-99, 166-173) mapped by rayon over replicate ids (src/main.rs:212-225); `Context`
keeps inputs and outputs resident in HBM for repeated launches and multi-GPU reductions.

There is no CPU fallback: if the HIP library is missing or no gfx950 device is present, every
entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

from . import abi

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # .../ecdna-evo_amd
# ECDNA_SSA_LIB: development override (same-box A/B of two builds, tools/ab_build.sh)
LIB_PATH = os.environ.get("ECDNA_SSA_LIB") or os.path.join(PKG_ROOT, "lib", "libecdna_ssa.so")

EXPORTS = [
    "ecdna_ssa_abi_version",
    "ecdna_ssa_strerror",
    "ecdna_ssa_last_error_message",
    "ecdna_ssa_device_count",
    "ecdna_ssa_run",
    "ecdna_ssa_ctx_create",
    "ecdna_ssa_ctx_set_outputs",
    "ecdna_ssa_ctx_launch",
    "ecdna_ssa_ctx_sync",
    "ecdna_ssa_ctx_device_outputs",
    "ecdna_ssa_ctx_download",
    "ecdna_ssa_ctx_download_snapshots",
    "ecdna_ssa_ctx_download_stats",
    "ecdna_ssa_ctx_download_rng_words",
    "ecdna_ssa_ctx_row_stride",
    "ecdna_ssa_ctx_geometry",
    "ecdna_ssa_ctx_instance",
    "ecdna_ssa_ctx_destroy",
    "ecdna_ssa_comm_unique_id",
    "ecdna_ssa_comm_init_rank",
    "ecdna_ssa_comm_init_all",
    "ecdna_ssa_comm_destroy",
    "ecdna_ssa_reduce_hist",
    "ecdna_ssa_ctx_reduce",
]


class EngineError(RuntimeError):
    pass


_lib = None


def _ensure_single_hip_runtime():
    # torch ships its own libamdhip64.so.7; importing it first makes the soname resolve to that copy,
    # so the engine and torch (streams, RCCL) share one HIP runtime in a process that uses both.
    if os.environ.get("ECDNA_NO_TORCH_PRELOAD"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} is missing: build it with `make -C ecdna-evo_amd` (or __graft_entry__.build())")
    _ensure_single_hip_runtime()
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    L.ecdna_ssa_abi_version.restype = C.c_int
    L.ecdna_ssa_strerror.argtypes = [C.c_int]
    L.ecdna_ssa_strerror.restype = C.c_char_p
    L.ecdna_ssa_last_error_message.restype = C.c_char_p
    L.ecdna_ssa_device_count.restype = C.c_int
    L.ecdna_ssa_run.argtypes = [P(abi.Params), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ecdna_ssa_run.restype = C.c_int
    L.ecdna_ssa_ctx_create.argtypes = [P(abi.Params), P(C.c_void_p)]
    L.ecdna_ssa_ctx_create.restype = C.c_int
    L.ecdna_ssa_ctx_set_outputs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_set_outputs.restype = C.c_int
    L.ecdna_ssa_ctx_launch.argtypes = [C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_launch.restype = C.c_int
    L.ecdna_ssa_ctx_sync.argtypes = [C.c_void_p, P(C.c_float), P(C.c_float)]
    L.ecdna_ssa_ctx_sync.restype = C.c_int
    L.ecdna_ssa_ctx_device_outputs.argtypes = [C.c_void_p, P(C.c_void_p), P(C.c_void_p)]
    L.ecdna_ssa_ctx_device_outputs.restype = C.c_int
    L.ecdna_ssa_ctx_download.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_download.restype = C.c_int
    L.ecdna_ssa_ctx_download_snapshots.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_download_snapshots.restype = C.c_int
    L.ecdna_ssa_ctx_download_stats.argtypes = [C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_download_stats.restype = C.c_int
    L.ecdna_ssa_ctx_download_rng_words.argtypes = [C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_download_rng_words.restype = C.c_int
    L.ecdna_ssa_ctx_row_stride.argtypes = [C.c_void_p]
    L.ecdna_ssa_ctx_row_stride.restype = C.c_int64
    L.ecdna_ssa_ctx_geometry.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint64)]
    L.ecdna_ssa_ctx_geometry.restype = C.c_int
    L.ecdna_ssa_ctx_instance.argtypes = [C.c_void_p, P(abi.Instance)]
    L.ecdna_ssa_ctx_instance.restype = C.c_int
    L.ecdna_ssa_ctx_destroy.argtypes = [C.c_void_p]
    L.ecdna_ssa_ctx_destroy.restype = C.c_int
    L.ecdna_ssa_comm_unique_id.argtypes = [C.c_void_p]
    L.ecdna_ssa_comm_unique_id.restype = C.c_int
    L.ecdna_ssa_comm_init_rank.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, P(C.c_void_p)]
    L.ecdna_ssa_comm_init_rank.restype = C.c_int
    L.ecdna_ssa_comm_init_all.argtypes = [C.c_int, P(C.c_int), P(C.c_void_p)]
    L.ecdna_ssa_comm_init_all.restype = C.c_int
    L.ecdna_ssa_comm_destroy.argtypes = [C.c_void_p]
    L.ecdna_ssa_comm_destroy.restype = C.c_int
    L.ecdna_ssa_reduce_hist.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.ecdna_ssa_reduce_hist.restype = C.c_int
    L.ecdna_ssa_ctx_reduce.argtypes = [C.c_void_p, C.c_void_p]
    L.ecdna_ssa_ctx_reduce.restype = C.c_int
    ver = L.ecdna_ssa_abi_version()
    # (a same-box A/B, tools/ab_build.sh, may load a library of an earlier ABI version whose Params layout is this
    # one's: ECDNA_SSA_ABI_ANY=1 accepts versions ABI_SAME_LAYOUT_SINCE .. ABI_VERSION, never a newer one;
    # results then follow that library's draw mapping)
    any_ok = os.environ.get("ECDNA_SSA_ABI_ANY") == "1" and abi.ABI_SAME_LAYOUT_SINCE <= ver <= abi.ABI_VERSION
    if ver != abi.ABI_VERSION and not any_ok:
        raise EngineError("ABI version mismatch between libecdna_ssa.so and ecdna_evo_amd.abi")
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != 0:
        L = lib()
        raise EngineError(f"{what}: {L.ecdna_ssa_strerror(rc).decode()} ({rc}): "
                          f"{L.ecdna_ssa_last_error_message().decode()}")


def device_count() -> int:
    return lib().ecdna_ssa_device_count()


class Comm:
    """An RCCL communicator made by the engine's C ABI (ecdna_ssa_comm_init_all / init_rank): the multi-GPU
    reduction of ecdna_ssa_ctx_reduce."""

    def __init__(self, handle):
        self.h = handle

    @staticmethod
    def init_all(devices) -> list:
        devs = (C.c_int * len(devices))(*devices)
        out = (C.c_void_p * len(devices))()
        _check(lib().ecdna_ssa_comm_init_all(len(devices), devs, out), "ecdna_ssa_comm_init_all")
        return [Comm(C.c_void_p(out[i])) for i in range(len(devices))]

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * abi.COMM_ID_BYTES)()
        _check(lib().ecdna_ssa_comm_unique_id(buf), "ecdna_ssa_comm_unique_id")
        return bytes(buf)

    @staticmethod
    def init_rank(uid: bytes, n_ranks: int, rank: int, device: int) -> "Comm":
        buf = (C.c_uint8 * abi.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(lib().ecdna_ssa_comm_init_rank(buf, n_ranks, rank, device, C.byref(h)), "ecdna_ssa_comm_init_rank")
        return Comm(h)

    def close(self):
        if getattr(self, "h", None):
            lib().ecdna_ssa_comm_destroy(self.h)
            self.h = None


class Result:
    def __init__(self, summaries, hist, totals, rows=None, row_stride=0):
        self.summaries = summaries
        self.hist = hist
        self.totals = totals
        self.rows = rows
        self.row_stride = row_stride
        self.snapshots = None  # [n][S] abi.SNAPSHOT_DTYPE
        self.snapshot_rows = None  # [n][S][stride] u16 under FLAG_SNAPSHOT_ROWS
        self.stats = None  # [n] abi.STATS_DTYPE under FLAG_REP_STATS
        self.rng_words = None  # [n] u64 under FLAG_REFERENCE_DRAWS: ChaCha8 stream position at the end

    def row(self, i: int) -> np.ndarray:
        return self.rows[i, : int(self.summaries[i]["nplus"])]

    def snapshot_row(self, i: int, s: int) -> np.ndarray:
        return self.snapshot_rows[i, s, : int(self.snapshots[i, s]["nplus"])]


class Context:
    """A device-resident run (ecdna_ssa_ctx): create once, launch many times."""

    def __init__(self, spec: "abi.RunSpec"):
        self.spec = spec
        self.params = spec.params()
        h = C.c_void_p()
        _check(lib().ecdna_ssa_ctx_create(C.byref(self.params), C.byref(h)), "ecdna_ssa_ctx_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().ecdna_ssa_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_outputs(self, d_hist: int = 0, d_totals: int = 0):
        _check(lib().ecdna_ssa_ctx_set_outputs(self.h, d_hist or None, d_totals or None), "set_outputs")

    def launch(self, stream: int = 0):
        _check(lib().ecdna_ssa_ctx_launch(self.h, stream or None), "ecdna_ssa_ctx_launch")

    def sync(self):
        s, hh = C.c_float(), C.c_float()
        _check(lib().ecdna_ssa_ctx_sync(self.h, C.byref(s), C.byref(hh)), "ecdna_ssa_ctx_sync")
        return s.value, hh.value

    def reduce(self, comm: "Comm"):
        """All-reduce (sum) this context's histogram and totals over `comm` on its launch stream (RCCL)."""
        _check(lib().ecdna_ssa_ctx_reduce(self.h, comm.h), "ecdna_ssa_ctx_reduce")

    def geometry(self):
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib().ecdna_ssa_ctx_geometry(self.h, C.byref(a), C.byref(b)), "geometry")
        return a.value, b.value

    def instance(self) -> dict:
        """The kernel instance this context launches (schedule, pairing, rotation, K, VGPRs, ...): ABI v7."""
        ins = abi.Instance()
        _check(lib().ecdna_ssa_ctx_instance(self.h, C.byref(ins)), "instance")
        return ins.as_dict()

    def row_stride(self) -> int:
        return int(lib().ecdna_ssa_ctx_row_stride(self.h))

    def download(self, want_rows: bool = False) -> Result:
        p = self.params
        summ = abi.summaries_array(p.n_replicates)
        hist = np.zeros(p.n_param_sets * p.hist_bins, dtype=np.uint64)
        tot = abi.totals_array(p.n_param_sets)
        rows = None
        stride = 0
        if want_rows:
            stride = self.row_stride()
            if stride <= 0:
                raise EngineError("rows are not downloadable from a chunked run")
            rows = np.zeros((p.n_replicates, stride), dtype=np.uint16)
        _check(lib().ecdna_ssa_ctx_download(self.h, summ.ctypes.data, hist.ctypes.data, tot.ctypes.data,
                                            rows.ctypes.data if rows is not None else None), "download")
        res = Result(summ, hist.reshape(p.n_param_sets, p.hist_bins), tot, rows, stride)
        if p.n_snapshots:
            S = p.n_snapshots
            meta = np.zeros((p.n_replicates, S), dtype=abi.SNAPSHOT_DTYPE)
            srows = None
            if p.flags & abi.FLAG_SNAPSHOT_ROWS:
                st = (p.cell_cap + 63) // 64 * 64  # snapshot rows always use the 128-B aligned stride
                srows = np.zeros((p.n_replicates, S, st), dtype=np.uint16)
            _check(lib().ecdna_ssa_ctx_download_snapshots(self.h, meta.ctypes.data,
                                                          srows.ctypes.data if srows is not None else None),
                   "download_snapshots")
            res.snapshots = meta
            res.snapshot_rows = srows
        if p.flags & abi.FLAG_REP_STATS:
            st = np.zeros(p.n_replicates, dtype=abi.STATS_DTYPE)
            _check(lib().ecdna_ssa_ctx_download_stats(self.h, st.ctypes.data), "download_stats")
            res.stats = st
        if p.flags & abi.FLAG_REFERENCE_DRAWS:
            w = np.zeros(p.n_replicates, dtype=np.uint64)
            _check(lib().ecdna_ssa_ctx_download_rng_words(self.h, w.ctypes.data), "download_rng_words")
            res.rng_words = w
        return res


def run(spec: "abi.RunSpec", want_rows: bool = False) -> Result:
    """Run every replicate of `spec` on device `spec.device` and return host copies of the results."""
    with Context(spec) as ctx:
        ctx.launch()
        ctx.sync()
        return ctx.download(want_rows=want_rows)
