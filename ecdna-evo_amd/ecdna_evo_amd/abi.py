"""ctypes mirror of include/ecdna_ssa.h (the engine's C ABI).

Structs, enums and a `RunSpec` builder that turns the reference's run options
(`SimulationOptions`, src/main.rs:27-44, built by `Cli::build`,
src/clap_app.rs:137-229) into an `ecdna_ssa_params_t` whose host arrays stay
alive as long as the RunSpec does.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

ABI_VERSION = 12
# the oldest library an A/B may load under ECDNA_SSA_ABI_ANY=1: the same Params layout as this ABI (v10 appended
# max_workgroups; v11 and v12 changed no struct)
ABI_SAME_LAYOUT_SINCE = 10

# ecdna_process_t (ProcessType, src/clap_app.rs:311-315)
PURE_BIRTH = 0
BIRTH_DEATH = 1

# ecdna_seg_t (SegregationOptions, src/clap_app.rs:232-238)
SEG_DETERMINISTIC = 0
SEG_BINOMIAL = 1
SEG_BINOMIAL_NO_UNEVEN = 2
SEG_BINOMIAL_NO_NMINUS = 3
SEGREGATION_NAMES = {
    "deterministic": SEG_DETERMINISTIC,
    "binomial": SEG_BINOMIAL,
    "binomial-no-uneven": SEG_BINOMIAL_NO_UNEVEN,
    "binomial-no-nminus": SEG_BINOMIAL_NO_NMINUS,
}

# ecdna_event_t (channel order, src/main.rs:140-145)
EV_PROLIF_NMINUS, EV_PROLIF_NPLUS, EV_DEATH_NMINUS, EV_DEATH_NPLUS = 0, 1, 2, 3

# ecdna_stop_t
STOP_NONE, STOP_MAX_CELLS, STOP_MAX_TIME, STOP_MAX_ITER, STOP_ABSORBING, STOP_ERROR = range(6)
STOP_NAMES = ["None", "MaxCells", "MaxTime", "MaxIter", "Absorbing", "Error"]

# ecdna_rep_error_t
REP_OK, REP_ERR_OVERFLOW, REP_ERR_EMPTY, REP_ERR_CELL_CAP, REP_ERR_REJECTION, REP_ERR_INTERNAL = range(6)

FLAG_TIME_F32 = 0x1
FLAG_BD_CAP_COMPAT = 0x2
FLAG_EVENT_HASH = 0x4
FLAG_SNAPSHOT_ROWS = 0x8

OK = 0
E_INVALID, E_HIP, E_NOMEM, E_NODEVICE, E_STATE, E_COMM = -1, -2, -3, -4, -5, -6
COMM_ID_BYTES = 128

MAX_ITER = 1_000_000_000  # src/main.rs:23
MAX_CELLS = 1_000_000_000  # src/main.rs:25


class Rates(C.Structure):
    _fields_ = [("b0", C.c_float), ("b1", C.c_float), ("d0", C.c_float), ("d1", C.c_float)]


class Params(C.Structure):
    _fields_ = [
        ("process", C.c_int32),
        ("segregation", C.c_int32),
        ("rates", C.POINTER(Rates)),
        ("n_param_sets", C.c_uint32),
        ("hist_bins", C.c_uint32),
        ("reps_per_set", C.c_uint64),
        ("seed", C.c_uint64),
        ("first_replicate", C.c_uint64),
        ("n_replicates", C.c_uint64),
        ("max_cells", C.c_uint64),
        ("max_time", C.c_double),
        ("max_iter", C.c_uint64),
        ("cell_cap", C.c_uint32),
        ("flags", C.c_uint32),
        ("init_copies", C.POINTER(C.c_uint16)),
        ("init_nplus", C.c_uint32),
        ("bin_kmax", C.c_uint32),
        ("init_nminus", C.c_uint64),
        ("init_set_offsets", C.POINTER(C.c_uint32)),
        ("init_set_nminus", C.POINTER(C.c_uint64)),
        ("device", C.c_int32),
        ("big_cap", C.c_uint32),
        ("snapshot_cells", C.POINTER(C.c_uint64)),
        ("n_snapshots", C.c_uint32),
        ("replicate_stride", C.c_uint32),
        ("stats_target_hist", C.POINTER(C.c_uint64)),
        ("set_cost_hint", C.POINTER(C.c_float)),
        ("max_workgroups", C.c_uint32),
        ("reserved0", C.c_uint32),
    ]


STATS_DTYPE = np.dtype([("mean", "<f8"), ("entropy", "<f8"), ("frequency", "<f8"), ("ks", "<f8"),
                        ("mean_rel", "<f8"), ("entropy_rel", "<f8"), ("frequency_diff", "<f8"), ("cells", "<u8")])
assert STATS_DTYPE.itemsize == 64
FLAG_REP_STATS = 0x10
FLAG_BIN_STORE = 0x20  # cells binned by copy number; bin_kmax = 64 or 256
# the reference's own draw structure (ChaCha8 streams seed*10+r, first reaction, rand_distr samplers, f32 time;
# row store only): seed for seed the oracle's compat mode
FLAG_REFERENCE_DRAWS = 0x40
FLAG_ALL = 0x7F  # every defined flag (ecdna_ssa_ctx_create rejects other bits since ABI v11)


# ecdna_ssa_instance_t (ABI v7): the kernel instance a context launches (ecdna_ssa_ctx_instance)
KERNEL_KINDS = {0: "ssa_stepper (rows)", 1: "ssa_stepper_bins (bins)", 2: "ssa_stepper_refdraws (reference draws)"}
SCHEDULE_NAMES = {-1: "n/a", 0: "occupancy-first", 1: "max-ILP", 2: "occupancy-first, 128-VGPR cap", 3: "max-ILP, paired lanes"}


class Instance(C.Structure):
    _fields_ = [
        ("kernel", C.c_int32),
        ("schedule", C.c_int32),
        ("paired", C.c_int32),
        ("rotation", C.c_int32),
        ("rot_tick_log2", C.c_int32),
        ("drain_control", C.c_int32),
        ("cost_order", C.c_int32),
        ("runtime_flags", C.c_int32),
        ("bin_kmax", C.c_uint32),
        ("bin_c32", C.c_uint32),
        ("block_lanes", C.c_uint32),
        ("blocks_per_cu", C.c_uint32),
        ("cus", C.c_uint32),
        ("n_chunks", C.c_uint32),
        ("vgprs", C.c_uint32),
        ("lds_bytes", C.c_uint32),
        ("scratch_bytes", C.c_uint32),
        ("window", C.c_uint32),
        ("chunk_replicates", C.c_uint64),
        ("grid_lanes", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        d = {f: int(getattr(self, f)) for f, _ in self._fields_}
        d["kernel_name"] = KERNEL_KINDS.get(d["kernel"], "?")
        d["schedule_name"] = SCHEDULE_NAMES.get(d["schedule"], "?")
        return d


SNAPSHOT_DTYPE = np.dtype([("time", "<f8"), ("nminus", "<u8"), ("nplus", "<u8"), ("taken", "<u4"),
                           ("reserved", "<u4")])
assert SNAPSHOT_DTYPE.itemsize == 32


def default_snapshots(cells: int, n_snapshots: int = 11):
    """build_snapshots_from_cells (src/clap_app.rs:121-134): [1, 1+dx, ..., cells], dx = cells / 10."""
    dx = cells // (n_snapshots - 1)
    x = [1] * n_snapshots
    for i in range(1, n_snapshots - 1):
        x[i] = x[i - 1] + dx
    x[n_snapshots - 1] = cells
    return sorted(x)


SUMMARY_DTYPE = np.dtype(
    [
        ("nminus", "<u8"),
        ("nplus", "<u8"),
        ("iters", "<u8"),
        ("events_by_type", "<u8", (4,)),
        ("uneven", "<u8"),
        ("time", "<f8"),
        ("event_hash", "<u8"),
        ("stop_reason", "<u4"),
        ("error", "<u4"),
    ]
)
assert SUMMARY_DTYPE.itemsize == 88

TOTALS_DTYPE = np.dtype(
    [
        ("replicates", "<u8"),
        ("events", "<u8"),
        ("events_by_type", "<u8", (4,)),
        ("uneven", "<u8"),
        ("nminus", "<u8"),
        ("nplus", "<u8"),
        ("stop_reasons", "<u8", (6,)),
        ("errors", "<u8"),
    ]
)
assert TOTALS_DTYPE.itemsize == 128


def _ptr(arr: Optional[np.ndarray], ctype):
    if arr is None:
        return C.POINTER(ctype)()
    return arr.ctypes.data_as(C.POINTER(ctype))


@dataclass
class RunSpec:
    """One run of `n_replicates` replicates — the batched form of run_simulations (src/main.rs:55-211)."""

    process: int = PURE_BIRTH
    segregation: int = SEG_BINOMIAL
    rates: Sequence[Sequence[float]] = ((1.0, 1.0, 0.0, 0.0),)  # [b0, b1, d0, d1] per set
    reps_per_set: Optional[int] = None  # default: all replicates in set 0
    seed: int = 26  # src/clap_app.rs:63
    first_replicate: int = 0
    n_replicates: int = 12  # src/clap_app.rs:89
    replicate_stride: int = 1  # replicate i has global id first_replicate + i * replicate_stride
    max_cells: int = 1000  # src/clap_app.rs:149
    max_time: Optional[float] = None  # default: floor(log2(cells) + 4), src/clap_app.rs:151
    max_iter: int = MAX_ITER
    cell_cap: Optional[int] = None  # default: max(max_cells, largest initial N+ count)
    hist_bins: int = 1025
    flags: int = FLAG_EVENT_HASH
    init: Optional[Dict[int, int]] = None  # histogram {copies: cells}; default {1: 1} (src/clap_app.rs:188-191)
    init_per_set: Optional[List[Dict[int, int]]] = None
    device: int = 0
    snapshots: Optional[Sequence[int]] = None  # cell counts (sorted here); None = no snapshots
    stats_target: Optional[Sequence[int]] = None  # target histogram [hist_bins] for ABC distances
    bin_kmax: int = 0  # FLAG_BIN_STORE: binned copy numbers 1..bin_kmax (0 = 64)
    set_cost_hint: Optional[Sequence[float]] = None  # per set: start costlier sets first (speed only)
    big_cap: int = 0  # FLAG_BIN_STORE: large-k row capacity (cells with k > bin_kmax); 0 = cell_cap
    max_workgroups: int = 0  # persistent-grid cap (0 = fill the device); for contexts sharing a GPU (speed only)
    _keep: list = field(default_factory=list, repr=False)

    def stride(self) -> int:
        """The id step as the C ABI reads it: replicate_stride 0 means 1 (include/ecdna_ssa.h)."""
        return self.replicate_stride if self.replicate_stride else 1

    def replicate_ids(self) -> np.ndarray:
        """Global ids of the call's replicates, in summary order."""
        return self.first_replicate + np.arange(self.n_replicates, dtype=np.uint64) * np.uint64(self.stride())

    def last_replicate(self) -> int:
        return self.first_replicate + max(0, self.n_replicates - 1) * self.stride()

    def resolved_max_time(self) -> float:
        if self.max_time is not None:
            return float(self.max_time)
        # (f32::log2(cells as f32) + 4f32) as u64, then `years as f32`
        years = np.log2(np.float32(self.max_cells)) + np.float32(4.0)
        return float(np.float32(int(years)))

    @staticmethod
    def _copies_of(hist: Dict[int, int]):
        """EcDNADistribution::new from a histogram: n- = hist[0], one u16 per N+ cell, keys sorted
        (the reference iterates a HashMap, whose order is random per process: SURVEY.md App. A.2)."""
        nminus = int(hist.get(0, 0))
        cells = []
        for k in sorted(int(k) for k in hist if int(k) > 0):
            if k > 65535:
                raise ValueError(f"copy number {k} does not fit u16")
            cells.extend([k] * int(hist[k]))
        return np.asarray(cells, dtype=np.uint16), nminus

    def params(self) -> Params:
        # ctypes silently masks values that do not fit a field (a stride of 2^32 would become 0, i.e. 1):
        # reject them here instead
        for name, bits in (("replicate_stride", 32), ("big_cap", 32), ("bin_kmax", 32), ("hist_bins", 32),
                           ("n_replicates", 64), ("first_replicate", 64), ("seed", 64), ("max_cells", 64),
                           ("max_iter", 64)):
            v = getattr(self, name)
            if not (0 <= int(v) < (1 << bits)):
                raise ValueError(f"{name} = {v} does not fit the ABI's u{bits} field")
        if self.cell_cap is not None and not (0 <= int(self.cell_cap) < (1 << 32)):
            raise ValueError(f"cell_cap = {self.cell_cap} does not fit the ABI's u32 field")
        self._keep = []
        rates = np.asarray(self.rates, dtype=np.float32).reshape(-1, 4)
        n_sets = rates.shape[0]
        rates_arr = (Rates * n_sets)(*[Rates(*map(float, r)) for r in rates])
        self._keep.append(rates_arr)
        p = Params()
        p.process = self.process
        p.segregation = self.segregation
        p.rates = C.cast(rates_arr, C.POINTER(Rates))
        p.n_param_sets = n_sets
        p.hist_bins = self.hist_bins
        rps = self.reps_per_set
        if rps is None:
            rps = max(1, self.last_replicate() + 1)
        p.reps_per_set = rps
        p.seed = self.seed
        p.first_replicate = self.first_replicate
        p.n_replicates = self.n_replicates
        p.replicate_stride = self.replicate_stride
        p.max_cells = self.max_cells
        p.max_time = self.resolved_max_time()
        p.max_iter = self.max_iter
        p.flags = self.flags
        p.bin_kmax = self.bin_kmax
        p.big_cap = self.big_cap
        p.max_workgroups = self.max_workgroups
        p.device = self.device
        if self.snapshots:
            snaps = np.asarray(sorted(int(x) for x in self.snapshots), dtype=np.uint64)
            self._keep.append(snaps)
            p.snapshot_cells = _ptr(snaps, C.c_uint64)
            p.n_snapshots = len(snaps)
        if self.set_cost_hint is not None:
            hint = np.asarray(self.set_cost_hint, dtype=np.float32)
            if hint.shape != (n_sets,):
                raise ValueError("set_cost_hint needs one value per parameter set")
            self._keep.append(hint)
            p.set_cost_hint = _ptr(hint, C.c_float)
        if self.stats_target is not None:
            tgt = np.asarray(self.stats_target, dtype=np.uint64)
            if tgt.shape != (self.hist_bins,):
                raise ValueError("stats_target must have hist_bins entries")
            self._keep.append(tgt)
            p.stats_target_hist = _ptr(tgt, C.c_uint64)
        max_np = 0
        if self.init_per_set is not None:
            if len(self.init_per_set) != n_sets:
                raise ValueError("init_per_set needs one histogram per parameter set")
            parts = [self._copies_of(h) for h in self.init_per_set]
            offs = np.zeros(n_sets + 1, dtype=np.uint32)
            offs[1:] = np.cumsum([len(c) for c, _ in parts])
            copies = np.concatenate([c for c, _ in parts]).astype(np.uint16) if offs[-1] else np.zeros(1, np.uint16)
            nms = np.asarray([nm for _, nm in parts], dtype=np.uint64)
            self._keep += [copies, offs, nms]
            p.init_copies = _ptr(copies, C.c_uint16)
            p.init_nplus = 0
            p.init_nminus = 0
            p.init_set_offsets = _ptr(offs, C.c_uint32)
            p.init_set_nminus = _ptr(nms, C.c_uint64)
            max_np = int(np.max(np.diff(offs))) if n_sets else 0
        else:
            copies, nm = self._copies_of(self.init if self.init is not None else {1: 1})
            buf = copies if len(copies) else np.zeros(1, np.uint16)
            self._keep.append(buf)
            p.init_copies = _ptr(buf, C.c_uint16)
            p.init_nplus = len(copies)
            p.init_nminus = nm
            max_np = len(copies)
        cap = self.cell_cap
        if cap is None:
            cap = max(int(min(self.max_cells, 2**32 - 1)), max_np, 1)
        p.cell_cap = cap
        return p


def cost_hint(rates: Sequence[Sequence[float]], inits: Optional[Sequence[Dict[int, int]]] = None) -> List[float]:
    """A rough relative cost per replicate of each parameter set, for RunSpec.set_cost_hint: events to grow
    a birth-death population scale with (b1 + d1) / (b1 - d1) (net growth per event of the N+ type), and
    an event costs more as copy numbers grow (2k segregation bits beyond the first Philox words, cells
    beyond the LDS bins): factor 1 + mean initial copy number / 16. Only the ORDER of the values matters
    (longest-processing-time starts); a poor estimate costs speed, never results."""
    out = []
    for s, r in enumerate(rates):
        b1, d1 = float(r[1]), float(r[3])
        events = (b1 + d1) / max(b1 - d1, 0.05)
        k = 1.0
        if inits is not None:
            h = {int(key): int(v) for key, v in inits[s].items() if int(key) > 0}
            if h:
                k = sum(key * v for key, v in h.items()) / max(1, sum(h.values()))
        out.append(events * (1.0 + k / 16.0))
    return out


def summaries_array(n: int) -> np.ndarray:
    return np.zeros(n, dtype=SUMMARY_DTYPE)


def totals_array(n_sets: int) -> np.ndarray:
    return np.zeros(n_sets, dtype=TOTALS_DTYPE)


def as_ptr(arr: np.ndarray):
    return C.c_void_p(arr.ctypes.data)
