#!/usr/bin/env python3
"""Benchmark: Gillespie reaction-events/s of the MI355X SSA engine (BASELINE.json metric).

Workload (N=1 line = BASELINE.json configs[2], "C3"): 2^20 independent replicates per GPU of the
reference's birth-death process (b0=1, b1=1.5, d0=d1=0.3, Binomial segregation, initial {1: 1},
stop at 1e4 cells or t = floor(log2(1e4)+4) = 17 years), seed 42. Weak scaling: rank g runs the
global replicate ids [g*2^20, (g+1)*2^20) — per-GPU work is fixed as N grows — and the only
collective is one all-reduce of the copy-number histogram + totals per step (RCCL over xGMI).

One step = one full run of the hot path on every GPU: zero outputs, the persistent SSA stepper
kernel over all 2^20 replicates, the histogram kernel, and (N>1) the all-reduce. Inputs are
resident in HBM before the timed region.

Cell store (--store): "bins" (default, ECDNA_FLAG_BIN_STORE: per-replicate copy-number counters in
LDS) or "rows" (one u16 per cell in HBM in the reference's swap_remove order). Both
simulate the same process and count the same events; each is bit-exact with its oracle restatement.

`--scaling strong` is the metric's fixed-total reading of C3: 2^20 replicates in total, rank g of N runs the
contiguous ids [g 2^20 / N, (g+1) 2^20 / N) — the reference's fixed `runs` replicates over its worker pool
(src/main.rs:212-224). At N=1 it is the same run as the weak line.

Other BASELINE.json configs (--workload; the default line above is C3): c2 = 65,536 pure-birth replicates
to 1e4 cells (configs[1]); c4 = the ABC sweep, 1024 (b1, d, k0) parameter sets x 4,096 replicates
(configs[3]); c5 = 262,144 birth-death turnover replicates from 1,000 cells to 1e6 cells or t = 1000
(configs[4]). These are strong-scaling runs of a fixed total, sharded over the ranks by interleaved
global ids (rank g of G runs ids g, g+G, ...: every GPU gets the same mix of parameter sets,
DESIGN.md §7).

Extra JSON fields:
  roofline      — the stepper kernel against HBM: algorithmic bytes per launch over
                  its average duration (HIP events on the launch stream), vs 8 TB/s; `traffic` =
                  measured HBM bytes per launch from the committed rocprofv3 PMC summary, if present;
                  rows: `hbm_requests` = the same kernel against the random-access request ceiling that
                  bounds it (requests per event from the PMC summary x events/s, vs the calibrated
                  random read-modify-write rate); bins: `valu_issue` = its vector instructions per
                  second against the chip's wave64 VALU issue rate, which bounds it (instructions per
                  event from the PMC summary x events/s).
  cpu_baseline  — the reference-semantics CPU restatement (oracle/, ChaCha8 + first-reaction +
                  BTPE, "port") on a bounded sample of the same workload, rank 0 at N=1 only.
"""
import argparse
import dataclasses
import json
import os
import sys
import time
from typing import Optional

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "ecdna-evo_amd"))

import torch  # noqa: E402  (first: one HIP runtime for torch and the engine)
import torch.distributed as dist  # noqa: E402

from ecdna_evo_amd import abi, engine, shard  # noqa: E402

METRIC = "Gillespie reaction-events/sec at 2^20 replicates, 1/2/4/8 MI355X"
REPS_PER_GPU = 1 << 20
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
# algorithmic bytes per event: per-cell u16 row with swap_remove
B_PROLIF_EVEN, B_PROLIF_UNEVEN, B_DEATH_NPLUS = 10, 8, 6
B_SUMMARY = 88
# wave64 VALU instructions the chip can issue per second: 256 CUs x 4 SIMD-32 x 2.4 GHz / 2 cycles
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2


def valu_measured_ceilings():
    """Measured issue rates (wave-instr/s, whole chip) of single-opcode streams at full occupancy
    (tools/valu_probe.hip -> profiles/r01g_valu_issue_probe.txt): the 2-cycle class (VOP2 and/or/xor/
    add/sub/lshrrev/mov with VGPR operands, f32 add/mul) and the 4-cycle class (VOP3 encodings, SGPR
    operands, lshlrev, bfe, 24/32-bit multiplies, conversions, f64 add/mul)."""
    rates = {}
    try:
        with open(os.path.join(REPO, "profiles", "r01g_valu_issue_probe.txt")) as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 2 and parts[-1] == "chip":
                    rates[parts[0]] = float(parts[-3])
    except Exception:
        pass
    two = [rates[k] for k in ("and_b32", "xor_v", "add_u32_v", "mov_b32") if k in rates]
    four = [rates[k] for k in ("add_u32", "lshl_add_u32", "bfe_u32", "add_f64", "mul_f64", "cvt_f64_u32") if k in rates]
    return (sum(two) / len(two) if two else None, sum(four) / len(four) if four else None)


# bin store tunable: copy numbers 1..32 as LDS counters (4 groups: a shorter pick scan; at C3 a
# picked cell has k > 32 with probability 0.6 %, those go to the large-k row). C3: 125 ms vs 132 ms with 64.
BENCH_BIN_KMAX = 32


# bin_kmax per workload (measured). K is part of the draw mapping (it fixes the canonical cell order,
# DESIGN.md §3.3), so it is a property of the WORKLOAD, never of the GPU count: the same replicate ids give the same
# results on 1, 2, ..., 8 GPUs. K = 32 where the pick scan dominates (C3 issue-bound:
# 5 % faster than 64; C2), K = 64 where copy numbers spread (C4: k0 up to 128, 8-GPU makespan 156 -> 131 ms; C5: 1e6
# cells). C5 is the 8-GPU config (BASELINE.json configs[4]): its 8-, 4- and 2-GPU shards run faster at K = 64 (9.9
# against 10.9 s, 13.0 against 14.0, 15.5 against 16.2; profiles/r04s_c5_kmax.txt, r04u_kmax_rule.txt) and the whole
# run on one GPU slower (28.8 against 22.6 s); until round 5 the one-GPU run took K = 32, which made its results
# differ from the shards' seed for seed.
WORKLOAD_KMAX = {"c2": 32, "c3": BENCH_BIN_KMAX, "c4": 64, "c5": 64}
# C4 shards split by initial copy number (shard.k0_split): the sets of k0 = 128 on a K = 256 context,
# concurrently with the rest on K = 64, the two persistent grids capped at these workgroup counts. The split is part of
# the workload (which K a replicate runs at), at every GPU count; the caps are speed only (results never depend on the
# grid), measured for 1, 2, 4 and 8 GPUs (rank-0 shards, same box: whole K = 64 -> split 727 -> 638 ms at 1 GPU,
# 372 -> 322 at 2, 189 -> 185 at 4; at 8 the eight shards' makespan 124 -> 108 ms; profiles/r05_c4_split.txt); other
# counts take those of the nearest measured count below.
C4_SPLIT_K0, C4_SPLIT_KMAX = 128, 256
C4_SPLIT_CAPS = {1: (496, 528), 2: (496, 528), 4: (384, 512), 8: (336, 624)}


def c4_split_caps(n_gpus: int):
    """(narrow, heavy) workgroup caps of the C4 k0 split for a sweep spread over n_gpus GPUs."""
    return C4_SPLIT_CAPS[max(g for g in C4_SPLIT_CAPS if g <= max(1, n_gpus))]


def default_kmax(workload: str, n: int = 0) -> int:
    """The workload's bin store K (the same for any shard size n: K is part of the draw mapping)."""
    return WORKLOAD_KMAX[workload]


def workload_spec(first: int, n: int, total: int, seed: int = 42, device: int = 0, store: str = "bins",
                  bin_kmax: Optional[int] = None, workload: str = "c3", stride: int = 1,
                  max_cells: Optional[int] = None) -> abi.RunSpec:
    """Replicates first, first + stride, ... (n of them) of the workload's `total` (SURVEY.md §8d shapes);
    bin_kmax None = the workload's default for n replicates (default_kmax); max_cells None = the workload's (rehearsals of
    the multi-rank paths shrink it, tests/test_gpu_bench_dist.py)."""
    if bin_kmax is None:
        bin_kmax = default_kmax(workload, n)
    common = dict(seed=seed, first_replicate=first, n_replicates=n, replicate_stride=stride, hist_bins=1025,
                  flags=abi.FLAG_BIN_STORE if store == "bins" else 0, device=device)
    if workload == "c3":
        d = dict(process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), reps_per_set=total, max_cells=10_000)
    elif workload == "c2":
        d = dict(process=abi.PURE_BIRTH, rates=((1.0, 1.0, 0.0, 0.0),), reps_per_set=total, max_cells=10_000)
    elif workload == "c4":  # b1 = b0 * s (16 values in [1, 2.5]), d0 = d1 = d (8 values in [0, 0.7]), k0 = 1 .. 128
        rates, inits = [], []
        for i in range(1024):
            sel, dd = 1.0 + 1.5 * (i % 16) / 15.0, 0.7 * ((i // 16) % 8) / 7.0
            rates.append((1.0, sel, dd, dd))
            inits.append({1 << (i // 128): 1})
        d = dict(process=abi.BIRTH_DEATH, rates=rates, reps_per_set=total // 1024, max_cells=10_000,
                 init_per_set=inits, set_cost_hint=abi.cost_hint(rates, inits))  # costly sets start first
    elif workload == "c5":
        # the large-k row holds at most 2^16 cells (128 KB per replicate instead of cell_cap's 2 MB, so the
        # 262,144 replicates fit in HBM in one chunk)
        d = dict(process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), reps_per_set=total, max_cells=1_000_000,
                 max_time=1000.0, init={1: 1000}, big_cap=1 << 16 if store == "bins" else 0)
    else:
        raise ValueError(workload)
    if max_cells is not None:
        d["max_cells"] = max_cells
    return abi.RunSpec(segregation=abi.SEG_BINOMIAL, bin_kmax=bin_kmax if store == "bins" else 0, **common, **d)


# --workload: (replicates: per GPU for the weak-scaling C3 line, total otherwise; description)
WORKLOADS = {
    "c3": (REPS_PER_GPU, "C3 (BASELINE.json configs[2]): 2^20 replicates/GPU, birth-death b0=1 b1=1.5 d0=d1=0.3, "
                         "binomial segregation, init {1:1}, stop 1e4 cells or t=17, seed 42"),
    "c2": (65_536, "C2 (BASELINE.json configs[1]): 65,536 replicates in total, pure birth b=1, binomial "
                   "segregation, init {1:1}, stop 1e4 cells or t=17, seed 42"),
    "c4": (4_194_304, "C4 (BASELINE.json configs[3]): ABC sweep, 1024 (b1, d, k0) sets x 4,096 replicates = "
                      "4,194,304 in total, stop 1e4 cells or t=17, seed 42"),
    "c5": (262_144, "C5 (BASELINE.json configs[4]): 262,144 replicates in total, birth-death turnover b=1 d=0.9, "
                    "binomial segregation, init {1:1000}, stop 1e6 cells or t=1000, seed 42"),
}


def algorithmic_bytes(words, n_reps: int, init_cells: int = 1) -> int:
    """words: one ecdna_totals_t as 16 u64 (replicates, events, events_by_type[4], uneven, ...)."""
    uneven = int(words[6])
    even = int(words[2 + abi.EV_PROLIF_NPLUS]) - uneven
    return (B_PROLIF_EVEN * even + B_PROLIF_UNEVEN * uneven + B_DEATH_NPLUS * int(words[2 + abi.EV_DEATH_NPLUS])
            + n_reps * (2 * init_cells + B_SUMMARY))


# the sources that decide the stepper's instruction stream: a committed PMC summary describes THIS build only
# when its recorded digest of them matches (tools/pmc_summary.py stamps it)
KERNEL_SOURCES = ("ecdna-evo_amd/csrc/ssa_kernels.hip", "ecdna-evo_amd/csrc/ssa_device.hpp",
                  "ecdna-evo_amd/csrc/ssa_launch.h", "ecdna-evo_amd/csrc/ssa_logtab.h",
                  "ecdna-evo_amd/csrc/ssa_api.cpp", "ecdna-evo_amd/Makefile")


def kernel_sources_digest() -> str:
    import hashlib

    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(REPO, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read() + b"\0")
    return h.hexdigest()


def load_pmc(store: str):
    """The committed rocprofv3 PMC summary of the stepper on this workload (profiles/pmc_c3[_bins].json),
    or {} when it was measured on other kernel sources than the ones built here (its counters would not
    describe this build)."""
    try:
        with open(os.path.join(REPO, "profiles", "pmc_c3_bins.json" if store == "bins" else "pmc_c3.json")) as f:
            pmc = json.load(f)
    except Exception:
        return {}
    if pmc.get("kernel_sources_sha256") != kernel_sources_digest():
        return {"stale": True, "round": pmc.get("round"), "git_head": pmc.get("git_head")}
    return pmc


def usable_cores() -> int:
    """Host cores this process may use, as rayon's default pool counts them (the reference's replicate
    loop, src/main.rs:221-224): the CPU affinity set, capped by a cgroup v2 CPU quota if one is set."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except Exception:
        pass
    return max(1, n)


def cores_basis() -> str:
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota = f.read().strip()
    except Exception:
        quota = "n/a"
    return f"usable cores = min(CPU affinity set {aff}, cgroup v2 cpu.max '{quota}'); os.cpu_count() {os.cpu_count()}"


def rmw_ceiling():
    """Random 2-B read-modify-write pairs/s the chip sustains (tools/rmw_shapes.hip, 4 GiB buffer,
    best lane count; profiles/r01d_access_microbench.jsonl)."""
    best = None
    try:
        with open(os.path.join(REPO, "profiles", "r01d_access_microbench.jsonl")) as f:
            for line in f:
                d = json.loads(line)
                if d.get("shape") == "rmw_u16":
                    best = max(best or 0.0, d["ops_per_s"])
    except Exception:
        pass
    return best


@dataclasses.dataclass
class RankParts:
    weak: bool             # the metric's weak-scaling C3 line
    c3_strong: bool        # C3's fixed-total reading
    total: int             # replicates over all ranks
    reps: int              # replicates on this rank
    spec: abi.RunSpec      # this rank's shard
    parts: list            # [(RunSpec, local offset)]: the contexts the rank launches (C4: split by k0)


def rank_parts(workload: str, n_gpus: int, rank: int, scaling: str = "weak", store: str = "bins",
               bin_kmax: Optional[int] = None, k0_split: str = "auto", total: Optional[int] = None,
               reps_per_gpu: int = REPS_PER_GPU, max_cells: Optional[int] = None, device: int = 0,
               refdraws: bool = False) -> RankParts:
    """What rank `rank` of `n_gpus` runs for a workload: its shard of global replicate ids and the engine contexts
    it launches. Which K (draw mapping) a replicate runs at depends on its id and the workload only,
    never on n_gpus, so every GPU count gives the same per-replicate results (tests/test_bench_workloads.py)."""
    weak = workload == "c3" and scaling == "weak"
    c3_strong = workload == "c3" and scaling == "strong"
    if weak:  # the metric's line: 2^20 replicates per GPU, rank g owns ids [g 2^20, (g+1) 2^20)
        reps = reps_per_gpu
        total = reps * n_gpus
        first, n = shard.weak_range(rank, reps)
        stride = 1
    elif c3_strong:  # the metric's fixed-total reading: 2^20 in total, rank g owns a contiguous 1/N of them
        total = total or REPS_PER_GPU
        first, n = shard.shard_range(rank, n_gpus, total)
        stride = 1
        reps = n
    else:  # a fixed total over the ranks, interleaved ids
        total = total or WORKLOADS[workload][0]
        first, n, stride = shard.interleaved_range(rank, n_gpus, total)
        reps = n
    spec = workload_spec(first, n, total, device=device, store=store, bin_kmax=bin_kmax, workload=workload,
                         stride=stride, max_cells=max_cells)
    if refdraws:
        spec = dataclasses.replace(spec, flags=spec.flags | abi.FLAG_REFERENCE_DRAWS, _keep=[])
    split_caps = c4_split_caps(n_gpus) if (workload == "c4" and k0_split == "auto" and store == "bins" and
                                           bin_kmax is None) else None
    parts = shard.k0_split(spec, C4_SPLIT_K0, C4_SPLIT_KMAX, split_caps) if split_caps else [(spec, 0)]
    return RankParts(weak, c3_strong, total, reps, spec, parts)


def cpu_baseline(threads: int, workload: str = "c3"):
    """Reference-semantics CPU path (oracle compat mode) timed on a bounded sample of the workload: its
    first replicates (C4: ids spread evenly over the id range, so the sample spans every set)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # test infrastructure: the CPU baseline only

    total = WORKLOADS[workload][0]

    def sample(n, mode):
        stride = max(1, total // n) if workload == "c4" else 1  # C4: evenly spread over the 1024 sets
        spec = workload_spec(0, n, total, workload=workload, stride=stride)
        t0 = time.time()
        r = oracle.run(spec, mode=mode, n_threads=threads)
        return int(r.totals["events"].sum()), max(time.time() - t0, 1e-3)

    n0 = 16 if workload == "c5" else 1024  # C5: ~2e7 events per replicate
    _, dt = sample(n0, "compat")
    target_s = float(os.environ.get("ECDNA_BENCH_CPU_SECONDS", "10"))
    n = int(min(total, max(n0, n0 * target_s / dt)))
    ev, dt = sample(n, "compat")
    # for information: the same sample through the engine's own draw mapping on the CPU
    n_ph = max(n0, n // 2)
    ev_ph, dt_ph = sample(n_ph, "philox")
    what = "C3 shape, replicates 0..{0} of 2^20".format(n - 1) if workload == "c3" else \
        f"{workload.upper()} shape, {n} of its {total} replicates"
    return {"value": ev / dt, "unit": "events/s", "cores": threads, "kind": "port", "cores_basis": cores_basis(),
            "sample": f"{what} ({ev} events, {dt:.1f} s wall), "
                      f"oracle compat mode (ChaCha8 streams seed*10+i, first-reaction, BTPE), "
                      f"{threads} threads",
            "philox_mode_value": ev_ph / dt_ph,
            "philox_mode_sample": f"replicates 0..{n_ph - 1}, oracle philox mode (the engine's draw mapping, "
                                  f"direct method, popcount binomial), {threads} threads"}


def main():
    # exactly one JSON line on stdout: library chatter (e.g. RCCL's version banner, printed to fd 1 when a
    # communicator is created) goes to stderr; the result line is written to the saved stdout
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reps-per-gpu", type=int, default=REPS_PER_GPU)
    ap.add_argument("--store", choices=("bins", "rows"), default="bins")
    ap.add_argument("--bin-kmax", type=int, choices=(32, 64, 256), default=None,
                    help="bin store K (default: the workload's, WORKLOAD_KMAX)")
    ap.add_argument("--dump-hist", default="", help="rank 0 saves the reduced histogram and totals (.npz)")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3",
                    help="BASELINE.json config; c3 (default) is the metric's weak-scaling line")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="c3 only: weak (default) = 2^20 replicates per GPU; strong = 2^20 replicates in total, "
                         "contiguous shards of 2^20 / N (the reference's fixed `runs` over its worker pool, "
                         "src/main.rs:212-224)")
    ap.add_argument("--total", type=int, default=None,
                    help="rehearsal only: replicates in total for the strong-scaling workloads (c2/c4/c5)")
    ap.add_argument("--max-cells", type=int, default=None, help="rehearsal only: override the workload's cell cap")
    ap.add_argument("--k0-split", choices=("auto", "off"), default="auto",
                    help="c4, bin store: run the k0 = 128 sets of the shard on a concurrent K = 256 context (auto, any "
                         "GPU count), or the whole shard on one K = 64 context (off; the k0 = 128 replicates then "
                         "run at K = 64 and differ seed for seed)")
    ap.add_argument("--draws", choices=("philox", "reference"), default="philox",
                    help="reference: the Rust reference's own draws seed for seed (ECDNA_FLAG_REFERENCE_DRAWS, "
                         "DESIGN.md §4.1; row store only): the seed-for-seed mode's throughput, not the metric's")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # under torchrun (even at one rank) the RCCL path runs: process group, all-reduce, barriers
    distributed = "RANK" in os.environ and "MASTER_ADDR" in os.environ
    # rehearsal knobs for a one-GPU box (tests/test_gpu_bench_dist.py): every rank on cuda:0, reduced over
    # gloo (RCCL refuses two ranks on one device); the driver's runs use neither
    backend = os.environ.get("ECDNA_BENCH_BACKEND", "nccl")
    if os.environ.get("ECDNA_BENCH_ONE_DEVICE") == "1":
        local = 0
    if distributed:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend=backend)
    else:
        torch.cuda.set_device(0)
    n_gpus = world
    if args.scaling == "strong" and args.workload != "c3":
        ap.error("--scaling strong applies to c3 (the other workloads are fixed totals already)")
    refdraws = args.draws == "reference"
    if refdraws and args.store != "rows":
        ap.error("--draws reference runs on the row store only (--store rows)")
    rp = rank_parts(args.workload, n_gpus, rank, scaling=args.scaling, store=args.store, bin_kmax=args.bin_kmax,
                    k0_split=args.k0_split, total=args.total, reps_per_gpu=args.reps_per_gpu, max_cells=args.max_cells,
                    device=local if distributed else 0, refdraws=refdraws)
    weak, c3_strong, total, reps, spec, parts = rp.weak, rp.c3_strong, rp.total, rp.reps, rp.spec, rp.parts
    n_sets = len(spec.rates)
    ctxs = [engine.Context(sp) for sp, _ in parts]
    ctx = ctxs[0]
    hist = torch.zeros(n_sets * spec.hist_bins, dtype=torch.int64, device="cuda")
    tot = torch.zeros(n_sets * 16, dtype=torch.int64, device="cuda")
    part_out = []
    if len(ctxs) == 1:
        ctx.set_outputs(hist.data_ptr(), tot.data_ptr())
    else:  # each part writes its own outputs; the step sums them
        for c in ctxs:
            h_p, t_p = torch.zeros_like(hist), torch.zeros_like(tot)
            c.set_outputs(h_p.data_ptr(), t_p.data_ptr())
            part_out.append((h_p, t_p))
    torch_stream = torch.cuda.Stream()
    torch.cuda.set_stream(torch_stream)  # torch ops and the engine's kernels share this stream
    stream = torch_stream.cuda_stream
    part_streams = [torch.cuda.Stream() for _ in ctxs] if len(ctxs) > 1 else []

    tot_local = torch.zeros_like(tot)

    def step():
        if len(ctxs) == 1:
            ctx.launch(stream)
        else:  # the parts run concurrently, each on its own stream, joined on the step's stream
            start = torch.cuda.Event()
            start.record(torch_stream)
            for c, s in zip(ctxs, part_streams):
                s.wait_event(start)
                c.launch(s.cuda_stream)
            for s in part_streams:
                torch_stream.wait_stream(s)
            torch.add(part_out[0][0], part_out[1][0], out=hist)
            torch.add(part_out[0][1], part_out[1][1], out=tot)
        tot_local.copy_(tot)  # this GPU's totals, before the reduction
        if distributed:
            shard.reduce_outputs(hist, tot)

    def sync_all():
        """(stepper ms, histogram ms) of the step: the parts' longest (they run concurrently)"""
        ms = [c.sync() for c in ctxs]
        return max(m[0] for m in ms), max(m[1] for m in ms)

    for _ in range(args.warmup):
        step()
        sync_all()
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms, hist_ms = [], []
    for _ in range(args.steps):
        step()
        s_ms, h_ms = sync_all()
        kernel_ms.append(s_ms)
        hist_ms.append(h_ms)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    local_words = tot_local.cpu().numpy().reshape(n_sets, 16).sum(axis=0)  # per-set totals, summed
    local_events = int(local_words[1])
    local_alg = algorithmic_bytes(local_words, reps, init_cells=1000 if args.workload == "c5" else 1)
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    ev = torch.tensor([local_events], dtype=torch.int64, device="cuda")
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(ev)
    elapsed = float(t.item())
    events_per_step = int(ev.item())
    # the all-reduced histogram must account for every cell of every replicate
    tot_sets = tot.cpu().numpy()
    tot_host = tot_sets.reshape(n_sets, 16).sum(axis=0)
    assert int(tot_host[0]) == total, f"all-reduced totals count {int(tot_host[0])} replicates, expected {total}"
    assert int(tot_host[1]) == events_per_step
    stop_reasons = {abi.STOP_NAMES[i]: int(tot_host[9 + i]) for i in range(6)}
    errors = int(tot_host[15])
    # the workloads are sized so that no replicate hits a capacity (cell_cap, C5's big_cap) or overflow error:
    # a replicate cut short by one would make the events/s line count a different process
    assert errors == 0, f"{errors} replicates stopped with an error (stop reasons {stop_reasons})"

    if rank == 0 and args.dump_hist:
        import numpy as np

        np.savez(args.dump_hist, hist=hist.cpu().numpy(), totals=tot_sets)
    if rank == 0:
        avg_kernel_s = sum(kernel_ms) / len(kernel_ms) * 1e-3
        achieved = local_alg / avg_kernel_s / 1e9
        # (the committed PMC summaries: C3, philox; the strong reading's one-GPU run is the same launch)
        pmc = load_pmc(args.store) if args.workload == "c3" and n_gpus == 1 and not refdraws else {}
        traffic = pmc.get("hbm_bytes_per_launch")
        kernel_eps = local_events / avg_kernel_s
        transactions = None
        issue = None
        if args.store == "bins" and "valu_insts_per_event" in pmc:
            per_event = pmc["valu_insts_per_event"]
            two, four = valu_measured_ceilings()
            issue = {
                "valu_wave_insts_per_event": per_event,
                "per_s": per_event * kernel_eps,
                "peak_per_s": VALU_ISSUE_PEAK,
                "frac": per_event * kernel_eps / VALU_ISSUE_PEAK,
                "measured_2cycle_class_per_s": two,
                "measured_4cycle_class_per_s": four,
                "frac_of_measured_4cycle_class": per_event * kernel_eps / four if four else None,
                # scalar and LDS instructions take issue slots too (round 6: an added s_mov costs 0.6 of an added
                # v_xor at C3, profiles/r06n_marginal_valu_salu.txt)
                "salu_wave_insts_per_event": (pmc["salu_wave_insts_per_wave_event"] / 64.0
                                              if "salu_wave_insts_per_wave_event" in pmc else None),
                "lds_wave_insts_per_event": (pmc["lds_wave_insts_per_wave_event"] / 64.0
                                             if "lds_wave_insts_per_wave_event" in pmc else None),
                "note": "the bin store keeps every common-case event in LDS and registers, so the stepper is "
                        "bounded by instruction issue, not HBM (DESIGN.md §5): vector instructions first, scalar "
                        "control next; wave-instructions per event from the committed PMC summary (SQ_INSTS_VALU / "
                        "_SALU / _LDS); the spec peak assumes 2 cycles per wave64 instruction, which only the VOP2 "
                        "logic/add/mov class reaches on gfx950 — most of the stepper's instructions are in the "
                        "measured 4-cycle class (tools/valu_probe.hip)",
            }
        if args.store == "rows" and "read_requests_per_event" in pmc:
            per_event = pmc["read_requests_per_event"] + pmc["write_requests_per_event"]
            ceiling = rmw_ceiling()
            transactions = {
                "requests_per_event": per_event,
                "per_s": per_event * kernel_eps,
                "random_rmw_ceiling_per_s": 2 * ceiling if ceiling else None,
                "frac": per_event * kernel_eps / (2 * ceiling) if ceiling else None,
                "note": "random 2-B cell accesses move whole 64-B read / 32-B write requests, so the "
                        "stepper is bounded by HBM request rate, not bytes (DESIGN.md §5); requests per "
                        "event from the committed PMC summary, ceiling from tools/rmw_shapes.hip",
            }
        cpu = None
        if n_gpus == 1 and not args.no_cpu_baseline:
            # every usable core, as the reference's rayon pool (src/main.rs:221-224)
            threads = int(os.environ.get("ECDNA_BENCH_CPU_THREADS", "0")) or usable_cores()
            cpu = cpu_baseline(threads, args.workload)
        lanes = sum(c.geometry()[1] for c in ctxs)
        instance = ctx.instance()  # the kernel instance timed (auto rules of ecdna_ssa_ctx_create)
        line = {
            "metric": METRIC if args.workload == "c3" else f"Gillespie reaction-events/sec, {args.workload.upper()}",
            "value": events_per_step * args.steps / elapsed,
            "unit": "events/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if weak else "strong",
            "vs_baseline": None,
            # integer cell/counter work plus the reference's f32 propensities (src/main.rs:67, 139) and f32 time step;
            # the channel's cumulative sums and the engine's clock in f64 (draw mapping v8)
            "dtype": "u16+f32" if refdraws else "u16+f32 (f64 channel sums and clock)",
            "draws": "reference (ChaCha8 seed*10+i, first-reaction, BINV/BTPE, f32 time; seed for seed)"
                     if refdraws else "philox (the engine's draw mapping v8, DESIGN.md §3)",
            "store": args.store,
            "data": "synthetic",
            "config": {
                "workload": WORKLOADS[args.workload][1] if not c3_strong else
                            "C3 (BASELINE.json configs[2]), fixed total: 2^20 replicates over all GPUs, birth-death b0=1 "
                            "b1=1.5 d0=d1=0.3, binomial segregation, init {1:1}, stop 1e4 cells or t=17, seed 42",
                "cell_store": f"bins (copy-number counters in LDS, k<={spec.bin_kmax}; ECDNA_FLAG_BIN_STORE)"
                              if args.store == "bins" else "rows (u16 per cell in HBM, swap_remove order)",
                "replicates_per_gpu": reps,
                "replicates_total": total,
                "events_per_step": events_per_step,
                "stop_reasons": stop_reasons,
                "replicate_errors": errors,
                "parallelism": f"replicas{n_gpus} ({'contiguous' if args.workload == 'c3' else 'interleaved'} replicate-id shards, "
                               f"1 RCCL all-reduce of the histogram)",
                "grid_lanes": lanes,
                "instance": instance,
                "k0_split": None if len(ctxs) == 1 else {
                    "parts": [{"replicates": sp.n_replicates, "bin_kmax": sp.bin_kmax, "max_workgroups": sp.max_workgroups,
                               "instance": c.instance()} for (sp, _), c in zip(parts, ctxs)],
                    "note": f"the shard's k0 >= {C4_SPLIT_K0} sets on a K = {C4_SPLIT_KMAX} context, concurrently with "
                            "the rest (shard.k0_split, DESIGN.md §7); kernel_ms_avg is the longer part's"},
                "kernel_ms_avg": avg_kernel_s * 1e3,
                "hist_kernel_ms_avg": sum(hist_ms) / len(hist_ms),
                "kernel_events_per_s_per_gpu": kernel_eps,
            },
            "roofline": {
                # what binds the stepper: vector-instruction issue for the bin store (its events stay in LDS
                # and registers), HBM request rate for the row store; achieved / peak / frac below are the
                # contract's nominal HBM view (SURVEY.md §8d algorithmic bytes of the reference's u16-row
                # representation over the kernel's duration, vs 8 TB/s), which neither store is bound by
                "bound": "divergent_samplers" if refdraws else ("valu_issue" if args.store == "bins" else "hbm_requests"),
                "issue_frac": issue["frac"] if issue else None,
                "frac_kind": "nominal_hbm_algorithmic_bytes",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "pmc_source": None if not pmc else (
                    f"stale ({pmc.get('round')}): the committed PMC summary was measured on other kernel "
                    f"sources; counter fields omitted" if pmc.get("stale") else
                    f"profiles/pmc_c3{'_bins' if args.store == 'bins' else ''}.json, round {pmc.get('round')}, "
                    f"git {pmc.get('git_head')}, kernel sources match this build"),
                # the committed counters describe this instance only if the PMC run chose the same one
                "pmc_instance_matches": (pmc.get("instance") == instance) if pmc and not pmc.get("stale") else None,
                "hbm_requests": transactions,
                "valu_issue": issue,
            },
            "cpu_baseline": cpu,
        }
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    for c in ctxs:
        c.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
