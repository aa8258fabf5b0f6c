"""Throughput of the engine on every BASELINE.json config shape that runs on one GPU
(configs[1..4]; C4 and C5 as the per-GPU shard of their 8-GPU runs). Development/measurement tool.
c3s = the metric's fixed-total C3 reading (2^20 replicates over PROBE_GPUS GPUs), shard PROBE_RANK.
Usage: [PROBE_FLAGS=0x20] [PROBE_KMAX=256] [PROBE_SEG=s] [PROBE_RANK=r] [PROBE_GPUS=8] python tools/probe_configs.py [c2 c3 c4 c5 c3s]"""
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402


def c4_shard(rank=0, gpus=8, interleaved=None):
    """ABC sweep: 1024 (b1, d, k0) sets x 4096 replicates; rank `rank` of `gpus`: global
    ids rank, rank + gpus, ... (interleaved, the default: every GPU gets every set) or the contiguous
    block of 128 sets (PROBE_SHARD=contiguous: one initial copy number per GPU, unbalanced)."""
    rates, inits = [], []
    for i in range(1024):
        s = 1.0 + 1.5 * (i % 16) / 15.0
        d = 0.7 * ((i // 16) % 8) / 7.0
        k0 = 1 << (i // 128)
        rates.append((1.0, s, d, d))
        inits.append({k0: 1})
    per = 4096
    n = 1024 * per // gpus
    if interleaved is None:
        interleaved = os.environ.get("PROBE_SHARD", "interleaved") == "interleaved"
    first, stride = (rank, gpus) if interleaved else (rank * n, 1)
    hint = abi.cost_hint(rates, inits) if os.environ.get("PROBE_COST_HINT", "1") == "1" else None
    return abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=rates, reps_per_set=per, first_replicate=first,
                       n_replicates=n, replicate_stride=stride, max_cells=10_000, init_per_set=inits,
                       hist_bins=1025, flags=0, set_cost_hint=hint)


def c4_subset(ex, gpus=8):
    """The sets of one initial copy number k0 = 2^ex of the C4 sweep (128 sets), with the replicates per set one
    rank of `gpus` holds: which sets set the 8-GPU shard's critical path (tools/c4_sub.py)."""
    rates, inits = [], []
    for i in range(ex * 128, ex * 128 + 128):
        s = 1.0 + 1.5 * (i % 16) / 15.0
        d = 0.7 * ((i // 16) % 8) / 7.0
        rates.append((1.0, s, d, d))
        inits.append({1 << ex: 1})
    per = 4096 // gpus
    return abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=rates, reps_per_set=per, n_replicates=128 * per,
                       max_cells=10_000, init_per_set=inits, hist_bins=1025, flags=0,
                       set_cost_hint=abi.cost_hint(rates, inits))


def c5_shard(rank=0, gpus=8):
    n = 262_144 // gpus
    return abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.9, 0.9),), reps_per_set=262_144,
                       first_replicate=rank * n, n_replicates=n, max_cells=1_000_000, max_time=1000.0,
                       init={1: 1000}, hist_bins=1025, flags=0, big_cap=int(os.environ.get("PROBE_BIG_CAP", 1 << 16)))


def c3_strong_shard(rank=0, gpus=8):
    """The metric's fixed-total reading of C3: 2^20 replicates in total, rank `rank` of `gpus` runs the contiguous
    ids [rank 2^20 / gpus, (rank + 1) 2^20 / gpus) (bench.py --scaling strong)."""
    total = 1 << 20
    first, last = rank * total // gpus, (rank + 1) * total // gpus
    return abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), reps_per_set=total,
                       first_replicate=first, n_replicates=last - first, max_cells=10_000, hist_bins=1025, flags=0)


CONFIGS = {
    "c2": lambda: abi.RunSpec(seed=42, n_replicates=65536, max_cells=10_000, flags=0),
    "c3": lambda: abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),),
                              n_replicates=1 << 20, max_cells=10_000, flags=0),
    "c4": c4_shard,
    "c5": c5_shard,
    "c3s": c3_strong_shard,
}


def main():
    for name in sys.argv[1:] or list(CONFIGS):
        gpus = int(os.environ.get("PROBE_GPUS", "8"))  # the layout the shard belongs to (1: the whole config)
        spec = CONFIGS[name](int(os.environ.get("PROBE_RANK", "0")), gpus) if name in ("c4", "c5", "c3s") else CONFIGS[name]()
        spec = dataclasses.replace(spec, flags=spec.flags | int(os.environ.get("PROBE_FLAGS", "0"), 0),
                                   bin_kmax=int(os.environ.get("PROBE_KMAX", "0")), _keep=[])
        if "PROBE_SEG" in os.environ:  # another segregation rule (abi.SEG_*) on the same shape
            spec = dataclasses.replace(spec, segregation=int(os.environ["PROBE_SEG"]), _keep=[])
        t0 = time.time()
        ctx = engine.Context(spec)
        reps = 1 if name == "c5" else 2
        for _ in range(reps):
            t1 = time.time()
            ctx.launch()
            s_ms, h_ms = ctx.sync()
            wall = time.time() - t1
        res = ctx.download()
        t = res.totals
        ev = int(t["events"].sum())
        print(json.dumps({"config": name, "flags": spec.flags, "bin_kmax": spec.bin_kmax, "replicates": spec.n_replicates, "events": ev, "stepper_ms": s_ms,
                          "hist_ms": h_ms, "wall_ms": wall * 1e3, "events_per_s_kernel": ev / (s_ms * 1e-3),
                          "events_per_s_wall": ev / wall, "geometry": ctx.geometry(), "instance": ctx.instance(),
                          "stops": t["stop_reasons"].sum(axis=0).tolist(), "errors": int(t["errors"].sum()),
                          "setup_s": t1 - t0}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
