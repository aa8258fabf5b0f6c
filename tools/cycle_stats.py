"""Loop-section cycle counters of the bin stepper over one launch (development tool): where a wave's time
goes (replicate boundary, N- fast-forward, full event), per wave-iteration and per event. Needs a library
built with -DECDNA_CYCLE_STATS (EXTRA=-DECDNA_CYCLE_STATS bash tools/ab_build.sh WORKTREE cyc), selected
with ECDNA_SSA_LIB. Usage: [PROBE_KMAX=K] python tools/cycle_stats.py [c2|c3|c4|c5|c4k<ex>|c3s<G>] (C4 and C5: the 8-GPU rank-0 shard;
c4k<ex>: its sets of k0 = 2^ex; c3s<G>: the rank-0 shard of C3's fixed total over G GPUs, bench.py --scaling strong)"""
import ctypes as C
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_configs  # noqa: E402

KMAX = {"c2": 32, "c3": 32, "c4": 64, "c5": 64}
NAMES = ["cyc_boundary", "cyc_ff", "cyc_full", "iters", "ff_entries", "ff_steps", "full_lanes", "cyc_kernel",
         "f_prop_stop", "f_philox_channel", "f_pick", "f_segregation", "f_checks", "f_time_step", "f_updates"]


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c5"
    if name.startswith("c3s"):  # c3s<G>: bench.py --scaling strong's rank-0 shard at G GPUs
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        from ecdna_evo_amd import shard
        first, n = shard.shard_range(0, int(name[3:]), 1 << 20)
        spec = bench.workload_spec(first, n, 1 << 20)
        name = "c3"
    elif name.startswith("c4k"):  # c4k<ex>: the C4 shard's sets of k0 = 2^ex (probe_configs.c4_subset)
        spec = probe_configs.c4_subset(int(name[3:]))
    else:
        spec = probe_configs.CONFIGS[name](0, 8) if name in ("c4", "c5") else probe_configs.CONFIGS[name]()
    kmax = int(os.environ.get("PROBE_KMAX", KMAX.get(name, 64)))
    spec = dataclasses.replace(spec, flags=abi.FLAG_BIN_STORE, bin_kmax=kmax, _keep=[])
    lib = engine.lib()
    readers = []
    for sym in ("ecdna_dev_cycle_stats", "ecdna_dev_cycle_stats_ilp"):
        fn = getattr(lib, sym)
        fn.argtypes = [C.POINTER(C.c_ulonglong)]
        readers.append(fn)
    ctx = engine.Context(spec)
    buf = (C.c_ulonglong * 16)()
    for fn in readers:
        fn(buf)
    ctx.launch()
    ms, _ = ctx.sync()
    tot = [0] * 16
    for fn in readers:
        fn(buf)
        tot = [a + int(b) for a, b in zip(tot, buf)]
    d = dict(zip(NAMES, tot))
    ev = int(ctx.download().totals["events"].sum())
    it = max(d["iters"], 1)
    cyc = d["cyc_boundary"] + d["cyc_ff"] + d["cyc_full"]
    print(json.dumps({"config": name, "ms": ms, "events": ev, "geometry": ctx.geometry(), **d,
                      "per_iter": {k: round(d[k] / it, 2) for k in NAMES[:3] + NAMES[4:7] + NAMES[8:]},
                      "share": {k: round(d[k] / max(cyc, 1), 3) for k in NAMES[:3]},
                      "ff_steps_per_entry": round(d["ff_steps"] / max(d["ff_entries"], 1), 2)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
