"""Rare-block counters of the bin stepper over one launch (development tool): C3 (K = 32, default) or the
C5 rank-0 shard of the 8-GPU layout (`c5`, K = 64). Needs a library built with -DECDNA_PATH_STATS
(EXTRA=-DECDNA_PATH_STATS bash tools/ab_build.sh WORKTREE pstats), selected with ECDNA_SSA_LIB. Prints
wave-iterations, active lanes, and per rare block the fraction of wave-iterations that execute it (at
least one lane in the block). Usage: python tools/path_stats.py [c3|c5|c4k<ex>]"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_configs  # noqa: E402

workload = sys.argv[1] if len(sys.argv) > 1 else "c3"
if workload.startswith("c4k"):  # the C4 shard's sets of k0 = 2^ex (probe_configs.c4_subset), K = 64
    import dataclasses

    spec = dataclasses.replace(probe_configs.c4_subset(int(workload[3:])), flags=abi.FLAG_BIN_STORE,
                               bin_kmax=int(os.environ.get("PROBE_KMAX", "64")), _keep=[])
elif workload == "c5":
    import dataclasses

    spec = dataclasses.replace(probe_configs.c5_shard(0), flags=abi.FLAG_BIN_STORE, bin_kmax=64, _keep=[])
else:
    spec = abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=1 << 20,
                       max_cells=10_000, flags=abi.FLAG_BIN_STORE, bin_kmax=32)
lib = engine.lib()
fn = lib.ecdna_dev_path_stats
fn.argtypes = [C.POINTER(C.c_ulonglong)]
ctx = engine.Context(spec)
buf = (C.c_ulonglong * 8)()
names = ["wave_iters", "lane_iters", "boundary", "lemire_reject", "large_pick", "binomial_words", "large_row_update",
         "capacity_gate"]
for rep in range(1 if workload == "c5" else 2):
    fn(buf)
    ctx.launch()
    ms, _ = ctx.sync()
    fn(buf)
    d = {k: int(v) for k, v in zip(names, buf)}
    w = max(d["wave_iters"], 1)
    frac = {k: round(d[k] / w, 5) for k in names[2:]}
    ev = int(ctx.download().totals["events"].sum())
    print(json.dumps({"ms": ms, **d, "events": ev, "lanes_per_wave_iter": round(d["lane_iters"] / w, 2),
                      "fraction_of_wave_iters": frac}), flush=True)
