"""Rotation counters of one C3 launch (development tool). Needs a library built with -DECDNA_ROT_STATS
(tools/ab_build.sh-style: EXTRA=-DECDNA_ROT_STATS bash tools/ab_build.sh <ref> <name>), selected with
ECDNA_SSA_LIB. Prints parks, claim rounds, fresh/parked claims, steal rounds, ticks with/without parking."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402

spec = abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=1 << 20,
                   max_cells=10_000, flags=abi.FLAG_BIN_STORE, bin_kmax=32)
lib = engine.lib()
fn = lib.ecdna_dev_rot_stats
fn.argtypes = [C.POINTER(C.c_ulonglong)]
ctx = engine.Context(spec)
buf = (C.c_ulonglong * 12)()
for rep in range(2):
    fn(buf)
    ctx.launch()
    ms, _ = ctx.sync()
    fn(buf)
    names = ["parks", "claim_rounds", "claims_fresh", "claims_parked", "steal_rounds", "tick_lanes_park",
             "tick_lanes_nopark", "-", "wave_cyc_tick", "wave_cyc_boundary", "wave_cyc_total", "-"]
    print(json.dumps({"ms": ms, **{k: int(v) for k, v in zip(names, buf)}}), flush=True)
