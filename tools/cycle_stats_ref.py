"""Section cycle counters of the reference-draws stepper (ssa_stepper_refdraws, ECDNA_FLAG_REFERENCE_DRAWS) over one
launch (development tool): where a wave's time goes per event (replicate boundary, ChaCha8 top-up,
stop checks + first-reaction Exp1 draws, cell pick, segregation, the rest), plus the sampler counts (refills in the
top-up and inside events, Exp1 retries, BTPE / BINV draws). Needs a library built with -DECDNA_CYCLE_STATS
(EXTRA=-DECDNA_CYCLE_STATS bash tools/ab_build.sh WORKTREE cyc), selected with ECDNA_SSA_LIB.
Usage: python tools/cycle_stats_ref.py [c3|c2] [replicates]"""
import ctypes as C
import dataclasses
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ecdna-evo_amd"))
sys.path.insert(0, REPO)
from ecdna_evo_amd import abi, engine  # noqa: E402

import bench  # noqa: E402

NAMES = ["cyc_boundary", "cyc_topup", "cyc_first_reaction", "cyc_pick", "cyc_btpe", "cyc_rest", "cyc_binv", "",
         "lane_iters", "wave_iters_refilled", "lane_refills_topup", "lane_refills_inner", "exp1_retries",
         "btpe_draws", "binv_draws", "cyc_kernel"]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else (1 << 20 if wl == "c3" else 65_536)
    spec = bench.workload_spec(0, n, n, store="rows", workload=wl)
    spec = dataclasses.replace(spec, flags=spec.flags | abi.FLAG_REFERENCE_DRAWS, _keep=[])
    lib = engine.lib()
    fn = lib.ecdna_dev_cycle_stats_ref
    fn.argtypes = [C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 16)()
    ctx = engine.Context(spec)
    fn(buf)
    ctx.launch()
    ms, _ = ctx.sync()
    fn(buf)
    d = {k: int(v) for k, v in zip(NAMES, buf) if k}
    res = ctx.download()
    ev = int(res.totals["events"].sum())
    geo = ctx.geometry()
    ctx.close()
    waves = geo[1] // 64
    sec = [k for k in NAMES[:7]]
    tot = sum(d[k] for k in sec)
    print(json.dumps({"config": f"{wl} reference draws", "replicates": n, "ms": ms, "events": ev, "events_per_s": ev / ms * 1e3,
                      "grid_lanes": geo[1], **d,
                      "share": {k: round(d[k] / max(tot, 1), 3) for k in sec},
                      "cycles_per_wave_event": {k: round(d[k] * 64 / max(ev, 1), 1) for k in sec},
                      "per_event": {k: round(d[k] / max(ev, 1), 4) for k in NAMES[9:15] if k},
                      "waves": waves}), flush=True)


if __name__ == "__main__":
    main()
