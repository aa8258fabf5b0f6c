"""The metric's fixed-total reading of C3 on one GPU: 2^20 replicates split over G = 1, 2, 4, 8 GPUs, every shard of
every G run one after another on this GPU (bench.py --scaling strong's shards). Prints per shard the stepper time (median
of REPS launches; best and worst too), the instance, and per G the makespan (slowest shard's median) and the projected
speed-up T(1) / makespan(G).
Development / measurement tool. Usage: [C3S_GPUS=1,2,4,8] [C3S_REPS=3] [PROBE_KMAX=32] [KNOB=..] python tools/c3_strong.py"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ecdna_evo_amd import engine, shard  # noqa: E402

import bench  # noqa: E402

TOTAL = 1 << 20


def main():
    gpus = [int(x) for x in os.environ.get("C3S_GPUS", "1,2,4,8").split(",")]
    reps = int(os.environ.get("C3S_REPS", "3"))
    kmax = int(os.environ.get("PROBE_KMAX", "0")) or None
    ranks_env = os.environ.get("C3S_RANKS")
    t1 = None
    for g in gpus:
        ms_all, ev_all = [], 0
        ranks = range(g) if not ranks_env else [int(r) for r in ranks_env.split(",") if int(r) < g]
        for r in ranks:
            first, n = shard.shard_range(r, g, TOTAL)
            spec = bench.workload_spec(first, n, TOTAL, bin_kmax=kmax)
            ctx = engine.Context(spec)
            ms = []
            for _ in range(reps):
                ctx.launch()
                s, _h = ctx.sync()
                ms.append(s)
            res = ctx.download()
            ev = int(res.totals["events"].sum())
            err = int(res.totals["errors"].sum())
            ins = ctx.instance()
            ctx.close()
            best = min(ms)
            med = sorted(ms)[len(ms) // 2]
            ms_all.append(med)
            ev_all += ev
            print(json.dumps({"gpus": g, "rank": r, "replicates": n, "events": ev, "errors": err,
                              "stepper_ms": [round(x, 2) for x in ms], "median_ms": round(med, 2), "best_ms": round(best, 2),
                              "worst_ms": round(max(ms), 2),
                              "events_per_s": ev / (best * 1e-3), "instance": ins}), flush=True)
        mk = max(ms_all)
        if g == 1:
            t1 = mk
        print(json.dumps({"gpus": g, "makespan_ms": round(mk, 2), "makespan_of": "median of repeats", "mean_ms": round(sum(ms_all) / len(ms_all), 2),
                          "events": ev_all, "projected_events_per_s": ev_all / (mk * 1e-3),
                          "projected_speedup": (t1 / mk) if t1 else None}), flush=True)


if __name__ == "__main__":
    main()
