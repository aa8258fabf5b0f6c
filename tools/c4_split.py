"""The C4 8-GPU shard split by initial copy number: the sets with k0 >= 2^SPLIT_EX (the shard's critical
path) run on a wide-K instance (K = 256 by default: their cells stay in LDS bins instead of the large-k
row) concurrently, on a second stream, with the rest on the K = 64 instance. The shard's interleaved ids (rank r of 8:
r, r + 8, ...) hit the sets in order, so each class is one contiguous range of local indices and becomes its own
context (shard.k0_split). Each grid is capped (RunSpec.max_workgroups) so that the two persistent kernels share the
CUs. Prints the makespan (wall time between events around both launches) per setting, against the whole shard on
one context. Development / measurement tool.
Usage: [C4S_RANK=0] [C4S_GPUS=8] [C4S_SPLITS=6,7] [C4S_WIDE=256] [C4S_BLOCKS="A:B,..."] python tools/c4_split.py"""
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402  (first: one HIP runtime)

from ecdna_evo_amd import abi, engine, shard  # noqa: E402
import probe_configs  # noqa: E402


def timed(ctxs, reps=3):
    streams = [torch.cuda.Stream() for _ in ctxs]
    best = None
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        for c, s in zip(ctxs, streams):
            s.wait_event(e0)
            c.launch(s.cuda_stream)
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    per = [c.sync()[0] for c in ctxs]
    ev = sum(int(c.download().totals["events"].sum()) for c in ctxs)
    err = sum(int(c.download().totals["errors"].sum()) for c in ctxs)
    return best, per, ev, err


def main():
    rank = int(os.environ.get("C4S_RANK", "0"))
    gpus = int(os.environ.get("C4S_GPUS", "8"))
    wide = int(os.environ.get("C4S_WIDE", "256"))
    base = dataclasses.replace(probe_configs.c4_shard(rank, gpus), flags=abi.FLAG_BIN_STORE, bin_kmax=64, _keep=[])
    whole = engine.Context(base)
    ms, per, ev, err = timed([whole])
    print(json.dumps({"setting": "whole K=64", "gpus": gpus, "rank": rank, "makespan_ms": ms, "stepper_ms": per,
                      "events": ev, "errors": err, "instance": whole.instance()}), flush=True)
    whole.close()
    for ex in [int(x) for x in os.environ.get("C4S_SPLITS", "7").split(",")]:
        for pair in os.environ.get("C4S_BLOCKS", "320:640,384:512,0:0").split(","):
            caps = tuple(int(x) for x in pair.split(":"))
            parts = shard.k0_split(base, 1 << ex, wide, caps)
            ctxs = [engine.Context(sp) for sp, _ in parts]
            ms, per, ev, err = timed(ctxs)
            print(json.dumps({"setting": f"k0>=2^{ex} on K={wide}", "gpus": gpus, "rank": rank, "blocks": list(caps),
                              "makespan_ms": ms, "stepper_ms": per,
                              "replicates": [sp.n_replicates for sp, _ in parts], "events": ev, "errors": err,
                              "grid_lanes": [c.instance()["grid_lanes"] for c in ctxs]}), flush=True)
            for c in ctxs:
                c.close()


if __name__ == "__main__":
    main()
