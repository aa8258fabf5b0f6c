"""The C4 8-GPU shard split by initial copy number: the sets with k0 >= 2^SPLIT_EX (the shard's critical
path) run on a wide-K instance (K = 256 by default: their cells stay in LDS bins instead of the large-k
row) concurrently, on a second stream, with the rest on the K = 64 instance. The shard's interleaved ids (rank r of 8:
r, r + 8, ...) hit the sets in order, so each class is one contiguous range of local indices and becomes its own
context (first_replicate, n, stride 8). Each grid is capped (ECDNA_SSA_MAX_BLOCKS, read at create) so that the two
persistent kernels share the CUs. Prints the makespan (wall time between events around both launches) per setting,
against the whole shard on one context. Development / measurement tool.
Usage: [C4S_RANK=0] [C4S_SPLITS=6,7] [C4S_WIDE=256] [C4S_BLOCKS="A:B,..."] python tools/c4_split.py"""
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402  (first: one HIP runtime)

from ecdna_evo_amd import abi, engine  # noqa: E402
import probe_configs  # noqa: E402


def ctx_with(spec, max_blocks):
    if max_blocks:
        os.environ["ECDNA_SSA_MAX_BLOCKS"] = str(max_blocks)
    else:
        os.environ.pop("ECDNA_SSA_MAX_BLOCKS", None)
    try:
        return engine.Context(spec)
    finally:
        os.environ.pop("ECDNA_SSA_MAX_BLOCKS", None)


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
    wide = int(os.environ.get("C4S_WIDE", "256"))
    base = dataclasses.replace(probe_configs.c4_shard(rank, 8), flags=abi.FLAG_BIN_STORE, bin_kmax=64, _keep=[])
    n, first, stride = base.n_replicates, base.first_replicate, base.stride()
    whole = ctx_with(base, 0)
    ms, per, ev, err = timed([whole])
    print(json.dumps({"setting": "whole K=64", "makespan_ms": ms, "stepper_ms": per, "events": ev, "errors": err,
                      "instance": whole.instance()}), flush=True)
    whole.close()
    for ex in [int(x) for x in os.environ.get("C4S_SPLITS", "6,7").split(",")]:
        s0 = 128 * ex  # first set with k0 = 2^ex (sets are ordered by k0 in blocks of 128)
        i0 = (4096 * s0 - first + stride - 1) // stride  # first local index in those sets
        narrow = dataclasses.replace(base, n_replicates=i0, _keep=[])
        heavy = dataclasses.replace(base, first_replicate=first + i0 * stride, n_replicates=n - i0, bin_kmax=wide,
                                    _keep=[])
        for pair in os.environ.get("C4S_BLOCKS", "0:0,512:256,640:128,512:512,384:512").split(","):
            ba, bb = (int(x) for x in pair.split(":"))
            ca, cb = ctx_with(narrow, ba), ctx_with(heavy, bb)
            ms, per, ev, err = timed([ca, cb])
            print(json.dumps({"setting": f"k0>=2^{ex} on K={wide}", "blocks": [ba, bb], "makespan_ms": ms,
                              "stepper_ms": per, "replicates": [i0, n - i0], "events": ev, "errors": err,
                              "grid_lanes": [ca.instance()["grid_lanes"], cb.instance()["grid_lanes"]]}), flush=True)
            ca.close()
            cb.close()


if __name__ == "__main__":
    main()
