"""torchrun worker for tests/test_gpu_abc_gather.py (not a test module): one engine context per rank over
interleaved replicate ids with the fused ABC statistics on, then the ABC step's exchange
(shard.gather_structured) of every replicate's statistics and summary into global id order.
Backend from ECDNA_GATHER_BACKEND: "nccl" (RCCL, device buffers) or "gloo" (host buffers; lets two ranks
share the one GPU of a test box)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ecdna-evo_amd"))

from ecdna_evo_amd import abi, engine, shard  # noqa: E402

TOTAL = 3000


def spec(first, n, stride, device):
    target = np.zeros(129, np.uint64)
    target[0], target[1:20], target[128] = 50, 7, 2
    return abi.RunSpec(seed=11, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3), (1.0, 2.0, 0.4, 0.2)),
                       reps_per_set=TOTAL // 2, first_replicate=first, n_replicates=n, replicate_stride=stride,
                       max_cells=800, hist_bins=129, init={1: 2, 40: 1}, stats_target=target, device=device,
                       flags=abi.FLAG_REP_STATS | abi.FLAG_EVENT_HASH | abi.FLAG_BIN_STORE, bin_kmax=32)


def main():
    out = sys.argv[1]
    backend = os.environ.get("ECDNA_GATHER_BACKEND", "nccl")
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = 0 if backend == "gloo" else int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")
    first, n, stride = shard.interleaved_range(rank, world, TOTAL)
    res = engine.run(spec(first, n, stride, local))
    dev = "cuda" if backend == "nccl" else None
    stats = shard.gather_structured(res.stats, TOTAL, "interleaved", device=dev)
    summ = shard.gather_structured(res.summaries, TOTAL, "interleaved", device=dev)
    if rank == 0:
        np.savez(out, stats=stats.view(np.uint8), summaries=summ.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
