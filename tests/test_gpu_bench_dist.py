"""bench.py's N>1 path, rehearsed on a one-GPU box (the driver's 8-GPU scaling runs cannot be
launched from here).

- torchrun with one rank: the RCCL process group, barriers, the all-reduce of histogram and totals
  and the max-over-ranks timing all run, as they do at N = 2, 4, 8.
- torchrun with two ranks sharing cuda:0, reduced over gloo (RCCL refuses two ranks on one device):
  weak-scaling shards [0, n) and [n, 2n) of global replicate ids, each on its own engine context.

Both reduced histograms must equal a single-process run of the same global ids bit for bit (the
1-GPU == N-GPU identity), and each run must print exactly one JSON line with the
contract's fields."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_TOTAL = 1 << 15


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(nproc, reps_per_gpu, dump, extra_env, extra_args=()):
    env = dict(os.environ)
    env.update(extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", str(nproc), "--steps", "2", "--warmup", "1", "--reps-per-gpu", str(reps_per_gpu),
           "--no-cpu-baseline", "--dump-hist", str(dump), *extra_args]
    out = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


def _check_line(line, nproc, reps_per_gpu):
    assert line["n_gpus"] == nproc and line["steps"] == 2 and line["warmup"] == 1
    assert line["unit"] == "events/s" and line["scaling"] == "weak" and line["higher_is_better"] is True
    assert line["config"]["replicates_total"] == nproc * reps_per_gpu
    assert line["value"] > 0 and line["roofline"]["peak"] == 8000.0
    assert line["value"] == pytest.approx(line["config"]["events_per_step"] * 2 / (line["ms_per_step"] * 2e-3))


@pytest.mark.gpu
def test_bench_distributed_paths_match_one_process(tmp_path):
    one = _torchrun(1, N_TOTAL, tmp_path / "one.npz", {})
    _check_line(one, 1, N_TOTAL)
    two = _torchrun(2, N_TOTAL // 2, tmp_path / "two.npz",
                    {"ECDNA_BENCH_BACKEND": "gloo", "ECDNA_BENCH_ONE_DEVICE": "1"})
    _check_line(two, 2, N_TOTAL // 2)

    # the same global ids in one process, through the engine directly
    sys.path.insert(0, REPO)
    import bench
    from ecdna_evo_amd import engine

    ctx = engine.Context(bench.workload_spec(0, N_TOTAL, N_TOTAL))
    ctx.launch()
    ctx.sync()
    res = ctx.download()
    ctx.close()
    ref_hist = res.hist.astype(np.int64).reshape(-1)
    ref_tot = res.totals.view(np.uint64).astype(np.int64).reshape(-1)
    for f in ("one.npz", "two.npz"):
        d = np.load(tmp_path / f)
        np.testing.assert_array_equal(d["hist"], ref_hist)
        np.testing.assert_array_equal(d["totals"].astype(np.int64), ref_tot)
    assert one["config"]["events_per_step"] == two["config"]["events_per_step"] == int(ref_tot[1])


# the strong-scaling lines BASELINE.json places on 8 GPUs (C4: the ABC sweep's interleaved shards with the cost
# hint's start order; C5: the turnover run), scaled down: (total replicates, cell cap)
STRONG = {"c4": (1024 * 16, None), "c5": (512, 20_000), "c2": (4096, 2_000)}


@pytest.mark.gpu
@pytest.mark.parametrize("workload", sorted(STRONG))
def test_bench_strong_scaling_paths_match_one_process(tmp_path, workload):
    """bench.py --workload c2/c4/c5 under torchrun: one rank over RCCL, and two ranks sharing cuda:0 over gloo
    (interleaved global-id shards g, g + 2, ...; C4 with its per-set cost hint and its k0 split). The reduced
    histogram and totals equal one engine run of every id (C4: of each k0 class at its K) bit for bit, and the line
    reports strong scaling."""
    total, cells = STRONG[workload]
    extra = ["--workload", workload, "--total", str(total)] + (["--max-cells", str(cells)] if cells else [])
    one = _torchrun(1, 0, tmp_path / "one.npz", {}, extra)
    two = _torchrun(2, 0, tmp_path / "two.npz", {"ECDNA_BENCH_BACKEND": "gloo", "ECDNA_BENCH_ONE_DEVICE": "1"}, extra)
    for line, n in ((one, 1), (two, 2)):
        assert line["n_gpus"] == n and line["scaling"] == "strong" and line["config"]["replicates_total"] == total
        assert line["config"]["replicate_errors"] == 0

    sys.path.insert(0, REPO)
    import bench
    from ecdna_evo_amd import engine

    from ecdna_evo_amd import shard

    spec = bench.workload_spec(0, total, total, workload=workload, max_cells=cells)
    # C4: the bench splits every rank's shard by initial copy number (its k0 = 128 replicates on K = 256,
    # bench.C4_SPLIT_CAPS at 1 and 2 GPUs), so the reference runs the same two classes of ids
    parts = shard.k0_split(spec, bench.C4_SPLIT_K0, bench.C4_SPLIT_KMAX, (0, 0)) if workload == "c4" else [(spec, 0)]
    ref_hist, ref_tot = 0, 0
    for sp, _ in parts:
        ctx = engine.Context(sp)
        ctx.launch()
        ctx.sync()
        res = ctx.download()
        ctx.close()
        ref_hist = ref_hist + res.hist.astype(np.int64).reshape(-1)
        ref_tot = ref_tot + res.totals.view(np.uint64).astype(np.int64).reshape(-1)
    for f in ("one.npz", "two.npz"):
        d = np.load(tmp_path / f)
        np.testing.assert_array_equal(d["hist"], ref_hist, err_msg=f)
        np.testing.assert_array_equal(d["totals"].astype(np.int64), ref_tot, err_msg=f)
    assert one["config"]["events_per_step"] == two["config"]["events_per_step"] == int(ref_tot.reshape(-1, 16)[:, 1].sum())
