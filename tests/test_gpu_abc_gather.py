"""The ABC step's exchange on the GPU path (a gather of per-replicate records beside the
histogram all-reduce): engine contexts over interleaved replicate ids compute the fused statistics
(abc.md:38-55), shard.gather_structured brings every replicate's statistics and summary into global id
order, and the result must equal one single-process run of all ids byte for byte.
- torchrun with one rank: the RCCL path (device exchange buffers);
- torchrun with two ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one device): the
  reordering of real interleaved shards."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,backend", [(1, "nccl"), (2, "gloo")])
def test_gather_of_rep_stats_matches_one_run(tmp_path, engine_mod, nproc, backend):
    sys.path.insert(0, HERE)
    import abc_gather_worker as w

    out = tmp_path / "g.npz"
    env = dict(os.environ, ECDNA_GATHER_BACKEND=backend)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(HERE, "abc_gather_worker.py"),
           str(out)]
    r = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    full = engine_mod.run(w.spec(0, w.TOTAL, 1, 0))
    d = np.load(out)
    assert d["stats"].tobytes() == full.stats.tobytes()
    assert d["summaries"].tobytes() == full.summaries.tobytes()
