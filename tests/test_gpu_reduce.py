"""The multi-GPU reduction of the C ABI (ABI v6, include/ecdna_ssa.h): RCCL communicators
made by the engine and the all-reduce of a run's histogram and totals (ncclUint64, ncclSum). On this one-GPU
box the communicators have one rank, so the reduced outputs must equal the unreduced ones bit for bit; the
2-rank sum is covered by the CPU gloo tests of the same sharding (tests/test_multiprocess.py) and the
torch.distributed path of bench.py (tests/test_gpu_bench_dist.py)."""
import numpy as np
import pytest

from ecdna_evo_amd import abi

SPEC = dict(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3), (1.0, 2.0, 0.5, 0.5)), reps_per_set=512,
            n_replicates=1024, max_cells=2000, hist_bins=257, flags=abi.FLAG_BIN_STORE, bin_kmax=32)


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["init_all", "init_rank"])
def test_ctx_reduce_at_one_rank_is_identity(engine_mod, how):
    spec = abi.RunSpec(**SPEC)
    if how == "init_all":
        (comm,) = engine_mod.Comm.init_all([0])
    else:
        comm = engine_mod.Comm.init_rank(engine_mod.Comm.unique_id(), 1, 0, 0)
    try:
        with engine_mod.Context(spec) as ctx:
            ctx.launch()
            ctx.sync()
            before = ctx.download()
            ctx.reduce(comm)
            ctx.sync()
            after = ctx.download()
        np.testing.assert_array_equal(after.hist, before.hist)
        for f in before.totals.dtype.names:
            np.testing.assert_array_equal(after.totals[f], before.totals[f], err_msg=f)
        assert int(after.totals["replicates"].sum()) == 1024 and after.hist.sum() > 0
    finally:
        comm.close()


@pytest.mark.gpu
def test_reduce_hist_on_caller_buffers(engine_mod):
    """ecdna_ssa_reduce_hist on device buffers the caller owns (torch tensors set as the context's outputs),
    enqueued on the caller's stream."""
    import ctypes as C

    import torch

    spec = abi.RunSpec(**SPEC)
    (comm,) = engine_mod.Comm.init_all([0])
    try:
        hist = torch.zeros(2 * 257, dtype=torch.int64, device="cuda")
        tot = torch.zeros(2 * 16, dtype=torch.int64, device="cuda")
        s = torch.cuda.Stream()
        with engine_mod.Context(spec) as ctx:
            ctx.set_outputs(hist.data_ptr(), tot.data_ptr())
            ctx.launch(s.cuda_stream)
            ctx.sync()
            h0, t0 = hist.cpu().clone(), tot.cpu().clone()
            rc = engine_mod.lib().ecdna_ssa_reduce_hist(comm.h, C.c_void_p(hist.data_ptr()), C.c_void_p(tot.data_ptr()),
                                                        2, 257, C.c_void_p(s.cuda_stream))
            assert rc == 0, engine_mod.lib().ecdna_ssa_last_error_message()
            s.synchronize()
        assert torch.equal(hist.cpu(), h0) and torch.equal(tot.cpu(), t0)
        assert int(t0.view(2, 16)[:, 0].sum()) == 1024
    finally:
        comm.close()
