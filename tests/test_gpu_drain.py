"""Bin store drain control (ssa_api.cpp launch): when lanes run more than two replicates
each, the youngest wave slot of every SIMD stops taking fresh replicates near the end of the work
queue. Replicates are keyed by id, not by lane, so switching it off (ECDNA_SSA_ADMIT=0) must not change
a single output."""
import numpy as np
import pytest


@pytest.mark.gpu
@pytest.mark.parametrize("kmax", [32, 64])
def test_gpu_drain_control_does_not_change_results(kmax, engine_mod, monkeypatch):
    from ecdna_evo_amd import abi

    # 512 blocks of 256 lanes = 2 blocks per CU on 256 CUs; 300k replicates > 2 grids' worth, so the
    # drain control is active in the first run
    spec = abi.RunSpec(seed=7, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), n_replicates=300_000,
                       max_cells=64, init={1: 1}, bin_kmax=kmax, flags=abi.FLAG_EVENT_HASH | abi.FLAG_BIN_STORE)
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", "512")
    on = engine_mod.run(spec)
    monkeypatch.setenv("ECDNA_SSA_ADMIT", "0")
    off = engine_mod.run(spec)
    for f in on.summaries.dtype.names:
        a, b = on.summaries[f], off.summaries[f]
        if f == "time":
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, err_msg=f)
    np.testing.assert_array_equal(on.hist, off.hist)
    assert int(on.summaries["iters"].sum()) > 0
