"""Bin store replicate rotation (DESIGN.md §5 "Rotation"): waves park their lanes' replicates every
2^k loop iterations and lanes resume waiting replicates of their XCD's partition, possibly on another
CU; lanes whose partition is drained steal fresh replicates of other partitions and run them pinned.

Replicates are keyed by id, never by lane, so none of this may change a single output bit. Rotation is
forced here far harder than any production run does it: a tick every 1 or 8 iterations, parking
whenever one replicate waits, 1 or 8 workgroups (1: one XCD's lanes run everything, seven partitions
entirely through the steal path). Each case is checked bit for bit against the CPU oracle.
"""

import numpy as np
import pytest

from ecdna_evo_amd import abi
from test_gpu_parity import _compare

H = abi.FLAG_EVENT_HASH
B = abi.FLAG_BIN_STORE
BD = ((1.0, 1.5, 0.3, 0.3),)


def rotation_cases():
    c = {}
    c["bd_k32"] = abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=BD, n_replicates=4096, max_cells=150,
                              bin_kmax=32, flags=H | B)
    c["bd_k64_u16"] = abi.RunSpec(seed=43, process=abi.BIRTH_DEATH, rates=BD, n_replicates=3000, max_cells=150,
                                  flags=H | B)
    # copy numbers above K: the large-k row in HBM follows its replicate from CU to CU
    c["big_row"] = abi.RunSpec(seed=44, process=abi.BIRTH_DEATH, rates=((1.0, 1.3, 0.6, 0.7),), n_replicates=2048,
                               max_cells=120, init={40: 2, 70: 1, 1: 2}, hist_bins=300, bin_kmax=32, flags=H | B)
    c["no_uneven"] = abi.RunSpec(seed=45, segregation=abi.SEG_BINOMIAL_NO_UNEVEN, n_replicates=2048,
                                 max_cells=100, init={17: 2, 3: 2}, bin_kmax=32, flags=H | B)
    c["deterministic_f32"] = abi.RunSpec(seed=46, segregation=abi.SEG_DETERMINISTIC, process=abi.BIRTH_DEATH,
                                         rates=BD, n_replicates=2048, max_cells=120, init={3: 1},
                                         flags=H | B | abi.FLAG_TIME_F32)
    c["snapshots"] = abi.RunSpec(seed=47, process=abi.BIRTH_DEATH, rates=((1.0, 1.1, 0.9, 0.9),),
                                 n_replicates=2048, max_cells=80, init={2: 20, 33: 2}, snapshots=[15, 21, 30, 60],
                                 bin_kmax=32, flags=H | B | abi.FLAG_SNAPSHOT_ROWS | abi.FLAG_TIME_F32)
    c["abc_sets"] = abi.RunSpec(seed=48, process=abi.BIRTH_DEATH,
                                rates=((1.0, 1.0, 0.1, 0.1), (1.0, 1.5, 0.1, 0.1), (1.0, 2.0, 0.3, 0.2),
                                       (1.0, 2.5, 0.0, 0.4)),
                                reps_per_set=640, n_replicates=2560, max_cells=120, hist_bins=257,
                                init_per_set=[{1: 1}, {2: 1}, {4: 1, 0: 3}, {8: 2}], bin_kmax=32, flags=H | B)
    # stop reasons and errors mixed: extinction, the row-capacity error, max_iter
    c["errors"] = abi.RunSpec(seed=49, process=abi.BIRTH_DEATH, rates=((1.0, 1.0, 0.4, 0.4),), n_replicates=1024,
                              max_cells=300, max_iter=200, cell_cap=128, init={1: 1, 0: 1}, bin_kmax=32, flags=H | B)
    return c


CASES = rotation_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["2", "3"])  # 3: the 128-VGPR K = 64 / u16 build (the default elsewhere)
@pytest.mark.parametrize("blocks,tick", [(8, 0), (8, 3), (1, 2)])
@pytest.mark.parametrize("name", sorted(CASES))
def test_gpu_rotation_matches_oracle(name, blocks, tick, sched, engine_mod, oracle_mod, monkeypatch):
    spec = CASES[name]
    monkeypatch.setenv("ECDNA_SSA_SCHED", sched)
    monkeypatch.setenv("ECDNA_SSA_ROTATE", "1")
    monkeypatch.setenv("ECDNA_SSA_ROT_TICK", str(tick))
    monkeypatch.setenv("ECDNA_SSA_ROT_PARK_MIN", "1")
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", str(blocks))
    gpu = engine_mod.run(spec, want_rows=True)
    cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
    _compare(gpu, cpu, f"{name}/blocks{blocks}/tick{tick}/sched{sched}")


@pytest.mark.gpu
@pytest.mark.parametrize("kmax", [32, 64])
def test_gpu_rotation_on_off_identical_at_scale(kmax, engine_mod, monkeypatch):
    """The production setting (auto: lanes run >= 2 replicates each; a tick every 2^11 iterations)
    against no rotation, on 300k birth-death replicates over a 512-block grid."""
    spec = abi.RunSpec(seed=7, process=abi.BIRTH_DEATH, rates=BD, n_replicates=300_000, max_cells=400,
                       bin_kmax=kmax, flags=H | B)
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", "512")
    runs = {}
    for mode, tick, sched in (("2", "11", "2"), ("2", "6", "2"), ("2", "11", "3"), ("0", "11", "2")):
        monkeypatch.setenv("ECDNA_SSA_ROTATE", mode)
        monkeypatch.setenv("ECDNA_SSA_ROT_TICK", tick)
        monkeypatch.setenv("ECDNA_SSA_SCHED", sched)  # 3: the 128-VGPR build at K = 64
        runs[(mode, tick, sched)] = engine_mod.run(spec)
    ref = runs[("0", "11", "2")]
    for key, r in runs.items():
        for f in ref.summaries.dtype.names:
            a, b = r.summaries[f], ref.summaries[f]
            if f == "time":
                a, b = a.view(np.uint64), b.view(np.uint64)
            np.testing.assert_array_equal(a, b, err_msg=f"{key}: {f}")
        np.testing.assert_array_equal(r.hist, ref.hist, err_msg=str(key))
    assert int(ref.summaries["iters"].sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("rotate,blocks,tick", [("1", 8, 2), ("1", 1, 0), ("0", 8, 10)])
@pytest.mark.parametrize("store", ["bins", "rows"])
def test_gpu_set_cost_hint_start_order_matches_oracle(store, rotate, blocks, tick, engine_mod, oracle_mod,
                                                      monkeypatch):
    """set_cost_hint (include/ecdna_ssa.h) only reorders which replicates start first: through the plain
    work queue, the rotation's item walk (partitions walk the cost order) and the steal path, results
    stay bit-exact with the oracle, which ignores the hint."""
    import dataclasses

    base = CASES["abc_sets"]
    spec = dataclasses.replace(base, set_cost_hint=[1.0, 4.0, 2.0, 8.0], first_replicate=3, replicate_stride=1,
                               n_replicates=2557, flags=H | (B if store == "bins" else 0), _keep=[])
    monkeypatch.setenv("ECDNA_SSA_ROTATE", rotate)
    monkeypatch.setenv("ECDNA_SSA_ROT_TICK", str(tick))
    monkeypatch.setenv("ECDNA_SSA_ROT_PARK_MIN", "1")
    monkeypatch.setenv("ECDNA_SSA_MAX_BLOCKS", str(blocks))
    monkeypatch.setenv("ECDNA_SSA_MAX_CHUNK", "1000")  # three chunks: the order is chunk-local
    gpu = engine_mod.run(spec, want_rows=False)
    cpu = oracle_mod.run(spec, mode="philox")
    for f in cpu.summaries.dtype.names:
        a, b = gpu.summaries[f], cpu.summaries[f]
        if f == "time":
            a, b = a.view(np.uint64), b.view(np.uint64)
        np.testing.assert_array_equal(a, b, err_msg=f"{store}/{rotate}/{blocks}/{tick}: {f}")
    np.testing.assert_array_equal(gpu.hist, cpu.hist)
