"""Randomized GPU-vs-oracle parity: 60 RunSpecs drawn from a fixed-seed generator over every knob of
the ABI (process, segregation, rates, initial distributions with small and large copy numbers, cell
caps, time and iteration caps, f32 time, the birth-death cap flag, parameter sets, replicate-id
offsets, snapshots). Every output must be bit-identical."""
import numpy as np
import pytest

from ecdna_evo_amd import abi
from test_gpu_parity import _compare


def random_spec(i):
    g = np.random.default_rng(1000 + i)
    process = int(g.integers(0, 2))
    n_sets = int(g.choice([1, 1, 2, 3]))
    rates = []
    for _ in range(n_sets):
        b0, b1 = float(g.uniform(0.2, 2.0)), float(g.uniform(0.2, 3.0))
        d0 = float(g.uniform(0, 1.5)) if process else 0.0
        d1 = float(g.uniform(0, 1.5)) if process else 0.0
        rates.append((b0, b1, d0, d1))
    init = {}
    for _ in range(int(g.integers(1, 5))):
        k = int(g.choice([1, 2, 3, 5, 16, 17, 40, 333, 4000]))
        init[k] = init.get(k, 0) + int(g.integers(1, 60))
    if g.random() < 0.3:
        init[0] = int(g.integers(1, 40))
    cells0 = sum(v for k, v in init.items())
    max_cells = int(cells0 + g.integers(5, 1500))
    reps_per_set = int(g.integers(5, 40))
    first = int(g.choice([0, 0, 17, 100_000]))
    n = reps_per_set * n_sets - (first % reps_per_set if first else 0)
    flags = abi.FLAG_EVENT_HASH
    if g.random() < 0.3:
        flags |= abi.FLAG_TIME_F32
    if process and g.random() < 0.3:
        flags |= abi.FLAG_BD_CAP_COMPAT
    snaps = None
    if g.random() < 0.4:
        snaps = sorted(int(x) for x in g.integers(1, max_cells + 5, int(g.integers(1, 8))))
        flags |= abi.FLAG_SNAPSHOT_ROWS
    cap = None
    if g.random() < 0.2:
        cap = int(max(len([1 for k in init if k]) and sum(v for k, v in init.items() if k), 1) + g.integers(0, 200))
    return abi.RunSpec(
        process=process, segregation=int(g.integers(0, 4)), rates=rates, reps_per_set=reps_per_set,
        first_replicate=first, n_replicates=max(n, 1), seed=int(g.integers(0, 2**63)), max_cells=max_cells,
        max_time=float(g.choice([1e9, float(g.uniform(0.5, 12.0))])), max_iter=int(g.choice([1_000_000_000, 5000])),
        cell_cap=cap, hist_bins=int(g.choice([2, 64, 1025])), init=init, snapshots=snaps, flags=flags)


def _first_set_fits(spec):
    # replicate ids must map inside the parameter sets
    return (spec.first_replicate + spec.n_replicates - 1) // spec.reps_per_set < len(spec.rates)


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(60))
def test_random_spec_parity(i, engine_mod, oracle_mod):
    spec = random_spec(i)
    if not _first_set_fits(spec):
        spec.first_replicate = 0
        spec.n_replicates = spec.reps_per_set * len(spec.rates)
    gpu = engine_mod.run(spec, want_rows=True)
    cpu = oracle_mod.run(spec, mode="philox", want_rows=True)
    _compare(gpu, cpu, f"random[{i}]")


def test_random_specs_are_valid_for_the_oracle(oracle_mod):
    """CPU side: every generated spec runs in the oracle (keeps the GPU test's inputs honest)."""
    for i in range(60):
        spec = random_spec(i)
        if not _first_set_fits(spec):
            spec.first_replicate = 0
            spec.n_replicates = spec.reps_per_set * len(spec.rates)
        oracle_mod.run(spec, mode="philox")

