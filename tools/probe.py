"""Quick throughput probe of the HIP engine on the BASELINE.json configs (development tool)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402


def probe(name, spec, reps=2):
    t0 = time.time()
    ctx = engine.Context(spec)
    chunk, lanes = ctx.geometry()
    for r in range(reps):
        t1 = time.time()
        ctx.launch()
        ssa_ms, hist_ms = ctx.sync()
        wall = time.time() - t1
        res = ctx.download()
        ev = int(res.totals["events"].sum())
        print(f"{name}: rep {r} events={ev:.3e} ssa={ssa_ms:.1f}ms hist={hist_ms:.1f}ms wall={wall*1e3:.1f}ms "
              f"-> {ev / (ssa_ms * 1e-3):.3e} ev/s (kernel) {ev / wall:.3e} ev/s (wall) chunk={chunk} lanes={lanes}",
              flush=True)
    ctx.close()
    print(f"{name}: total {time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    which = sys.argv[1:] or ["c2", "c3"]
    if "c2" in which:
        probe("C2 PB 65536x1e4", abi.RunSpec(seed=42, n_replicates=65536, max_cells=10_000, flags=0))
    if "c3" in which:
        probe("C3 BD 2^20x1e4", abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),),
                                            n_replicates=1 << 20, max_cells=10_000, flags=0))
    if "c2bins" in which:
        probe("C2 PB 65536x1e4 bins", abi.RunSpec(seed=42, n_replicates=65536, max_cells=10_000,
                                                  flags=abi.FLAG_BIN_STORE))
    if "c3bins1" in which:  # one launch only (profiling)
        probe("C3 BD 2^20x1e4 bins", abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),),
                                                 n_replicates=1 << 20, max_cells=10_000, flags=abi.FLAG_BIN_STORE), reps=1)
    if "c3bins" in which:
        probe("C3 BD 2^20x1e4 bins", abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),),
                                                 n_replicates=1 << 20, max_cells=10_000, flags=abi.FLAG_BIN_STORE))
