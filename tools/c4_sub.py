"""C4 8-GPU shard restricted to the sets of one initial copy number k0 (development tool): times the stepper on
the 512 replicates per set a rank holds, to see which sets set the shard's critical path.
Usage: [PROBE_KMAX=64] python tools/c4_sub.py <k0 exponent 0..7>..."""
import dataclasses
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import probe_configs  # noqa: E402

for ex in [int(x) for x in sys.argv[1:]]:
    spec = dataclasses.replace(probe_configs.c4_subset(ex), flags=abi.FLAG_BIN_STORE,
                               bin_kmax=int(os.environ.get("PROBE_KMAX", "64")), _keep=[])
    ctx = engine.Context(spec)
    for _ in range(2):
        ctx.launch()
        s_ms, _ = ctx.sync()
    t = ctx.download().totals
    print(json.dumps({"k0": 1 << ex, "replicates": spec.n_replicates, "stepper_ms": round(s_ms, 1),
                      "events": int(t["events"].sum()), "geometry": ctx.geometry(), "errors": int(t["errors"].sum())}),
          flush=True)
    ctx.close()
