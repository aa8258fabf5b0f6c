"""Sweep engine launch knobs (env vars read by ssa_api.cpp) on the C3 workload; one subprocess per
setting. Usage: python tools/sweep.py VAR=v1,v2,... [VAR2=...] [--reps N]"""
import itertools
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, json, time
sys.path.insert(0, os.path.join(%r, "ecdna-evo_amd"))
from ecdna_evo_amd import abi, engine
spec = abi.RunSpec(seed=42, process=abi.BIRTH_DEATH, rates=((1.0, 1.5, 0.3, 0.3),), reps_per_set=int(os.environ.get("SWEEP_REPS", 1 << 20)),
                   n_replicates=int(os.environ.get("SWEEP_REPS", 1 << 20)), max_cells=10_000,
                   flags=int(os.environ.get("SWEEP_FLAGS", "0"), 0), bin_kmax=int(os.environ.get("SWEEP_KMAX", "0")))
ctx = engine.Context(spec)
ms = []
for i in range(3):
    ctx.launch(); s, h = ctx.sync(); ms.append(s)
ev = int(ctx.download().totals["events"].sum())
print(json.dumps({"ms": ms, "events": ev, "lanes": ctx.geometry()[1]}))
''' % REPO


def main():
    axes = []
    for a in sys.argv[1:]:
        k, v = a.split("=", 1)
        axes.append([(k, x) for x in v.split(",")])
    for combo in itertools.product(*axes):
        env = dict(os.environ)
        env.update(dict(combo))
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=600)
        if out.returncode:
            print(dict(combo), "FAILED", out.stderr[-500:], flush=True)
            continue
        d = json.loads(out.stdout.strip().splitlines()[-1])
        best = min(d["ms"][1:])
        print(json.dumps({**dict(combo), "lanes": d["lanes"], "ms": [round(x, 1) for x in d["ms"]],
                          "ev_per_s": d["events"] / (best * 1e-3)}), flush=True)


if __name__ == "__main__":
    main()
