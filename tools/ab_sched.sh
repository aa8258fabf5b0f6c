#!/bin/bash
# Same library, both bin-stepper schedules (ECDNA_SSA_SCHED=0 occupancy-first, 1 max-ILP) on C2 and the
# C4 / C5 rank-0 shards, then the C3 sweep (auto = default there). Usage: bash tools/ab_sched.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_sched.log; mkdir -p gpurun_out; : > $O
for rep in 1 2; do
  for s in 0 1; do
    echo "== sched $s" >> $O
    ECDNA_SSA_SCHED=$s PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 200 python3 tools/probe_configs.py c2 c4 | grep "^{" >> $O
    ECDNA_SSA_SCHED=$s PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 | grep "^{" >> $O
  done
done
python3 - "$O" <<'PY'
import json, sys
cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.strip()
        continue
    d = json.loads(line)
    print(cur, d.get("config"), round(d["stepper_ms"], 1), "ms")
PY
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 300 python3 tools/sweep.py ECDNA_SSA_SCHED=2,0
