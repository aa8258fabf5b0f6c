#!/bin/bash
# Same-box A/B of prebuilt libraries (ecdna-evo_amd/lib_ab/<name>/) on the latency-bound shapes: C2, the
# C4 rank-0 shard (K = 32) and the C5 rank-0 shard (K = 64), twice each, interleaved.
# Usage: bash tools/ab_latency.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_latency.log; mkdir -p gpurun_out; : > $O
for rep in 1 2; do
  for n in "$@"; do
    L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
    echo "== $n" >> $O
    ECDNA_SSA_LIB=$L PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 200 python3 tools/probe_configs.py c2 c4 | grep "^{" >> $O
    ECDNA_SSA_LIB=$L PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 | grep "^{" >> $O
  done
done
python3 - "$O" <<'PY'
import json, sys
cur = None
for line in open(sys.argv[1]):
    if line.startswith("=="):
        cur = line.split()[1]
        continue
    d = json.loads(line)
    print(cur, d.get("config"), round(d["stepper_ms"], 1), "ms")
PY
