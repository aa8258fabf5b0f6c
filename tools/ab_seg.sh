#!/bin/bash
# Same-box A/B of prebuilt libraries (ecdna-evo_amd/lib_ab/<name>/) on C3 (bin store, K = 32) under each
# segregation rule (abi.SEG_*: 0 deterministic, 1 binomial, 2 binomial without uneven, 3 binomial without N-).
# Usage: bash tools/ab_seg.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for seg in 0 1 2 3; do
  for n in "$@"; do
    L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
    r=$(ECDNA_SSA_LIB=$L PROBE_SEG=$seg PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 200 python3 tools/probe_configs.py c3 | grep "^{")
    echo "$n seg$seg $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["stepper_ms"],1), "ms", d["events"], "events")')"
  done
done
