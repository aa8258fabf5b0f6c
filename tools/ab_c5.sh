#!/bin/bash
# Same-box A/B of prebuilt libraries on the C5 rank-0 shard (K = 64), twice each, interleaved.
# Usage: bash tools/ab_c5.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for n in "$@"; do
    L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
    echo -n "$n "
    ECDNA_SSA_LIB=$L PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 | grep "^{" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['stepper_ms'],1), 'ms')"
  done
done
