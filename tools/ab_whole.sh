#!/bin/bash
# Same-box A/B of prebuilt libraries on whole configs on one GPU: C4 (K = 64) and C5 (K = 64).
# Usage: bash tools/ab_whole.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for n in "$@"; do
  L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
  for c in c4 c5; do
    ECDNA_SSA_LIB=$L PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py $c |
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', '$c whole', round(d['stepper_ms'],1), 'ms')"
  done
done
