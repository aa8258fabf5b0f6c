#!/bin/bash
# C5 8-GPU rank-0 shard under paired lanes with 32 / 16 / 8 owners per wave (ECDNA_SSA_PAIR_OWNERS: fewer owners per
# wave, more waves per SIMD), and the C4 rank-0 shard (K = 64) for reference. Usage: bash tools/r04_po.sh [lib name]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/ecdna-evo_amd/lib_ab/${1:-po}/libecdna_ssa.so
for rep in 1 2; do
for PO in 32 16 8; do
  ECDNA_SSA_LIB=$L ECDNA_SSA_PAIR_OWNERS=$PO PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c5 shard owners/wave=$PO', round(d['stepper_ms'],1), 'ms', d.get('geometry'))"
done
done
