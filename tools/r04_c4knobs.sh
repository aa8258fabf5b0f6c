#!/bin/bash
# C4 8-GPU rank-0 shard (K = 64) under the engine's launch knobs, twice each (development sweep).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() { env "$@" PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c4 |
  python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$*', round(d['stepper_ms'],1), 'ms')"; }
for rep in 1 2; do
  run X=auto
  run ECDNA_SSA_ADMIT=0
  run ECDNA_SSA_ADMIT_SLOTS=2
  run ECDNA_SSA_ROTATE=1
  run ECDNA_SSA_BLOCKS_PER_CU=2
  run PROBE_COST_HINT=0
  run ECDNA_SSA_SCHED=0
  run ECDNA_SSA_SCHED=0 ECDNA_SSA_BLOCKS_PER_CU=3
  run ECDNA_SSA_C32=1
  run ECDNA_SSA_C32=1 ECDNA_SSA_SCHED=0
done
