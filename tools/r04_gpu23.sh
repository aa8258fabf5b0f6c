#!/bin/bash
# Round 4, final sources: the eight C4 shards (8-GPU layout, K = 64) one after another, then the eight C5 shards.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/c4_shards.sh
for r in 0 1 2 3 4 5 6 7; do
  PROBE_RANK=$r PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 120 python3 tools/probe_configs.py c5 |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('c5 rank $r', round(d['stepper_ms'],1), 'ms', d['events'], 'events', 'err', d['errors'])"
done
