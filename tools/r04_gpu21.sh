#!/bin/bash
# Round 4: the C5 K rule at the 2- and 4-GPU shard sizes (K = 32 against 64), and the whole C4 sweep at K = 32 / 64.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pr() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['stepper_ms'],1), 'ms', d['geometry'], 'err', d['errors'])"; }
for g in 2 4; do for k in 32 64; do
  PROBE_GPUS=$g PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 200 python3 tools/probe_configs.py c5 | pr "c5 ${g}-GPU shard K=$k"
done; done
for k in 32 64; do
  PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 200 python3 tools/probe_configs.py c4 | pr "c4 whole K=$k"
done
