#!/bin/bash
# Round 4: C5 (whole run on one GPU and the 8-GPU rank-0 shard) at K = 32 against K = 64, interleaved.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
pr() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['stepper_ms'],1), 'ms', d['geometry'], 'err', d['errors'], 'stops', d['stops'])"; }
for k in 32 64; do
  PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 300 python3 tools/probe_configs.py c5 | pr "c5 whole K=$k"
  PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 200 python3 tools/probe_configs.py c5 | pr "c5 shard K=$k"
done
