#!/bin/bash
# Round 4: the C4 8-GPU rank-0 shard at K = 64 and K = 256 (the costliest sets' cells, k0 = 128, sit above 64), twice
# each interleaved, then the whole C4 sweep at K = 256.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
pr() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['stepper_ms'],1), 'ms', d['geometry'], 'err', d['errors'])"; }
for rep in 1 2; do for k in 64 256; do
  PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 200 python3 tools/probe_configs.py c4 | pr "c4 shard K=$k"
done; done
PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=256 timeout -k 10 300 python3 tools/probe_configs.py c4 | pr "c4 whole K=256"
