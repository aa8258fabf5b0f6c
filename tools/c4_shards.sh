#!/bin/bash
# All eight C4 shards (ABC sweep, 8-GPU layout) one after another on this GPU: the 8-GPU makespan is the
# slowest shard. PROBE_SHARD=interleaved (default) or contiguous; K = 64 (PROBE_KMAX).
# Usage: [PROBE_SHARD=contiguous] bash tools/c4_shards.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/c4_shards_${PROBE_SHARD:-interleaved}.log; : > $O
for r in 0 1 2 3 4 5 6 7; do
  PROBE_RANK=$r PROBE_FLAGS=0x20 PROBE_KMAX=${PROBE_KMAX:-64} timeout -k 10 120 python3 tools/probe_configs.py c4 | grep "^{" >> $O
done
python3 -c "
import json
ds=[json.loads(l) for l in open('$O')]
for r,d in enumerate(ds): print('rank', r, round(d['stepper_ms'],1), 'ms', d['events'], 'events', '%.3e' % d['events_per_s_kernel'])
ms=[d['stepper_ms'] for d in ds]; ev=sum(d['events'] for d in ds)
print('makespan', round(max(ms),1), 'ms  mean', round(sum(ms)/len(ms),1), 'ms  8-GPU events/s', '%.3e' % (ev/max(ms)*1e3))"
