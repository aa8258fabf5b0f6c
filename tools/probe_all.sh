#!/bin/bash
# Stepper throughput on the C2 / C3 / C4-shard / C5-shard shapes, bin store K = 32, rotation auto and off.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 2 0; do
  ECDNA_SSA_ROTATE=$r PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 600 python3 tools/probe_configs.py ${CFGS:-c2 c3 c4 c5} > gpurun_out/probe_rot$r.log 2>&1
  python3 -c "
import json
for l in open('gpurun_out/probe_rot$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('rot=$r', d['config'], round(d['stepper_ms'],2), '%.4e' % d['events_per_s_kernel'])"
done
