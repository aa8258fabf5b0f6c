#!/bin/bash
# C4 rank-0 shard (8-GPU layout) and the whole C4 on one GPU at K = 32 / 64 / 256 (bin store).
# Usage: bash tools/c4_kmax.sh
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
O=gpurun_out/c4_kmax.log; : > $O
for k in 32 64 256; do
  PROBE_FLAGS=0x20 PROBE_KMAX=$k timeout -k 10 200 python3 tools/probe_configs.py c4 | grep "^{" | sed "s/^/shard K=$k /" >> $O
  PROBE_FLAGS=0x20 PROBE_KMAX=$k PROBE_GPUS=1 timeout -k 10 300 python3 tools/probe_configs.py c4 | grep "^{" | sed "s/^/whole K=$k /" >> $O
done
cut -c1-200 $O
