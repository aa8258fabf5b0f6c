#!/bin/bash
# Round 4: the C4 8-GPU shard's sets by initial copy number (which sets set the critical path), K = 64.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/c4_sub.py 7 6 5 4 3 0
PROBE_KMAX=256 timeout -k 10 120 python3 tools/c4_sub.py 7
