#!/bin/bash
# Same-box A/B of prebuilt libraries (ecdna-evo_amd/lib_ab/<name>/) on the bench's C4 shapes: the 8-GPU rank-0 shard
# split by initial copy number (tools/c4_split.py, bench caps) and the whole sweep's bench line, twice each, interleaved.
# Usage: bash tools/ab_c4.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  for n in "$@"; do
    L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
    ECDNA_SSA_LIB=$L C4S_SPLITS=7 C4S_BLOCKS=336:624 timeout -k 10 300 python3 tools/c4_split.py 2>/dev/null | python3 -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print('$n', 'c4 8-GPU rank 0', d['setting'], round(d['makespan_ms'], 1), 'ms')"
    ECDNA_SSA_LIB=$L timeout -k 10 300 python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().splitlines()[-1]); print('$n', 'c4 whole bench step', round(d['ms_per_step'], 1), 'ms')"
  done
done
