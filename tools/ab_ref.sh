#!/bin/bash
# Same-box A/B of prebuilt libraries (ecdna-evo_amd/lib_ab/<name>/) on the reference-draws C3 line (bench.py --store rows
# --draws reference: ssa_stepper_refdraws over 2^20 replicates), interleaved twice. Usage: bash tools/ab_ref.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for n in "$@"; do
    ECDNA_SSA_LIB=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so timeout -k 10 300 python3 bench.py --store rows \
      --draws reference --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "
import json, sys
d = json.loads(sys.stdin.readline())
print('$n', 'rep $rep', 'kernel_ms %.1f' % d['config']['kernel_ms_avg'], 'events/s %.4g' % d['value'],
      'vgprs', d['config']['instance']['vgprs'], 'lds', d['config']['instance']['lds_bytes'],
      'blocks_per_cu', d['config']['instance']['blocks_per_cu'])"
  done
done
