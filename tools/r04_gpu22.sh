#!/bin/bash
# Round 4: SQ instruction counts per wave-event of the C4 whole (K = 64 / u16) and C5 whole (K = 32 / u32) bench lines.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for w in c4 c5; do
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES \
    -T --output-format csv -d gpurun_out/pmc_$w -o pmc -- python3 bench.py --workload $w --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/pmc_$w.log 2>&1
  python3 tools/ab_pmc_summary.py gpurun_out/pmc_$w gpurun_out/pmc_$w.log "$w"
done
