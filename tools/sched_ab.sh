#!/bin/bash
# Same-box A/B of the bin stepper's schedules (ECDNA_SSA_SCHED) on bench.py workloads.
# Usage: bash tools/sched_ab.sh "<workload>:<steps>:<sched> ..."; results in gpurun_out/sched_ab.txt
set -o pipefail
mkdir -p gpurun_out
for item in $1; do
  IFS=: read -r w k s <<< "$item"
  ECDNA_SSA_SCHED=$s timeout -k 10 300 python bench.py --workload "$w" --steps "$k" --warmup 1 --no-cpu-baseline \
    > gpurun_out/sched_${w}_$s.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sched_${w}_$s.json'));print('$w','sched',$s,'kernel ms',round(d['config']['kernel_ms_avg'],1),'lanes',d['config']['grid_lanes'],'value',d['value'])" | tee -a gpurun_out/sched_ab.txt
done
