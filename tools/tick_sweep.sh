#!/bin/bash
# Rotation tick sweep (ECDNA_SSA_ROT_TICK = log2 iterations per tick) on a bench.py workload.
# Usage: bash tools/tick_sweep.sh <workload> "<ticks>"; results in gpurun_out/tick.txt
set -o pipefail
mkdir -p gpurun_out
for t in $2; do
  ECDNA_SSA_ROT_TICK=$t timeout -k 10 120 python bench.py --workload "$1" --no-cpu-baseline --steps 4 \
    > gpurun_out/tick_$1_$t.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/tick_$1_$t.json'));print('$1 tick',$t,round(d['config']['kernel_ms_avg'],1))" | tee -a gpurun_out/tick.txt
done
