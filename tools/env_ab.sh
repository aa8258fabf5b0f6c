#!/bin/bash
# Same-box A/B of one environment knob on a bench.py workload, alternating settings.
# Usage: bash tools/env_ab.sh <workload> <VAR> "<values>" <repeats>; results in gpurun_out/env_ab.txt
set -o pipefail
mkdir -p gpurun_out
for i in $(seq "$4"); do
  for v in $3; do
    env "$2=$v" timeout -k 10 120 python bench.py --workload "$1" --no-cpu-baseline --steps 3 \
      > gpurun_out/envab_$1_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/envab_$1_$v.json'));print('$1 $2=$v',round(d['config']['kernel_ms_avg'],1))" | tee -a gpurun_out/env_ab.txt
  done
done
