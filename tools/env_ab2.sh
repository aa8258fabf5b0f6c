#!/bin/bash
# C4 whole: rotation on/off under both K = 64 builds (default 130-VGPR and 128-VGPR), alternating.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for sc in 0 3; do
    for r in 2 0; do
      ECDNA_SSA_SCHED=$sc ECDNA_SSA_ROTATE=$r timeout -k 10 120 python bench.py --workload c4 --no-cpu-baseline --steps 3 \
        > gpurun_out/ab2.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('gpurun_out/ab2.json'));print('c4 sched=$sc rotate=$r',round(d['config']['kernel_ms_avg'],1))" | tee -a gpurun_out/env_ab2.txt
    done
  done
done
