#!/bin/bash
# Stall breakdown of the stepper on the bench workload (one step): SQ wave-state and instruction
# counters, one rocprofv3 --pmc pass per group (no tracing combined). Every name here was checked
# against `rocprofv3 -L` on gfx950: an unknown counter aborts rocprofv3, which then hangs.
# Usage: bash tools/gpu_sq_profile.sh <tag>
set -euo pipefail
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sq_$TAG
mkdir -p $O
i=0
for group in \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_WAVES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU" \
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group -T --output-format csv -d $O/p$i -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/p$i.log 2>&1
  echo "pass $i done"
done
