#!/bin/bash
# Schedule sweep of the bin stepper on every bench workload (ECDNA_SSA_SCHED: 0 occupancy-first, 1 max-ILP, 3 the
# 128-VGPR K = 64 / u16 build; ECDNA_SSA_PAIR for the paired lanes), for re-tuning ecdna_ssa_ctx_create's auto
# rules after a register-count change. Usage: bash tools/r04_sched.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sched; mkdir -p $O
p() { python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$1', round(d['stepper_ms'],1), 'ms')"; }
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 300 python3 tools/sweep.py ECDNA_SSA_SCHED=0,1,0,1 | tee $O/c3.log
for S in 0 1; do
  ECDNA_SSA_SCHED=$S PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 200 python3 tools/probe_configs.py c2 | p "c2 sched=$S"
  ECDNA_SSA_SCHED=$S PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c4 | p "c4-shard(K64) sched=$S"
  ECDNA_SSA_SCHED=$S PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c4 | p "c4-shard(K64) sched=$S"
done
ECDNA_SSA_SCHED=2 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 | p "c5-shard pair(auto)"
ECDNA_SSA_SCHED=1 ECDNA_SSA_PAIR=0 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 | p "c5-shard ilp-unpaired"
for S in 0 1 3; do
  ECDNA_SSA_SCHED=$S PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 300 python3 tools/probe_configs.py c4 | p "c4-whole sched=$S"
done
for S in 0 1; do
  ECDNA_SSA_SCHED=$S PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 300 python3 tools/probe_configs.py c5 | p "c5-whole sched=$S"
done
