#!/bin/bash
# Parity (all GPU tests) and an A/B of the speculative next-event load (auto / off / on) on C3, a
# 65,536-replicate C3 shard and C2; then the default bench line.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_prefetch; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests/ -q -m gpu -x > $O/gpu_tests.log 2>&1
echo tests ok
timeout -k 10 600 python3 tools/sweep.py ECDNA_SSA_PREFETCH=,0,1 > $O/c3.log 2>&1
SWEEP_REPS=65536 timeout -k 10 300 python3 tools/sweep.py ECDNA_SSA_PREFETCH=,0,1 > $O/c3_65k.log 2>&1
ECDNA_SSA_PREFETCH=0 timeout -k 10 300 python3 tools/probe_configs.py c2 > $O/c2_off.log 2>&1
timeout -k 10 300 python3 tools/probe_configs.py c2 > $O/c2_auto.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
echo done
