#!/bin/bash
# Round 3 same-box A/B: parity of the working tree, then C3 (K = 32) and the latency-bound shapes (C2, C4 and
# C5 rank-0 shards) for prebuilt libraries ecdna-evo_amd/lib_ab/<name>/ (tools/ab_build.sh).
# Usage: bash tools/r03_ab.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py tests/test_gpu_rotation.py \
  tests/test_gpu_drain.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -1 gpurun_out/ab_parity.log
bash tools/ab_libs.sh "$@" > gpurun_out/ab_c3.log 2>&1
cat gpurun_out/ab_c3.log
bash tools/ab_latency.sh "$@" 2>&1 | tail -20
