#!/bin/bash
# Rotation: parity (rotation cases + bin-store parity) then C3 tuning sweeps of tick and park threshold.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rotation.py tests/test_gpu_parity.py -k "rotation or bin" -x -q --timeout 120 --timeout-method thread > gpurun_out/rot_tests.log 2>&1 || { echo TESTS FAILED; tail -60 gpurun_out/rot_tests.log; exit 1; }
tail -1 gpurun_out/rot_tests.log
O=gpurun_out/rot_sweep.log
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 900 python3 tools/sweep.py ECDNA_SSA_ROT_TICK=${TICKS:-10,11,12} ECDNA_SSA_ROT_PARK_MIN=${PMINS:-16384,32768,65536,98304} > $O 2>&1
cat $O
