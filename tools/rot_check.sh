#!/bin/bash
# Rotation bring-up on one GPU box: rotation parity, bin-store parity, then C3 timings: the tree with
# rotation off / on (tick sweep) against the HEAD build (tools/ab_build.sh HEAD).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rotation.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rot_tests.log 2>&1 || { echo ROTATION TESTS FAILED; tail -60 gpurun_out/rot_tests.log; exit 1; }
tail -2 gpurun_out/rot_tests.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k bin -x -q --timeout 300 --timeout-method thread > gpurun_out/rot_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/rot_parity.log; exit 1; }
tail -2 gpurun_out/rot_parity.log
B=$PWD/ecdna-evo_amd/lib_ab/HEAD/libecdna_ssa.so
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 600 python3 tools/sweep.py "ECDNA_SSA_LIB=$B," ECDNA_SSA_ROTATE=0,2 > gpurun_out/rot_c3.log 2>&1
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 600 python3 tools/sweep.py ECDNA_SSA_ROTATE=2 ECDNA_SSA_ROT_TICK=9,10,12,13 >> gpurun_out/rot_c3.log 2>&1
cat gpurun_out/rot_c3.log
