set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -x -k "bin" > gpurun_out/g25_parity.log 2>&1 || { echo PARITY FAILED; tail -40 gpurun_out/g25_parity.log; exit 1; }
echo parity ok; tail -1 gpurun_out/g25_parity.log
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4 > gpurun_out/g25.log 2>&1
cat gpurun_out/g25.log
