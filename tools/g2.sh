set -euo pipefail
cd "$GRAFT_REPO_ROOT"
SWEEP_FLAGS=0x20 timeout -k 10 400 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=1,2,3,4,5,6 > gpurun_out/g2_sweep.log 2>&1
cat gpurun_out/g2_sweep.log
