set -euo pipefail
cd "$GRAFT_REPO_ROOT"
SWEEP_FLAGS=0x20 timeout -k 10 300 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=2,3,4 > gpurun_out/g15.log 2>&1
cat gpurun_out/g15.log
