set -euo pipefail
cd "$GRAFT_REPO_ROOT"
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4 > gpurun_out/g22.log 2>&1
cat gpurun_out/g22.log
