set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for C in 0 1; do
  ECDNA_SSA_BIN_C32=$C SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4 > gpurun_out/g19_c$C.log 2>&1
  echo C32=$C; cat gpurun_out/g19_c$C.log
done
