set -euo pipefail
cd "$GRAFT_REPO_ROOT"
SWEEP_FLAGS=0x20 ECDNA_SSA_LIB=$PWD/ecdna-evo_amd/lib_ab/k32/libecdna_ssa.so timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4,5 > gpurun_out/g9_k32.log 2>&1
cat gpurun_out/g9_k32.log
