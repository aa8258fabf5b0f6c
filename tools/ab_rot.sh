#!/bin/bash
# Same-box A/B of rotation variants on C3: the tree vs lib_ab/<names...>, rotation on (tick 11) and off.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=""
for n in "$@"; do L="$L,$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so"; done
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 900 python3 tools/sweep.py "ECDNA_SSA_LIB=$L" ECDNA_SSA_ROTATE=2,0 > gpurun_out/ab_rot.log 2>&1
cat gpurun_out/ab_rot.log
