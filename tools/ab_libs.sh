#!/bin/bash
# Same-box A/B of several prebuilt libraries (ecdna-evo_amd/lib_ab/<name>/) on C3 with the bin store (K = 32), interleaved
# twice. Usage: bash tools/ab_libs.sh <name>...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
L=""
for n in "$@"; do L="$L,$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so"; done
L=${L#,}
O=gpurun_out/ab_libs; mkdir -p $O
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 900 python3 tools/sweep.py "ECDNA_SSA_LIB=$L,$L" > $O/c3.log 2>&1
cat $O/c3.log
