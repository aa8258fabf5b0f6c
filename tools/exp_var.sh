#!/bin/bash
# C3 bin-store timings of several builds (ECDNA_SSA_LIB list), rotation off unless SWEEP_SEG is set.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
L=$PWD/ecdna-evo_amd/lib_ab
O=gpurun_out/exp_var; mkdir -p $O
libs=""
for v in "$@"; do if [ "$v" = tree ]; then libs="$libs,"; else libs="$libs,$L/$v/libecdna_ssa.so"; fi; done
SWEEP_SEG=${SWEEP_SEG:--1} SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 600 python3 tools/sweep.py "ECDNA_SSA_LIB=${libs#,}" > $O/c3.log 2>&1
cat $O/c3.log | sed "s#$L/##"
