#!/bin/bash
# Same-box A/B: the working-tree build vs ecdna-evo_amd/lib_ab/<ref>/ on C3 (sweep) and C2 + C5 shard.
# Usage: bash tools/ab_compare.sh <ref>   (build the ref first with tools/ab_build.sh <ref>)
set -euo pipefail
REF=${1:?ref}
cd "$GRAFT_REPO_ROOT"
B=$PWD/ecdna-evo_amd/lib_ab/$REF/libecdna_ssa.so
O=gpurun_out/ab_$REF; mkdir -p $O
timeout -k 10 600 python3 tools/sweep.py "ECDNA_SSA_LIB=,$B,,$B" > $O/c3.log 2>&1
for lib in "" "$B"; do
  tag=$([ -z "$lib" ] && echo tree || echo ref)
  ECDNA_SSA_LIB=$lib timeout -k 10 300 python3 tools/probe_configs.py c2 c5 > $O/probe_$tag.log 2>&1
done
echo done
