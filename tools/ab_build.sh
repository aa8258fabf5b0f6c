#!/bin/bash
# Build libecdna_ssa.so from the kernel/ABI sources of a git ref into ecdna-evo_amd/lib_ab/<ref>/,
# for a same-box A/B against the working tree (ECDNA_SSA_LIB=<that path> python tools/sweep.py ...).
# Usage: bash tools/ab_build.sh <git-ref>
set -euo pipefail
REF=${1:?git ref}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/ecdna-evo_amd/lib_ab/$REF
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$REF" ecdna-evo_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$OUT"
cd "$TMP/ecdna-evo_amd"
for f in csrc/ssa_kernels.hip csrc/ssa_api.cpp; do
  x=""; [ "${f##*.}" = cpp ] && x="-x hip"
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off $x -c "$f" -o "$TMP/$(basename "$f").o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libecdna_ssa.so" "$TMP"/*.o
echo "$OUT/libecdna_ssa.so"
