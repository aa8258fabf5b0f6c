#!/bin/bash
# Build libecdna_ssa.so from the kernel/ABI sources of a git ref into ecdna-evo_amd/lib_ab/<ref>/,
# for a same-box A/B against the working tree (ECDNA_SSA_LIB=<that path> python tools/sweep.py ...).
# Usage: [EXTRA=-DFLAG] [ILP_STRATEGY=max-ilp] bash tools/ab_build.sh <git-ref or WORKTREE> [out-name]
set -euo pipefail
REF=${1:?git ref}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/ecdna-evo_amd/lib_ab/${2:-$REF}
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
if [ "$REF" = WORKTREE ]; then mkdir -p "$TMP/ecdna-evo_amd"; cp -r "$ROOT/ecdna-evo_amd/csrc" "$TMP/ecdna-evo_amd/"; cp -r "$ROOT/include" "$TMP/"; else git -C "$ROOT" archive "$REF" ecdna-evo_amd/csrc include | tar -x -C "$TMP"; fi
mkdir -p "$OUT"
cd "$TMP/ecdna-evo_amd"
for f in csrc/*.hip csrc/*.cpp; do
  x=""; [ "${f##*.}" = cpp ] && x="-x hip"
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Werror=uninitialized ${EXTRA:-} $x -c "$f" -o "$TMP/$(basename "$f").o"
done
if grep -q ECDNA_ILP_BUILD csrc/ssa_kernels.hip; then  # (refs since the two-schedule build)
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -Werror=uninitialized ${EXTRA:-} -DECDNA_ILP_BUILD \
    -mllvm -amdgpu-sched-strategy=${ILP_STRATEGY:-max-ilp} -c csrc/ssa_kernels.hip -o "$TMP/ssa_kernels_ilp.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libecdna_ssa.so" "$TMP"/*.o -ldl
echo "$OUT/libecdna_ssa.so"
