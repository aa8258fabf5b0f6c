#!/bin/bash
# Build the working tree's libecdna_ssa.so with extra compile flags into ecdna-evo_amd/lib_ab/<tag>/
# (experiments: same-box comparison through ECDNA_SSA_LIB). Usage: bash tools/variant_build.sh <tag> [flags...]
set -euo pipefail
TAG=${1:?tag}; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/ecdna-evo_amd/lib_ab/$TAG
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
mkdir -p "$OUT"
cd "$ROOT/ecdna-evo_amd"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off "$@" -c csrc/ssa_kernels.hip -o "$TMP/k.o"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off "$@" -x hip -c csrc/ssa_api.cpp -o "$TMP/a.o"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off "$@" -DECDNA_ILP_BUILD \
  -mllvm -amdgpu-sched-strategy=max-ilp -c csrc/ssa_kernels.hip -o "$TMP/ki.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libecdna_ssa.so" "$TMP"/*.o
echo "$OUT/libecdna_ssa.so"
