#!/bin/bash
# Round 4 same-box A/B: parity of the working tree's library, then C3 (K = 32), the latency-bound shapes (C2, C4
# and C5 rank-0 shards) and one SQ-counter pass per library (VALU / SALU / LDS instructions of one C3 step) for
# prebuilt libraries ecdna-evo_amd/lib_ab/<name>/ (tools/ab_build.sh).
# Usage: [SKIP_PARITY=1] [SKIP_LATENCY=1] bash tools/r04_ab.sh <name>...
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "${SKIP_PARITY:-}" ]; then
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py tests/test_gpu_rotation.py \
  tests/test_gpu_drain.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -1 gpurun_out/ab_parity.log
fi
bash tools/ab_libs.sh "$@" > gpurun_out/ab_c3.log 2>&1
cat gpurun_out/ab_c3.log
if [ -z "${SKIP_LATENCY:-}" ]; then
bash tools/ab_latency.sh "$@" 2>&1 | tail -24
fi
for n in "$@"; do
  L=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so
  ECDNA_SSA_LIB=$L timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES \
    -T --output-format csv -d gpurun_out/ab_pmc_$n -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/ab_pmc_$n.log 2>&1
  tail -1 gpurun_out/ab_pmc_$n.log
  python3 tools/ab_pmc_summary.py gpurun_out/ab_pmc_$n gpurun_out/ab_pmc_$n.log "$n"
done
