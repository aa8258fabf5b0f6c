#!/bin/bash
# Round 4: where the C4 shard's critical path goes: loop-section cycles (c4k7: the k0 = 128 sets, c4k0: k0 = 1) and
# rare-block fractions (k0 = 128, default schedule) of instrumented builds (lib_ab/cyc, lib_ab/pstats).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
L=$PWD/ecdna-evo_amd/lib_ab
ECDNA_SSA_LIB=$L/cyc/libecdna_ssa.so timeout -k 10 120 python3 tools/cycle_stats.py c4k7
ECDNA_SSA_LIB=$L/cyc/libecdna_ssa.so timeout -k 10 120 python3 tools/cycle_stats.py c4k0
ECDNA_SSA_LIB=$L/pstats/libecdna_ssa.so ECDNA_SSA_SCHED=0 timeout -k 10 120 python3 tools/path_stats.py c4k7
