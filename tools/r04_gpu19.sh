#!/bin/bash
# Round 4 final check (after r04r): the full GPU suite, smoke, the default bench line, the profile set, the C5 bench
# line, then the C5 K = 32 / 64 probe (informational).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/round_check.sh
bash tools/gpu_profile.sh r04s bins
timeout -k 10 400 python3 bench.py --workload c5 --no-cpu-baseline > gpurun_out/r04s_bench_c5.json 2> gpurun_out/r04s_bench_c5.err; cat gpurun_out/r04s_bench_c5.json
bash tools/r04_gpu18.sh
