#!/bin/bash
# Round 4 final check (after the C5 K rule and the kAhead-only block reuse): the full GPU suite (with the new C5
# whole-instance test), smoke, the default bench line, the profile set, and the C5 bench line.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/round_check.sh
bash tools/gpu_profile.sh r04t bins
timeout -k 10 400 python3 bench.py --workload c5 --no-cpu-baseline > gpurun_out/r04t_bench_c5.json 2> gpurun_out/r04t_bench_c5.err; cat gpurun_out/r04t_bench_c5.json
