#!/bin/bash
# Round 4 final check: the full GPU suite, smoke, the default bench line, then the profile set (kernel trace, PMC).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/round_check.sh
bash tools/gpu_profile.sh r04q bins
for w in c2 c4 c5; do timeout -k 10 400 python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/r04q_bench_$w.json 2> gpurun_out/r04q_bench_$w.err; cat gpurun_out/r04q_bench_$w.json; done
