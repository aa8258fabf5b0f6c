#!/bin/bash
# A/B: stepper with and without the LDS tail window on the C3 bench, plus PMC passes of the window variant.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_window; mkdir -p $O
timeout -k 10 600 python3 -m pytest tests/ -q -m gpu -x > $O/gpu_tests.log 2>&1
echo tests ok
ECDNA_SSA_WINDOW=0 timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_nowin.json 2>/dev/null
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_win.json 2>/dev/null
echo bench ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write.log 2>&1
echo pmc ok
