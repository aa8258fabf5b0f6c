#!/bin/bash
# Round-end rehearsal on one GPU box: the full -m gpu suite, smoke(), and the default bench line.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/rc_tests.log 2>&1
echo "tests ok"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/rc_smoke.log 2>&1
echo "smoke ok"
timeout -k 10 400 python3 bench.py > gpurun_out/rc_bench.json 2> gpurun_out/rc_bench.err
cat gpurun_out/rc_bench.json
