set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c_gputests.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/r04c_gputests.log; exit 1; }
tail -2 gpurun_out/r04c_gputests.log
SKIP_PARITY=1 bash tools/r04_ab.sh base v6
