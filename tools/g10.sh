set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python3 -m pytest tests -m gpu -q -x --durations=15 > gpurun_out/g10_gpu_tests.log 2>&1 || { echo GPU TESTS FAILED; tail -80 gpurun_out/g10_gpu_tests.log; exit 1; }
echo gpu tests ok; tail -25 gpurun_out/g10_gpu_tests.log
timeout -k 10 300 python3 tools/probe.py c2bins c3bins > gpurun_out/g10_probe.log 2>&1
grep "rep 1" gpurun_out/g10_probe.log
