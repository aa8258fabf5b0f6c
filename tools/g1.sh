set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py -q -x > gpurun_out/g1_parity.log 2>&1 || { echo PARITY FAILED; tail -50 gpurun_out/g1_parity.log; exit 1; }
echo parity ok; tail -3 gpurun_out/g1_parity.log
timeout -k 10 300 python3 tools/probe.py c2bins c3bins > gpurun_out/g1_probe.log 2>&1
cat gpurun_out/g1_probe.log
