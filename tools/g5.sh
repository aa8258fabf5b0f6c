set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -x -k "bin" > gpurun_out/g5_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/g5_parity.log; exit 1; }
echo parity ok; tail -2 gpurun_out/g5_parity.log
timeout -k 10 300 python3 tools/probe.py c2bins c3bins > gpurun_out/g5_probe.log 2>&1
grep "rep 1" gpurun_out/g5_probe.log
