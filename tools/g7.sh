set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py -q -x > gpurun_out/g7_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/g7_parity.log; exit 1; }
echo parity ok; tail -1 gpurun_out/g7_parity.log
timeout -k 10 300 python3 tools/probe.py c2bins c3bins > gpurun_out/g7_probe.log 2>&1
grep "rep 1" gpurun_out/g7_probe.log
PMC_GROUPS=tools/pmc_groups_sq.txt bash tools/pmc_probe.sh ${TAG:-g7} python3 tools/probe.py c3bins1
