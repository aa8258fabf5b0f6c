set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py -q -x > gpurun_out/g16_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/g16_parity.log; exit 1; }
echo parity ok; tail -1 gpurun_out/g16_parity.log
timeout -k 10 300 python3 tools/probe.py c2bins c3bins > gpurun_out/g16_probe.log 2>&1
grep "rep 1" gpurun_out/g16_probe.log
PROBE_FLAGS=0x20 timeout -k 10 300 python3 tools/probe_configs.py c4 c5 > gpurun_out/g16_c45.log 2>&1
cat gpurun_out/g16_c45.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['config'], round(d['stepper_ms'],1), '%.3e' % d['events_per_s_kernel'])"
