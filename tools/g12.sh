set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/probe_configs.py c4 c5 > gpurun_out/g12_rows.log 2>&1
PROBE_FLAGS=0x20 timeout -k 10 300 python3 tools/probe_configs.py c2 c4 c5 > gpurun_out/g12_bins64.log 2>&1
PROBE_FLAGS=0x20 PROBE_KMAX=256 timeout -k 10 300 python3 tools/probe_configs.py c2 c3 c4 c5 > gpurun_out/g12_bins256.log 2>&1
cat gpurun_out/g12_*.log | grep config | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'], d['flags'], d['bin_kmax'], round(d['stepper_ms'],1), '%.3e' % d['events_per_s_kernel'], d['geometry'])"
