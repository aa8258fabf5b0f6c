set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -x -k "bin" > gpurun_out/g18_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/g18_parity.log; exit 1; }
echo parity ok; tail -1 gpurun_out/g18_parity.log
for K in 32 64; do
  SWEEP_FLAGS=0x20 SWEEP_KMAX=$K timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4,5 > gpurun_out/g18_k$K.log 2>&1
  echo K=$K; cat gpurun_out/g18_k$K.log
done
PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 300 python3 tools/probe_configs.py c2 c4 > gpurun_out/g18_c24.log 2>&1
cat gpurun_out/g18_c24.log | python3 -c "
import sys, json
for l in sys.stdin:
    if l.startswith('{'):
        d = json.loads(l); print(d['config'], 'K32', round(d['stepper_ms'],1), '%.3e' % d['events_per_s_kernel'])"
