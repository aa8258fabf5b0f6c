#!/bin/bash
# Round 4: parity of lib_ab/$B, then A and B on the whole C5 sweep (twice, interleaved), the C5 shard and C3.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A=${A:-base}; B=${B:-ahead32}
L=$PWD/ecdna-evo_amd/lib_ab
ECDNA_SSA_LIB=$L/$B/libecdna_ssa.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py \
  tests/test_gpu_rotation.py tests/test_gpu_drain.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ab_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/ab_parity.log; exit 1; }
tail -1 gpurun_out/ab_parity.log
for rep in 1 2; do for n in $A $B; do
  ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 300 python3 tools/probe_configs.py c5 |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$n c5 whole', round(d['stepper_ms'],1), 'ms')"
  ECDNA_SSA_LIB=$L/$n/libecdna_ssa.so PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 200 python3 tools/probe_configs.py c5 |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$n c5 shard', round(d['stepper_ms'],1), 'ms')"
done; done
bash tools/ab_libs.sh $A $B 2>&1 | grep "^{"
