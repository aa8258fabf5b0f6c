set -euo pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -m pytest tests/test_gpu_parity.py -q -x -k "bin" > gpurun_out/g24_parity.log 2>&1 || { echo PARITY FAILED; tail -60 gpurun_out/g24_parity.log; exit 1; }
echo parity ok; tail -1 gpurun_out/g24_parity.log
for P in 0 16 32 48; do
  ECDNA_SSA_PARK_BELOW=$P SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=4 > gpurun_out/g24_p$P.log 2>&1
  echo PARK_BELOW=$P; cat gpurun_out/g24_p$P.log
done
