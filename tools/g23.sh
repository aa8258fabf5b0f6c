set -euo pipefail
cd "$GRAFT_REPO_ROOT"
for R in 524288 1048576 2097152; do
  SWEEP_REPS=$R SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 200 python3 tools/sweep.py ECDNA_SSA_BLOCKS_PER_CU=3,4 > gpurun_out/g23_$R.log 2>&1
  echo R=$R; cat gpurun_out/g23_$R.log
done
