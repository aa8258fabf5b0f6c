set -euo pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 900 python3 tools/sweep.py SWEEP_REPS=524288,1048576,2097152,4194304 ECDNA_SSA_ROTATE=2,0 > gpurun_out/ns2.log 2>&1
cat gpurun_out/ns2.log
