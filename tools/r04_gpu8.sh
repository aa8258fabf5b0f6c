set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ECDNA_SSA_PAIR_OWNERS=16 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "paired or fast_forward" --timeout 300 --timeout-method thread > gpurun_out/po_parity.log 2>&1 || { echo PARITY FAILED; tail -30 gpurun_out/po_parity.log; exit 1; }
tail -1 gpurun_out/po_parity.log
bash tools/r04_po.sh po
