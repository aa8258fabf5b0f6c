set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A=${A:-chm}; B=${B:-ffm}
bash tools/r04_ab.sh $A $B
for n in $A $B; do
  ECDNA_SSA_LIB=$PWD/ecdna-evo_amd/lib_ab/$n/libecdna_ssa.so PROBE_GPUS=1 PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 300 python3 tools/probe_configs.py c5 |
    python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$n c5 whole', round(d['stepper_ms'],1), 'ms')"
done
