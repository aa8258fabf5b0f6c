set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A=base B=ph1 bash tools/r04_gpu7.sh
bash tools/r04_c4knobs.sh
