set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/round_check.sh
bash tools/gpu_profile.sh r04e bins
