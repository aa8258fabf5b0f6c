set -euo pipefail
cd "$GRAFT_REPO_ROOT"
PMC_GROUPS=tools/pmc_groups_mix.txt bash tools/pmc_probe.sh g11 python3 tools/probe.py c3bins1
