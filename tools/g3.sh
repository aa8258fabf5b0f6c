set -euo pipefail
cd "$GRAFT_REPO_ROOT"
PMC_GROUPS=tools/pmc_groups_lds.txt bash tools/pmc_probe.sh binsA python3 tools/probe.py c3bins1
grep -h -E "LDS|SQ_" gpurun_out/pmc_binsA/avail.txt | head -400 > gpurun_out/pmc_binsA/avail_sq.txt || true
