set -euo pipefail
cd "$GRAFT_REPO_ROOT"
head -2 tools/pmc_groups_lds.txt > /tmp/grp.txt
ECDNA_SSA_BLOCKS_PER_CU=4 PMC_GROUPS=/tmp/grp.txt bash tools/pmc_probe.sh binsB python3 tools/probe.py c3bins1
cat gpurun_out/pmc_binsB/p1.log | grep -E "C3|rep" || true
