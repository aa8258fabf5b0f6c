#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per counter group, counters filtered against `rocprofv3 -L` so an
# unknown name never reaches rocprofv3) over a probe command. Usage: bash tools/pmc_probe.sh <tag> <cmd...>
set -euo pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_$TAG
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/avail.txt 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  keep=""
  for c in $group; do
    if grep -q -w "$c" $O/avail.txt; then keep="$keep $c"; else echo "skip unknown counter $c"; fi
  done
  [ -z "$keep" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $keep -T --output-format csv -d $O/p$i -o pmc -- "$@" > $O/p$i.log 2>&1
  echo "pass $i done:$keep"
done < "${PMC_GROUPS:-tools/pmc_groups.txt}"
