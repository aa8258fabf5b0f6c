#!/bin/bash
# Same-box A/B of the bin-store stepper: parity of the working tree, then C3 (K=32) and C2/C4/C5-shard
# timings of the tree vs ecdna-evo_amd/lib_ab/<ref>/ (build it first: tools/ab_build.sh <ref>).
# Usage: bash tools/ab_bins.sh <ref> [probe configs, default "c2 c4"]
set -euo pipefail
REF=${1:?ref}
CFGS=${2:-c2 c4}
cd "$GRAFT_REPO_ROOT"
B=$PWD/ecdna-evo_amd/lib_ab/$REF/libecdna_ssa.so
O=gpurun_out/abb_$REF; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py -q -x --timeout 300 > $O/parity.log 2>&1 || { echo PARITY FAILED; tail -40 $O/parity.log; exit 1; }
echo parity ok; tail -1 $O/parity.log
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 600 python3 tools/sweep.py "ECDNA_SSA_LIB=,$B,,$B" > $O/c3.log 2>&1
cat $O/c3.log
for lib in "" "$B"; do
  tag=$([ -z "$lib" ] && echo tree || echo ref)
  ECDNA_SSA_LIB=$lib PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 300 python3 tools/probe_configs.py $CFGS > $O/probe_$tag.log 2>&1
  echo $tag; python3 -c "
import json,sys
for l in open('$O/probe_$tag.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['config'], round(d['stepper_ms'],2), '%.4e' % d['events_per_s_kernel'])"
done
