#!/bin/bash
# Same-box A/B on every config shape: GPU parity of the working tree, then C4 shards (ranks 7, 4, 0 of 8,
# K = 32), the C5 shard (K = 64) and C3 (K = 32) for the tree vs ecdna-evo_amd/lib_ab/<ref>/ (build it
# first: tools/ab_build.sh <git-ref> <ref>). Usage: bash tools/ab_configs.sh <ref>
set -euo pipefail
REF=${1:?ref}
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/abc_$REF; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random_parity.py tests/test_gpu_rotation.py \
  -q -x --timeout 300 > $O/parity.log 2>&1 || { echo PARITY FAILED; tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
B=$PWD/ecdna-evo_amd/lib_ab/$REF/libecdna_ssa.so
for lib in "" "$B"; do
  tag=$([ -z "$lib" ] && echo tree || echo $REF)
  for r in ${C4_RANKS:-7 4 0}; do
    ECDNA_SSA_LIB=$lib PROBE_RANK=$r PROBE_FLAGS=0x20 PROBE_KMAX=32 timeout -k 10 120 python3 tools/probe_configs.py c4 > $O/c4_${tag}_$r.log 2>&1
    python3 -c "import json,sys; d=[json.loads(l) for l in open('$O/c4_${tag}_$r.log') if l.startswith('{')][0]; print('$tag c4 rank $r', round(d['stepper_ms'],1), '%.3e' % d['events_per_s_kernel'])"
  done
  if [ -z "${SKIP_C5:-}" ]; then
    ECDNA_SSA_LIB=$lib PROBE_FLAGS=0x20 PROBE_KMAX=64 timeout -k 10 120 python3 tools/probe_configs.py c5 > $O/c5_$tag.log 2>&1
    python3 -c "import json; d=[json.loads(l) for l in open('$O/c5_$tag.log') if l.startswith('{')][0]; print('$tag c5', round(d['stepper_ms'],1), '%.3e' % d['events_per_s_kernel'])"
  fi
done
SWEEP_FLAGS=0x20 SWEEP_KMAX=32 timeout -k 10 600 python3 tools/sweep.py "ECDNA_SSA_LIB=,$B,,$B" > $O/c3.log 2>&1
cat $O/c3.log
