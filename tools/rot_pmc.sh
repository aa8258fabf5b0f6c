#!/bin/bash
# Rotation's steady-state cost: SQ wave-state and instruction counters of the C3 stepper at 2^22
# replicates (four grids of work per lane), rotation off (ECDNA_SSA_ROTATE=0) and on (=1), one
# rocprofv3 --pmc pass per counter group. Usage: bash tools/rot_pmc.sh
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/rot_pmc; mkdir -p $O
for rot in 0 1; do
  i=0
  for group in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES" \
               "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"; do
    i=$((i+1))
    ECDNA_SSA_ROTATE=$rot timeout -k 10 300 rocprofv3 --pmc $group -T --output-format csv -d $O/r${rot}_p$i -o pmc -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --reps-per-gpu 4194304 > $O/r${rot}_p$i.log 2>&1
    echo "rot=$rot pass $i done"
  done
done
python3 - <<'PY'
import csv, glob, collections
for rot in (0, 1):
    tot = collections.Counter(); dur = None
    for f in glob.glob(f"gpurun_out/rot_pmc/r{rot}_p*/**/pmc_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("ssa_stepper_bins"):
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
    print("rot", rot, {k: "%.4g" % v for k, v in sorted(tot.items())})
PY
