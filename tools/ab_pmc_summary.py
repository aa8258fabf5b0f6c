"""SQ instruction counts per wave-event of the bin stepper from one rocprofv3 --pmc pass over a 1-step bench
(tools/gpu_session.sh, step pmc). Development tool. Usage: python tools/ab_pmc_summary.py <pmc dir> <bench stdout> <name> [all]
(all: every counter of the pass per wave-event, e.g. the SQ_WAIT_* / SQ_ACTIVE_* stall split of tools/gpu_session.sh's
stall step; PMC_KERNEL: the kernel-name prefix summed, default ssa_stepper_bins)"""
import csv
import os
import glob
import json
import sys


def main(pmc_dir, bench_log, name, every=""):
    paths = glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True)
    if not paths:
        print(name, "no counter file")
        return
    tot = {}
    for r in csv.DictReader(open(paths[0])):
        if r["Kernel_Name"].startswith(os.environ.get("PMC_KERNEL", "ssa_stepper_bins")):
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            tot["VGPR"] = int(r["VGPR_Count"])
    ev = None
    for line in open(bench_log):
        if line.startswith("{"):
            ev = json.loads(line)["config"]["events_per_step"]
    if not ev:
        print(name, "no bench line", tot)
        return
    we = ev / 64.0
    out = {k: round(v / we, 2) for k, v in tot.items() if k.startswith("SQ_INSTS") or (every and k.startswith("SQ_"))}
    out["busy_cycles"] = tot.get("SQ_BUSY_CYCLES")
    out["VGPR"] = tot.get("VGPR")
    print(name, "per wave-event:", json.dumps(out))


if __name__ == "__main__":
    main(*sys.argv[1:5])
