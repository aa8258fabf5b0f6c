"""Sum rocprofv3 --pmc counters per kernel over the pass directories of tools/pmc_probe.sh.
Usage: python tools/pmc_kernels.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv
import glob
import json
import os
import sys


def main(d, sub=""):
    tot = {}
    for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if sub and sub not in k:
                continue
            key = k.split("(")[0][:90]
            tot.setdefault(key, {})
            tot[key][r["Counter_Name"]] = tot[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else ""), indent=1))
