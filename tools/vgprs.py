"""Resource usage per kernel instance from hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin): name, VGPRs,
SGPRs, scratch. Development tool. Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/vgprs.py [filter]"""
import re
import subprocess
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "TotalSGPRs", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0].split("\\")[0]] = int(m.group(1))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
except Exception:
    dem = names
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for r, d in zip(rows, dem):
    if flt in d:
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('TotalSGPRs', '?'):>4} s {r.get('ScratchSize', 0):>4} scr  occ {r.get('Occupancy', '?')}  {d.replace('void ecdna::', '').replace('(ecdna::StepperArgs)', '')}")
