"""Static issue-cost accounting of one kernel's ISA by source line, weighting each VALU instruction
with its measured issue class (profiles/r01g_valu_issue_probe.txt). Development tool.
Usage: python tools/isa_cost.py <file.s with .loc lines> <kernel symbol> [source-file-substring]"""
import collections
import re
import sys

TWO = {"v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32", "v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32",
       "v_lshrrev_b32_e32", "v_mov_b32_e32", "v_add_f32_e32", "v_mul_f32_e32", "v_not_b32_e32"}
FIVE = {"v_mad_u64_u32", "v_fma_f64", "v_fmac_f64_e32"}


def cost(op, args):
    if op.startswith("v_rcp_f64"):
        return 16.0
    if op in FIVE:
        return 5.0
    if op in TWO and not re.search(r"\bs\[?\d", args):
        return 2.3
    if op.startswith("v_"):
        return 4.2
    return 0.0


def main(path, sym, srcsub=""):
    s = open(path).read()
    i = s.index(sym + ":")
    j = s.index("s_endpgm", i)
    files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
    cur = ("?", 0)
    by_line = collections.Counter()
    n_line = collections.Counter()
    for line in s[i:j].splitlines():
        t = line.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if not t.startswith("v_"):
            continue
        op, _, args = t.partition(" ")
        by_line[cur] += cost(op, args)
        n_line[cur] += 1
    for (f, l), c in sorted(by_line.items(), key=lambda x: (x[0][0], x[0][1])):
        if srcsub in f:
            print(f"{f}:{l}\t{n_line[(f, l)]}\t{c:.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
