"""Static VALU accounting of one kernel's ISA by source line (build with -gline-tables-only -S), weighting
each instruction with its measured issue class (profiles/r01g_valu_issue_probe.txt). Development tool.
Usage: python tools/isa_lines.py <file.s> <kernel symbol> [first_line last_line]"""
import collections
import re
import sys

TWO = {"v_and_b32_e32", "v_or_b32_e32", "v_xor_b32_e32", "v_add_u32_e32", "v_sub_u32_e32", "v_subrev_u32_e32",
       "v_lshrrev_b32_e32", "v_mov_b32_e32", "v_add_f32_e32", "v_mul_f32_e32", "v_not_b32_e32"}


def cost(op, t):
    if "rcp_f64" in op:
        return 16.0
    if op in ("v_mad_u64_u32", "v_fma_f64", "v_fmac_f64_e32"):
        return 5.0
    if op in TWO and not re.search(r"\bs\[?\d", t):
        return 2.3
    return 4.2


def main(path, sym, lo=0, hi=10 ** 9):
    lo, hi = int(lo), int(hi)
    s = open(path).read()
    i = s.index(sym + ":")
    j = s.index("s_endpgm", i)
    files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
    cur = ("?", 0)
    by, n, ops, sal = collections.Counter(), collections.Counter(), collections.defaultdict(list), collections.Counter()
    for line in s[i:j].splitlines():
        t = line.strip()
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            cur = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if t.startswith("v_"):
            op = t.split()[0]
            by[cur] += cost(op, t)
            n[cur] += 1
            ops[cur].append(op[2:].replace("_e32", "").replace("_e64", "*"))
        elif t.startswith("s_") and not t.startswith(("s_waitcnt", "s_nop", "s_branch", "s_cbranch")):
            sal[cur] += 1
    for (f, l), c in sorted(by.items(), key=lambda x: (x[0][0], x[0][1])):
        if f.endswith("ssa_kernels.hip") and not (lo <= l <= hi):
            continue
        print(f"{f}:{l}\t{n[(f, l)]}\t{c:.0f}\tsalu {sal[(f, l)]}\t{' '.join(ops[(f, l)])[:120]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
