"""Basic blocks of one kernel's ISA (hipcc -S -gline-tables-only): per block its VALU / SALU / LDS / VMEM instruction
counts, the source lines its instructions come from, and its successors, so that the event loop's common path and
its rare blocks can be told apart and counted (profiles/r05_c3_attribution.txt). Development tool.
Usage: python tools/isa_blocks.py <file.s> <kernel symbol> [--json]"""
import collections
import json
import re
import sys


def parse(path, sym):
    s = open(path).read()
    i = s.index(sym + ":")
    j = s.index("s_endpgm", i)
    j = s.index("\n", s.index(".Lfunc_end", j))
    files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
    blocks, order = {}, []
    cur_name, cur = "entry", None
    loc = ("?", 0)

    def new(name):
        b = {"name": name, "valu": 0, "salu": 0, "lds": 0, "vmem": 0, "smem": 0, "other": 0, "lines": collections.Counter(),
             "succ": [], "ops": collections.Counter(), "term": None}
        blocks[name] = b
        order.append(name)
        return b

    cur = new(cur_name)
    for line in s[i:j].splitlines():
        t = line.split(";")[0].strip()
        if not t:
            continue
        m = re.match(r"(\.LBB\w+):", t)
        if m:
            if cur["term"] not in ("s_branch", "s_endpgm") and m.group(1) not in cur["succ"]:
                cur["succ"].append(m.group(1))  # fallthrough
            cur = new(m.group(1))
            continue
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if t.startswith("."):
            continue
        op = t.split()[0]
        if op.startswith("v_"):
            cur["valu"] += 1
            cur["lines"][loc] += 1
            cur["ops"][op] += 1
        elif op.startswith("ds_"):
            cur["lds"] += 1
            cur["lines"][loc] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            cur["vmem"] += 1
            cur["lines"][loc] += 1
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            cur["smem"] += 1
        elif op.startswith("s_"):
            if op in ("s_waitcnt", "s_nop") or op.startswith("s_waitcnt"):
                cur["other"] += 1
            else:
                cur["salu"] += 1
                cur["lines"][loc] += 1
            if op == "s_branch" or op.startswith("s_cbranch"):
                tgt = t.split()[1]
                cur["succ"].append(tgt)
                cur["term"] = "s_branch" if op == "s_branch" else op
                # a branch ends the basic block: what follows is the fallthrough block
                nxt = f"{cur['name'].split('+')[0]}+{len([o for o in order if o.startswith(cur['name'].split('+')[0])])}"
                if op != "s_branch":
                    cur["succ"].append(nxt)
                cur = new(nxt)
            elif op == "s_endpgm":
                cur["term"] = "s_endpgm"
        else:
            cur["other"] += 1
    return blocks, order


def main(path, sym, *opts):
    blocks, order = parse(path, sym)
    if "--json" in opts:
        out = []
        for n in order:
            b = blocks[n]
            out.append({k: v for k, v in b.items() if k not in ("lines", "ops")} |
                       {"lines": sorted(f"{f}:{l}" for (f, l) in b["lines"]), "ops": dict(b["ops"])})
        print(json.dumps(out))
        return
    tot = collections.Counter()
    for n in order:
        b = blocks[n]
        lines = sorted({l for (f, l) in b["lines"] if f.endswith(("ssa_kernels.hip", "ssa_device.hpp"))})
        rng = f"{lines[0]}-{lines[-1]}" if lines else "-"
        files = sorted({f for (f, l) in b["lines"]})
        print(f"{n:28s} v{b['valu']:4d} s{b['salu']:4d} lds{b['lds']:3d} vm{b['vmem']:3d}  lines {rng:11s} "
              f"{','.join(x.replace('.hip', '').replace('.hpp', '') for x in files)[:40]:40s} -> {' '.join(b['succ'])}")
        for k in ("valu", "salu", "lds", "vmem"):
            tot[k] += b[k]
    print("total", dict(tot))


if __name__ == "__main__":
    main(*sys.argv[1:])
