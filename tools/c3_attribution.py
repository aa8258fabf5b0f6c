"""Where the C3 kernel's VALU and SALU instructions go, per wave-iteration of the bin stepper.

Static part: the C3 instance's ISA (hipcc -S -gline-tables-only of the max-ILP build; tools/isa_blocks.py parses it),
every VALU / SALU instruction with the source line it comes from. Dynamic part: how often each basic block runs per
wave-iteration. A block is classed by the kernel lines it holds (the loop's regions below; a block with none takes
the class of the block before it), and each class has its measured frequency: 1 for the event's common path, the
rare blocks' fractions of wave-iterations from a -DECDNA_PATH_STATS run (tools/path_stats.py c3), 1/32 for the
N- fast-forward entry test, 2^-10 for the rotation tick, the replicate boundary's fraction. Instructions of the common
path are then bucketed by the function or source region they come from. The sum is compared with the PMC count
(SQ_INSTS_VALU / SALU, tools/ab_pmc_summary.py) converted to wave-iterations; the gap is what the static model misses
(loop trip counts in the binomial words, the Lemire loop). Development tool.

Usage: python tools/c3_attribution.py <kernels.s> <symbol> <path_stats.json line> <pmc summary line>"""
import collections
import json
import re
import sys

# kernel-file regions of ssa_stepper_bins' event loop (ssa_kernels.hip), in source order; lines of the helpers defined
# before the loop (540-860: rotation claims, bin counters, bin search, bags) say nothing about the call site and are
# left out of the classification
REGIONS = [
    (863, 877, "loop top"), (878, 912, "rotation tick"), (913, 918, "loop top"), (919, 1089, "replicate boundary"),
    (1090, 1090, "loop top"), (1091, 1098, "fast-forward entry test"), (1099, 1362, "N- fast-forward"),
    (1363, 1384, "propensities and stop tests"), (1385, 1407, "replicate stop"), (1408, 1422, "channel"),
    (1423, 1436, "word stream setup"), (1437, 1472, "pick"), (1473, 1479, "Lemire rejection"),
    (1480, 1483, "large-k pick"), (1484, 1515, "segregation"), (1516, 1519, "binomial words"),
    (1520, 1540, "segregation"), (1541, 1552, "commit"), (1553, 1560, "capacity checks"),
    (1561, 1576, "bin counter updates"), (1577, 1577, "commit"), (1578, 1601, "large-k row update"),
    (1602, 1620, "commit (spares, n-, time, hash)"),
]
HELPERS = [(542, 662, "rotation claims"), (684, 729, "bin counter updates"), (734, 777, "bin search"),
           (778, 862, "bins, bags")]
# ssa_device.hpp functions (line ranges)
DEVICE = [
    (27, 117, "Philox block"), (118, 143, "soft log"), (144, 160, "channel"), (161, 173, "time step (division)"),
    (174, 192, "bit helpers"), (193, 201, "pick"), (202, 212, "stage log table"), (213, 240, "word stream"),
    (241, 351, "binomial words"), (352, 400, "commit (spares, n-, time, hash)"),
]
RARE = {  # class -> path-stats key for its frequency per wave-iteration
    "Lemire rejection": "lemire_reject", "large-k pick": "large_pick", "binomial words": "binomial_words",
    "large-k row update": "large_row_update", "capacity checks": "capacity_gate", "replicate boundary": "boundary",
    "replicate stop": "boundary",
}


def region(table, line):
    for a, b, name in table:
        if a <= line <= b:
            return name
    return None


def parse(path, sym):
    """Basic blocks (labels .LBB* and the compiler's %bb.* comments) with the loop each sits in, and every VALU /
    SALU instruction with its source location."""
    s = open(path).read()
    i = s.index(sym + ":")
    j = s.index(".Lfunc_end", i)
    files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
    blocks, cur, loc = [], {"name": "entry", "loop": None, "ins": []}, ("?", 0)
    blocks.append(cur)
    for raw in s[i:j].splitlines():
        m = re.match(r"\s*(?:;\s*)?(%bb\.\d+|\.LBB\w+):(.*)", raw)
        if m:
            lm = re.search(r"Header=(\w+) Depth=(\d+)", m.group(2))
            cur = {"name": m.group(1), "loop": (lm.group(1), int(lm.group(2))) if lm else None, "ins": []}
            blocks.append(cur)
            continue
        t = raw.split(";")[0].strip()
        if not t:
            continue
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            loc = (files.get(m.group(1), m.group(1)), int(m.group(2)))
            continue
        if t.startswith("."):
            continue
        op = t.split()[0]
        kind = None
        if op.startswith("v_"):
            kind = "valu"
        elif op.startswith("s_") and not op.startswith(("s_waitcnt", "s_nop", "s_load", "s_buffer_load")):
            kind = "salu"
        if kind:
            cur["ins"].append((kind, loc[0], loc[1]))
    return blocks


def main(path, sym, stats_line, pmc_line):
    stats = json.loads(stats_line)
    pmc = json.loads(pmc_line[pmc_line.index("{"):])
    wave_iters = stats["wave_iters"]
    we_per_iter = stats["events"] / 64.0 / wave_iters  # PMC counts are per wave-event (events / 64)
    freq_of = {k: stats[v] / wave_iters for k, v in RARE.items()}
    freq_of.update({"fast-forward entry test": 1 / 32, "N- fast-forward": 0.0, "rotation tick": 2.0 ** -10})
    blocks = parse(path, sym)
    # the event loop: the loop the propensity block sits in
    main_hdr = next(b["loop"][0] for b in blocks
                    if b["loop"] and any(f.endswith("ssa_kernels.hip") and 1368 <= ln <= 1384 for (_, f, ln) in b["ins"]))

    def own_class(ins):
        """class from a set of instructions' lines: the binomial's device code, else the majority event-loop region"""
        if any(f.endswith("ssa_device.hpp") and 241 <= ln <= 351 for (_, f, ln) in ins):
            return "binomial words"
        kl = [region(REGIONS, ln) for (_, f, ln) in ins if f.endswith("ssa_kernels.hip") and region(REGIONS, ln)]
        return collections.Counter(kl).most_common(1)[0][0] if kl else None

    inner = collections.defaultdict(list)  # loops nested in the event loop: classed as a whole
    for b in blocks:
        if b["loop"] and b["loop"][0] != main_hdr:
            inner[b["loop"][0]].extend(b["ins"])
    # (a loop with only helper lines: the rotation claims' retry loops and the bag copies, run at a replicate boundary)
    inner_cls = {h: own_class(ins) or ("replicate boundary" if any(region(HELPERS, ln) for (_, f, ln) in ins
                                                                   if f.endswith("ssa_kernels.hip")) else "?")
                 for h, ins in inner.items()}
    in_loop = {h for h in inner} | {main_hdr}
    cls_prev = "loop top"
    by_cls = collections.defaultdict(lambda: collections.Counter())
    by_bucket = collections.defaultdict(lambda: collections.Counter())
    for b in blocks:
        if not b["loop"] or b["loop"][0] not in in_loop:
            continue  # outside the event loop: once per wave
        if b["loop"][0] != main_hdr:
            cls = inner_cls[b["loop"][0]]
        else:
            cls = own_class(b["ins"]) or cls_prev
            cls_prev = cls
        fr = freq_of.get(cls, 1.0)
        for kind, f, ln in b["ins"]:
            by_cls[cls][kind] += fr
            if fr == 1.0:  # the common path, by function / region
                if f.endswith("ssa_device.hpp"):
                    bucket = region(DEVICE, ln) or "ssa_device.hpp (other)"
                elif f.endswith("ssa_kernels.hip") and ln:
                    bucket = region(REGIONS, ln) or region(HELPERS, ln) or "?"
                elif ln == 0:
                    bucket = "no source line (moves, EXEC masks, loop control)"
                else:
                    bucket = f"{f} (library)"
                by_bucket[bucket][kind] += 1
    tot = collections.Counter()
    for c in by_cls.values():
        tot.update(c)
    meas = {k: pmc["SQ_INSTS_" + k.upper()] * we_per_iter for k in ("valu", "salu")}
    print(f"C3 bin stepper, per wave-iteration ({stats['lanes_per_wave_iter']} active lanes, "
          f"{we_per_iter:.4f} wave-events per wave-iteration)")
    print(f"measured (PMC): VALU {meas['valu']:.1f}  SALU {meas['salu']:.1f}   "
          f"static model: VALU {tot['valu']:.1f}  SALU {tot['salu']:.1f}   "
          f"unmodelled: VALU {meas['valu'] - tot['valu']:+.1f}  SALU {meas['salu'] - tot['salu']:+.1f}")
    print("\nby block class (frequency per wave-iteration x static count):")
    for cls, c in sorted(by_cls.items(), key=lambda kv: -kv[1]["valu"]):
        print(f"  {cls:40s} freq {freq_of.get(cls, 1.0):8.5f}  VALU {c['valu']:7.1f}  SALU {c['salu']:7.1f}")
    print("\ncommon path (frequency 1) by function / source region:")
    for name, c in sorted(by_bucket.items(), key=lambda kv: -kv[1]["valu"]):
        print(f"  {name:50s} VALU {c['valu']:5.0f}  SALU {c['salu']:5.0f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
