"""INTEGRATION.md's Rust binding against the C ABI it binds: the `extern "C"` block of §2.1 must
declare exactly the entry points of include/ecdna_ssa.h, each with the header's parameter count, and its #[repr(C)]
structs must list the header structs' fields in the same order with the same widths — the binding a maintainer of
fraterenz/ecdna-evo would paste into src/gpu.rs cannot drift from the library."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ecdna_ssa.h")
DOC = os.path.join(REPO, "INTEGRATION.md")

RUST_STRUCTS = {  # Rust mirror -> C typedef
    "EcdnaRates": "ecdna_rates_t",
    "EcdnaSsaParams": "ecdna_ssa_params_t",
    "EcdnaRepSummary": "ecdna_rep_summary_t",
    "EcdnaTotals": "ecdna_totals_t",
    "EcdnaRepStats": "ecdna_rep_stats_t",
    "EcdnaSnapshot": "ecdna_snapshot_t",
    "EcdnaSsaInstance": "ecdna_ssa_instance_t",
}
C_WIDTH = {"uint64_t": 8, "int64_t": 8, "double": 8, "uint32_t": 4, "int32_t": 4, "float": 4, "int": 4,
           "uint16_t": 2, "uint8_t": 1}
RUST_WIDTH = {"u64": 8, "i64": 8, "f64": 8, "u32": 4, "i32": 4, "f32": 4, "c_int": 4, "u16": 2, "u8": 1}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", re.sub(r"//[^\n]*", "", s, flags=re.S), flags=re.S)


def _header():
    with open(HEADER) as f:
        return _strip_c_comments(f.read())


def _rust_block():
    with open(DOC) as f:
        doc = f.read()
    sec = doc[doc.index("### 2.1"):doc.index("### 2.2")]
    m = re.search(r"```rust\n(.*?)```", sec, re.S)
    assert m, "no rust block in INTEGRATION.md §2.1"
    return re.sub(r"//[^\n]*", "", m.group(1))


def _params(arglist):
    a = arglist.strip()
    if a in ("", "void"):
        return 0
    depth, n = 0, 1
    for ch in a:
        depth += ch in "([<"
        depth -= ch in ")]>"
        n += ch == "," and depth == 0
    return n


def header_functions():
    h = _header()
    out = {}
    for m in re.finditer(r"\b(ecdna_ssa_\w+)\s*\(([^;{]*?)\)\s*;", h, re.S):
        out[m.group(1)] = _params(m.group(2))
    return out


def rust_functions():
    blk = _rust_block()
    ext = blk[blk.index('extern "C"'):]
    return {m.group(1): _params(m.group(2)) for m in re.finditer(r"pub fn (\w+)\s*\(([^;]*?)\)\s*(?:->[^;]*)?;", ext, re.S)}


def header_struct(name):
    h = _header()
    end = re.search(r"\}\s*" + name + r"\s*;", h)
    assert end, name
    start = h.rindex("typedef struct", 0, end.start())
    body = h[h.index("{", start) + 1:end.start()]
    fields = []
    for decl in body.split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        ptr = "*" in decl
        decl = decl.replace("const ", "").replace("*", " ")
        typ, rest = decl.split(" ", 1)
        for nm in rest.split(","):
            nm = nm.strip()
            arr = re.match(r"(\w+)\[(\w+)\]", nm)
            n = 1
            if arr:
                nm, n = arr.group(1), int(arr.group(2))
            fields.append((nm, 8 if ptr else C_WIDTH[typ] * n))
    return fields


def rust_struct(name):
    blk = _rust_block()
    m = re.search(r"pub struct " + name + r"\s*\{(.*?)\}", blk, re.S)
    assert m, name
    fields = []
    for f in m.group(1).split(","):
        f = " ".join(f.split())
        if not f:
            continue
        mm = re.match(r"pub (\w+): (.+)", f)
        assert mm, f
        nm, typ = mm.group(1), mm.group(2).strip()
        if typ.startswith("*"):
            w = 8
        else:
            arr = re.match(r"\[(\w+); (\d+)\]", typ)
            w = RUST_WIDTH[arr.group(1)] * int(arr.group(2)) if arr else RUST_WIDTH[typ]
        fields.append((nm, w))
    return fields


def test_every_header_entry_point_is_bound_with_its_arity():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 24
    assert set(h) == set(r), {"missing in INTEGRATION.md": sorted(set(h) - set(r)),
                              "not in the header": sorted(set(r) - set(h))}
    for name in h:
        assert h[name] == r[name], (name, h[name], r[name])


def test_every_rust_struct_mirrors_its_header_struct():
    for rname, cname in RUST_STRUCTS.items():
        assert rust_struct(rname) == header_struct(cname), rname


def test_the_binding_names_the_current_abi_version():
    m = re.search(r"#define ECDNA_SSA_ABI_VERSION (\d+)", _header())
    with open(DOC) as f:
        doc = f.read()
    assert f"must be {m.group(1)}" in doc and f"ABI version {m.group(1)}" in doc


def test_exported_symbols_are_the_header_entry_points():
    """the product library's Python binding lists the same entry points (engine.EXPORTS, checked against the .so's
    symbol table by tests/test_abi.py)"""
    import sys

    sys.path.insert(0, os.path.join(REPO, "ecdna-evo_amd"))
    from ecdna_evo_amd import engine

    assert set(engine.EXPORTS) == set(header_functions())


CLI = os.path.join(REPO, "ecdna-evo_amd", "bin", "ecdna-dynamics")


def test_cli_extra_flag_table_matches_help():
    """the CLI's extra flags (those past the reference's clap interface) are exactly
    the table's, checked against `ecdna-dynamics --help` both ways, and the `--draws reference` row says what the code
    does: subsamples continue the replicate's ChaCha8 stream (host/dynamics_main.cpp; src/main.rs:110-123)."""
    import subprocess

    import pytest

    if not os.path.exists(CLI):
        pytest.skip("ecdna-dynamics not built")
    help_text = subprocess.run([CLI, "--help"], capture_output=True, text=True, check=True).stdout
    # the extras are listed after the reference's last flag (-v, --verbosity) and before -h, --help
    tail = help_text[help_text.index("--verbosity"):help_text.index("--help")]
    help_flags = set(re.findall(r"^\s+(--[a-z0-9-]+)", tail, re.M))
    with open(DOC) as f:
        doc = f.read()
    table = doc[doc.index("| flag | meaning |"):]
    table = table[:table.index("\n\n")]
    doc_flags = set(re.findall(r"^\| `(--[a-z0-9-]+)", table, re.M))
    assert doc_flags == help_flags, (sorted(doc_flags - help_flags), sorted(help_flags - doc_flags))
    ref_row = next(ln for ln in table.splitlines() if ln.startswith("| `--draws"))
    assert "ChaCha8" in ref_row and "Philox side stream" not in ref_row
