"""The C ABI boundary without a GPU: the product library loads, exports every function that
include/ecdna_ssa.h declares, the ctypes mirror matches the header's struct layout, parameter
validation works, and — with no device — compute entry points fail loudly (no CPU fallback)."""
import ctypes as C
import json
import os
import re
import subprocess

import numpy as np
import pytest

from ecdna_evo_amd import abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "ecdna_ssa.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ecdna_ssa_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def product_lib():
    from ecdna_evo_amd import engine

    if not os.path.exists(engine.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    return engine.lib()


def test_library_exports_every_declared_symbol(product_lib):
    from ecdna_evo_amd import engine

    names = declared_functions()
    assert len(names) >= 14
    for n in names:
        assert hasattr(product_lib, n), f"libecdna_ssa.so does not export {n}"
    assert set(names) == set(engine.EXPORTS)


def test_library_is_gfx950_code_object():
    from ecdna_evo_amd import engine

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", engine.LIB_PATH], capture_output=True,
                         text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"amdgcn-amd-amdhsa--gfx942" not in blob  # MI355X only


def test_abi_version(product_lib):
    assert product_lib.ecdna_ssa_abi_version() == abi.ABI_VERSION


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    fields = {"ecdna_ssa_params_t": [f for f, _ in abi.Params._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){", 'printf("{");']
    for st, fs in fields.items():
        lines.append(f'printf("\\"{st}\\": {{\\"size\\": %zu", sizeof({st}));')
        for f in fs:
            lines.append(f'printf(", \\"{f}\\": %zu", offsetof({st}, {f}));')
        lines.append('printf("}, ");')
    lines.append('printf("\\"summary\\": %zu, \\"totals\\": %zu, \\"rates\\": %zu", sizeof(ecdna_rep_summary_t), '
                 'sizeof(ecdna_totals_t), sizeof(ecdna_rates_t));')
    for f in abi.SUMMARY_DTYPE.names:
        lines.append(f'printf(", \\"s_{f}\\": %zu", offsetof(ecdna_rep_summary_t, {f}));')
    for f in abi.TOTALS_DTYPE.names:
        lines.append(f'printf(", \\"t_{f}\\": %zu", offsetof(ecdna_totals_t, {f}));')
    lines.append('printf(", \\"instance\\": %zu", sizeof(ecdna_ssa_instance_t));')
    for f, _ in abi.Instance._fields_:
        lines.append(f'printf(", \\"i_{f}\\": %zu", offsetof(ecdna_ssa_instance_t, {f}));')
    lines += ['printf("}\\n");', "return 0;}"]
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = json.loads(subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout)
    p = got["ecdna_ssa_params_t"]
    assert p["size"] == C.sizeof(abi.Params)
    for f, _ in abi.Params._fields_:
        assert p[f] == getattr(abi.Params, f).offset, f
    assert got["summary"] == abi.SUMMARY_DTYPE.itemsize
    assert got["totals"] == abi.TOTALS_DTYPE.itemsize
    assert got["rates"] == C.sizeof(abi.Rates)
    for f in abi.SUMMARY_DTYPE.names:
        assert got[f"s_{f}"] == abi.SUMMARY_DTYPE.fields[f][1], f
    for f in abi.TOTALS_DTYPE.names:
        assert got[f"t_{f}"] == abi.TOTALS_DTYPE.fields[f][1], f
    assert got["instance"] == C.sizeof(abi.Instance)
    for f, _ in abi.Instance._fields_:
        assert got[f"i_{f}"] == getattr(abi.Instance, f).offset, f


def _has_gpu(lib):
    return lib.ecdna_ssa_device_count() > 0


def test_invalid_parameters_rejected(product_lib):
    bad = []
    s = abi.RunSpec(n_replicates=4)
    p = s.params()
    p.reps_per_set = 0
    bad.append(p)
    p = s.params()
    p.hist_bins = 1
    bad.append(p)
    p = s.params()
    p.segregation = 9
    bad.append(p)
    p = s.params()
    p.max_iter = 2**33
    bad.append(p)
    s2 = abi.RunSpec(n_replicates=4, cell_cap=2, init={1: 5})
    bad.append(s2.params())
    s3 = abi.RunSpec(rates=((1, 1, 0, 0), (1, 2, 0, 0)), reps_per_set=2, n_replicates=8)
    bad.append(s3.params())  # replicate 7 -> set 3 >= 2 sets
    bad_rates = [abi.RunSpec(rates=(r,), n_replicates=4) for r in
                 ((1, float("inf"), 0, 0), (1, 1, float("nan"), 0), (1, 1, 0, -0.5), (-1e-30, 1, 0, 0),
                  (1, 1e-20, 0, 0), (1, 1, 2e18, 0), (1e-45, 1, 0, 0))]
    bad += [r.params() for r in bad_rates]  # rates must be 0 or in [2^-60, 2^60] (ABI v8)
    s4 = abi.RunSpec(n_replicates=4, flags=abi.FLAG_REFERENCE_DRAWS | abi.FLAG_BIN_STORE)
    bad.append(s4.params())  # the reference draws run the row store only
    keep = [s, s2, s3, s4, bad_rates]  # noqa: F841  (host arrays referenced by the params)
    for q in bad:
        h = C.c_void_p()
        rc = product_lib.ecdna_ssa_ctx_create(C.byref(q), C.byref(h))
        assert rc == abi.E_INVALID, product_lib.ecdna_ssa_last_error_message()
        assert product_lib.ecdna_ssa_last_error_message()


def test_no_device_fails_loudly(product_lib):
    """On a machine without a gfx950 GPU the product refuses to run: there is no CPU fallback."""
    if _has_gpu(product_lib):
        pytest.skip("a GPU is present")
    from ecdna_evo_amd import engine

    s = abi.RunSpec(n_replicates=4)
    p = s.params()
    out = abi.summaries_array(4)
    rc = product_lib.ecdna_ssa_run(C.byref(p), out.ctypes.data, None, None, None)
    assert rc == abi.E_NODEVICE
    with pytest.raises(engine.EngineError):
        engine.run(s)
    assert np.all(out["iters"] == 0)


def test_strerror(product_lib):
    for code in (0, -1, -2, -3, -4, -5, -99):
        assert product_lib.ecdna_ssa_strerror(code)


def test_set_cost_hint_in_params():
    import ctypes as C

    spec = abi.RunSpec(rates=((1, 1, 0, 0), (1, 2, 0, 0)), reps_per_set=4, n_replicates=8, set_cost_hint=[1.0, 3.0])
    p = spec.params()
    assert p.set_cost_hint[0] == 1.0 and p.set_cost_hint[1] == 3.0
    assert not abi.RunSpec(n_replicates=4).params().set_cost_hint  # NULL by default
    with pytest.raises(ValueError):
        abi.RunSpec(rates=((1, 1, 0, 0),), set_cost_hint=[1.0, 2.0]).params()
    assert C.sizeof(abi.Params) % 8 == 0


def test_oracle_rejects_invalid_rates(oracle_mod):
    """The oracle keeps the product's contract: every rate 0 or in [2^-60, 2^60] (include/ecdna_ssa.h, ABI v8)."""
    for r in ((1, float("inf"), 0, 0), (1, 1, float("nan"), 0), (1, 1, 0, -0.5), (1, 3.0e38, 0, 0),
              (1, 1, 1e-45, 0), (2.0**60 * 1.01, 1, 0, 0)):
        with pytest.raises(ValueError):
            oracle_mod.run(abi.RunSpec(rates=(r,), n_replicates=2, max_cells=10))
    oracle_mod.run(abi.RunSpec(rates=((0, 2.0**60, 0, 2.0**-60),), n_replicates=2, max_cells=10))


def test_runspec_rejects_values_ctypes_would_mask():
    """ctypes silently truncates integers to the field width: a replicate_stride of 2^32 would reach C as 0
    (= 1, contiguous ids) while RunSpec.replicate_ids() kept the wide stride."""
    for kw in (dict(replicate_stride=1 << 32), dict(big_cap=1 << 32), dict(replicate_stride=-1),
               dict(cell_cap=1 << 32), dict(n_replicates=-1)):
        with pytest.raises(ValueError):
            abi.RunSpec(**kw).params()
    s = abi.RunSpec(n_replicates=3, first_replicate=5, replicate_stride=0)
    assert s.replicate_ids().tolist() == [5, 6, 7] and s.last_replicate() == 7  # stride 0 reads as 1, as in C


def test_oracle_rejects_wrapping_replicate_ids(oracle_mod):
    """first + (n - 1) * stride wrapping u64 is invalid in the oracle as in the engine (ssa_api.cpp validate)."""
    spec = abi.RunSpec(n_replicates=3, first_replicate=(1 << 64) - 2 ** 32, replicate_stride=(1 << 32) - 1,
                       reps_per_set=(1 << 64) - 1, max_cells=10)
    with pytest.raises(ValueError):
        oracle_mod.run(spec)


def test_reduce_entry_points_validate_arguments(product_lib):
    """The RCCL reduction rejects missing communicators / buffers before touching RCCL or a device."""
    import ctypes as C

    L = product_lib
    L.ecdna_ssa_reduce_hist.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p]
    L.ecdna_ssa_ctx_reduce.argtypes = [C.c_void_p, C.c_void_p]
    L.ecdna_ssa_comm_init_all.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    L.ecdna_ssa_comm_init_rank.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
    assert L.ecdna_ssa_reduce_hist(None, None, None, 1, 8, None) == abi.E_INVALID
    assert L.ecdna_ssa_ctx_reduce(None, None) == abi.E_INVALID
    assert L.ecdna_ssa_comm_init_all(0, None, None) == abi.E_INVALID
    uid = (C.c_uint8 * abi.COMM_ID_BYTES)()
    out = C.c_void_p()
    assert L.ecdna_ssa_comm_init_rank(uid, 2, 5, 0, C.byref(out)) == abi.E_INVALID  # rank >= n_ranks
    assert L.ecdna_ssa_comm_destroy(None) == 0
    L.ecdna_ssa_ctx_instance.argtypes = [C.c_void_p, C.c_void_p]
    assert L.ecdna_ssa_ctx_instance(None, None) == abi.E_INVALID
    assert L.ecdna_ssa_strerror(abi.E_COMM)
