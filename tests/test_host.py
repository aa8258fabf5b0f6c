"""The native host around the hot path (CPU only): CLI option resolution mirroring Cli::build
(src/clap_app.rs:137-229), output naming (src/lib.rs:27-45, src/process.rs:267-291), the JSON
histogram format (dynamics.md:8) and end-of-run subsampling (src/main.rs:110-123)."""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "ecdna-evo_amd", "bin", "ecdna-dynamics")
HOSTLIB = os.path.join(REPO, "ecdna-evo_amd", "lib", "libecdna_host.so")


@pytest.fixture(scope="module")
def host():
    if not (os.path.exists(CLI) and os.path.exists(HOSTLIB)):
        import __graft_entry__

        __graft_entry__.build()
    L = C.CDLL(HOSTLIB)
    L.ecdna_host_rate_str.argtypes = [C.c_float, C.c_char_p, C.c_size_t]
    L.ecdna_host_timepoint_dir.argtypes = [C.c_float, C.c_char_p, C.c_size_t]
    L.ecdna_host_filename.argtypes = [C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_uint64, C.c_char_p,
                                      C.c_size_t]
    L.ecdna_host_subsample.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                       C.c_uint32, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.ecdna_host_save.argtypes = [C.c_char_p, C.c_char_p, C.c_float, C.c_void_p, C.c_uint64, C.c_uint64, C.c_char_p,
                                  C.c_size_t]
    L.ecdna_host_load.argtypes = [C.c_char_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.ecdna_host_load.restype = C.c_int64
    L.ecdna_host_subsample_reference.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                                 C.c_uint64, C.POINTER(C.c_uint64), C.c_void_p,
                                                 C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    return L


def test_host_library_exports_every_declared_symbol(host):
    import re

    with open(os.path.join(REPO, "include", "ecdna_host.h")) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    names = sorted(set(re.findall(r"\b(ecdna_host_\w+)\s*\(", text)))
    assert len(names) == 7
    for n in names:
        assert hasattr(host, n), f"libecdna_host.so does not export {n}"


def _s(fn, *args):
    buf = C.create_string_buffer(512)
    assert fn(*args, buf, 512) >= 0
    return buf.value.decode()


def dry(*args):
    out = subprocess.run([CLI, "--dry-run", *args, "/tmp/ecdna_out"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout)


def test_cli_defaults(host):
    d = dry()
    # clap defaults (src/clap_app.rs:35-99): seed 26, runs 12, cells 1000, years floor(log2(1000)+4) = 13
    assert (d["process"], d["segregation"], d["seed"], d["runs"], d["cells"], d["years"]) == \
        ("PureBirth", "binomial", 26, 12, 1000, 13)
    assert d["snapshots"] == [1, 101, 201, 301, 401, 501, 601, 701, 801, 901, 1000]
    assert d["initial"] == {"0": 0, "1": 1} and d["first_idx"] == 260 and d["parallel"] is True


@pytest.mark.parametrize("cells,years", [(10, 7), (1000, 13), (10_000, 17), (1_000_000, 23), (3, 5)])
def test_cli_years_from_cells(host, cells, years):
    assert dry("--cells", str(cells))["years"] == years


@pytest.mark.parametrize("flag,value", [("--b0", "1e-20"), ("--b1", "1e30"), ("--d0", "-1"), ("--d1", "inf")])
def test_cli_rate_outside_the_engine_range_is_a_usage_error(host, flag, value):
    """The engine takes rates 0 or in [2^-60, 2^60] (include/ecdna_ssa.h, since ABI v8), a divergence from the
    reference's any-f32 clap values: reported before any GPU work, exit code 2."""
    out = subprocess.run([CLI, "--dry-run", flag, value, "/tmp/ecdna_out"], capture_output=True, text=True)
    assert out.returncode == 2 and "2^-60, 2^60" in out.stderr, out.stderr
    assert f"invalid value '{value}' for '{flag} <RATE>'" in out.stderr, out.stderr  # the argument as given
    for ok in ("0", "1e-18", "1e18"):
        assert subprocess.run([CLI, "--dry-run", flag, ok, "/tmp/ecdna_out"], capture_output=True).returncode == 0


def test_cli_process_type_from_death_rates(host):
    # is_birth_death = d0 > 0 | d1 > 0 (src/clap_app.rs:163-174)
    assert dry("--d0", "0", "--d1", "0")["process"] == "PureBirth"
    assert dry("--d1", "0.3")["process"] == "BirthDeath"
    assert dry("--d0", "0.1")["process"] == "BirthDeath"


def test_cli_years_mode_and_debug(host):
    d = dry("--years", "20", "--runs", "3", "-s")
    assert d["cells"] == 1_000_000_000 and d["years"] == 20 and d["runs"] == 3 and d["parallel"] is False
    d = dry("-d")
    assert (d["cells"], d["years"], d["runs"], d["verbosity"], d["parallel"]) == (300, 2, 1, 255, False)


def test_cli_lists_and_segregation(host, tmp_path):
    d = dry("--snapshots=50,5,500", "--subsamples=10,100", "--segregation", "binomial-no-uneven")
    assert d["snapshots"] == [5, 50, 500] and d["subsamples"] == [10, 100]
    assert d["segregation"] == "binomial-no-uneven"
    init = tmp_path / "init.json"
    init.write_text('{"0": 2, "1": 2, "10": 1, "20":1}')  # dynamics.md:8
    assert dry("--initial", str(init))["initial"] == {"0": 2, "1": 2, "10": 1, "20": 1}


@pytest.mark.parametrize("args", [["--cells", "5", "--years", "3"], ["-d", "--runs", "2"], ["--initial", "x.csv"],
                                  ["--snapshots", "5"], ["--segregation", "nope"], ["--b0"], ["--bogus"]])
def test_cli_rejects_like_clap(host, args):
    out = subprocess.run([CLI, *args, "/tmp/x"], capture_output=True, text=True)
    assert out.returncode == 2 and "error" in out.stderr


def test_cli_without_device_fails_loudly(host, tmp_path):
    from ecdna_evo_amd import engine

    if engine.device_count() > 0:
        pytest.skip("GPU present")
    out = subprocess.run([CLI, str(tmp_path)], capture_output=True, text=True)
    assert out.returncode == 1 and "gfx950" in out.stderr


@pytest.mark.parametrize("x", [1.0, 1.5, 0.3, 0.1, 2.5e-5, 100.0, 0.9, 1.2, 3.3333333, 1e7])
def test_rate_str_is_rust_f32_display(host, x):
    want = np.format_float_positional(np.float32(x), trim="-").replace(".", "dot")
    assert _s(host.ecdna_host_rate_str, x) == want


@pytest.mark.parametrize("t,want", [(13.0, "13dot0years"), (0.25, "0dot2years"), (9.96, "10dot0years"),
                                    (0.05, "0dot1years"), (5.75, "5dot8years"), (0.0, "0dot0years")])
def test_timepoint_dir(host, t, want):
    assert _s(host.ecdna_host_timepoint_dir, t) == want


def test_filenames(host):
    assert _s(host.ecdna_host_filename, 0, 1.0, 1.5, 0, 0, 420) == "1b0_1dot5b1_0d0_0d1_420idx"
    assert _s(host.ecdna_host_filename, 1, 1.0, 1.5, 0.3, 0.3, 7) == "1b0_1dot5b1_0dot3d0_0dot3d1_7idx"


def test_save_and_load_roundtrip(host, tmp_path):
    cells = np.array([3, 1, 3, 20, 1, 1], np.uint16)
    path = _s(host.ecdna_host_save, str(tmp_path).encode(), b"fname", 7.25, cells.ctypes.data, len(cells), 4)
    assert path == f"{tmp_path}/10cells/ecdna/7dot2years/fname.json"
    assert json.load(open(path)) == {"0": 4, "1": 3, "3": 2, "20": 1}
    out = np.zeros(16, np.uint16)
    nm = C.c_uint64()
    n = host.ecdna_host_load(path.encode(), out.ctypes.data, 16, C.byref(nm))
    assert n == 6 and nm.value == 4 and list(out[:n]) == [1, 1, 1, 3, 3, 20]


@pytest.mark.parametrize("body,want", [
    ('{"0": 5}', (0, 5)),                       # N- only
    ("{}", (0, 0)),                             # empty (the engine then reports the empty-distribution error)
    ('{"0":1,"2":2,"2":1}', (3, 1)),            # a repeated key adds up
    ('{"1": 4294967296}', -1),                  # more than 2^32 - 1 cells: refused before any allocation
    ('{"1": 3000000000, "2": 3000000000}', -1),
    ('{"0": 18446744073709551615, "0": 1}', -1),  # u64 overflow of a repeated key
    ('{"1": 99999999999999999999}', -1),        # out of u64
    ('{"65536": 1}', -1),                       # copy number beyond u16
    ('{"1": 2,}', -1), ('{"1" 2}', -1), ('["1", 2]', -1), ("", -1),
    ('{"1": 17}', -1),                          # more N+ cells than the caller's buffer (cap 16)
    ('{"1": 4000000000, "2": 1}', -1),          # rejected before 4e9 cells are expanded (8 GB)
])
def test_load_rejects_malformed(host, tmp_path, body, want):
    p = tmp_path / "d.json"
    p.write_text(body)
    out = np.zeros(16, np.uint16)
    nm = C.c_uint64()
    n = host.ecdna_host_load(str(p).encode(), out.ctypes.data, 16, C.byref(nm))
    if want == -1:
        assert n == -1
    else:
        assert (n, nm.value) == want


def _philox(ctr, key):
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c = list(ctr)
    k0, k1 = key
    for r in range(10):
        if r:
            k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
             p0 & 0xFFFFFFFF]
    return c


def subsample_py(nplus, nminus, nb, seed, rid, k):
    """Independent restatement of host::subsample (Floyd's algorithm over cell positions)."""
    N = nminus + len(nplus)
    if nb >= N:
        return list(nplus), nminus
    words, blk = [], 0

    def nxt():
        nonlocal blk
        if not words:
            words.extend(_philox([k, 0x80000000 | blk, rid & 0xFFFFFFFF, rid >> 32], [seed & 0xFFFFFFFF, seed >> 32]))
            blk += 1
        return words.pop(0)

    def below(n):
        m = nxt() * n
        if (m & 0xFFFFFFFF) < n:
            thr = (2**32 - n) % n
            while (m & 0xFFFFFFFF) < thr:
                m = nxt() * n
        return m >> 32

    pick = set()
    for j in range(N - nb, N):
        t = below(j + 1)
        pick.add(j if t in pick else t)
    out = [nplus[i - nminus] for i in sorted(pick) if i >= nminus]
    return out, sum(1 for i in pick if i < nminus)


@pytest.mark.parametrize("nb", [0, 1, 7, 50, 199, 200, 500])
def test_subsample_matches_restatement(host, nb):
    rng = np.random.default_rng(nb)
    nplus = rng.integers(1, 60, 150).astype(np.uint16)
    nminus = 50
    out = np.zeros(200, np.uint16)
    onp, onm = C.c_uint64(), C.c_uint64()
    assert host.ecdna_host_subsample(nplus.ctypes.data, len(nplus), nminus, nb, 42, 421, 1, out.ctypes.data,
                                     C.byref(onp), C.byref(onm)) == 0
    want_p, want_m = subsample_py(nplus.tolist(), nminus, nb, 42, 421, 1)
    assert list(out[: onp.value]) == want_p and onm.value == want_m
    assert onp.value + onm.value == min(nb, 200)


def test_subsample_is_uniform_without_replacement(host):
    nplus = np.arange(1, 41, dtype=np.uint16)  # 40 distinct N+ cells, plus 10 N- cells
    counts = np.zeros(41)
    nm_total = 0
    out = np.zeros(40, np.uint16)
    onp, onm = C.c_uint64(), C.c_uint64()
    for rid in range(3000):
        host.ecdna_host_subsample(nplus.ctypes.data, 40, 10, 10, 7, rid, 0, out.ctypes.data, C.byref(onp), C.byref(onm))
        sel = out[: onp.value]
        assert len(set(sel.tolist())) == len(sel)  # without replacement
        counts[sel] += 1
        nm_total += onm.value
    # each of the 50 cells is kept with probability 10/50
    assert abs(counts[1:].mean() / 3000 - 0.2) < 0.01 and abs(nm_total / (3000 * 10) - 0.2) < 0.015


def test_cli_cell_store_options(host):
    d = dry()
    assert (d["cell_store"], d["bin_kmax"]) == ("bins", 64)
    d = dry("--cell-store", "rows")
    assert d["cell_store"] == "rows"
    assert dry("--bin-kmax", "256")["bin_kmax"] == 256
    for bad in (["--cell-store", "tree"], ["--bin-kmax", "100"]):
        out = subprocess.run([CLI, "--dry-run", *bad, "/tmp/ecdna_out"], capture_output=True, text=True)
        assert out.returncode != 0


@pytest.mark.parametrize("runs", [1, 2, 5, 12, 100, 1001])
@pytest.mark.parametrize("gpus", [1, 2, 3, 8])
def test_cli_shards_match_shard_range(host, runs, gpus):
    """--gpus N splits the replicates exactly as ecdna_evo_amd.shard.shard_range (contiguous global ids), with
    never more shards than replicates (every device of the RCCL reduction holds a shard)."""
    from ecdna_evo_amd import shard

    g = min(gpus, runs)
    want = [list(shard.shard_range(r, g, runs)) for r in range(g)]
    assert dry("--runs", str(runs), "--gpus", str(gpus))["shards"] == want
    assert dry("--runs", str(runs), "--gpus", str(gpus), "--sequential")["shards"] == [[0, runs]]


def test_cli_draws_option(host):
    assert dry()["draws"] == "philox"
    d = dry("--draws", "reference")
    assert (d["draws"], d["cell_store"]) == ("reference", "rows")  # the reference's draws need the row store
    assert dry("--draws", "reference", "--cell-store", "rows")["cell_store"] == "rows"
    for bad in (["--draws", "chacha"], ["--draws", "reference", "--cell-store", "bins"],
                ["--draws", "reference", "--bin-kmax", "256"]):  # an explicit bin-store option is refused, not dropped
        out = subprocess.run([CLI, "--dry-run", *bad, "/tmp/ecdna_out"], capture_output=True, text=True)
        assert out.returncode == 2 and "error" in out.stderr, bad


# ---- end-of-run subsampling under the reference's draws (ecdna_host_subsample_reference): the replicate's ChaCha8
# stream continued (src/main.rs:110-123), ecdna-lib 3.0.2 into_subsampled reconstructed as rand 0.8.5
# SliceRandom::choose_multiple (seq::index::sample). Three restatements must agree: the host (product), the oracle
# (oracle_compat_subsample) and the pure-Python one below (which reads the oracle's sequential ChaCha8 words, so it
# also pins the seek to a word position).

def _index_sample_py(next_u32, length, amount):
    """rand 0.8.5 seq::index::sample for length < 2^32 (its algorithm choice in f32 and each algorithm's draws)."""
    f32 = np.float32

    def incl(lo, hi):  # UniformInt<u32>::sample_single_inclusive
        rng_ = (hi - lo + 1) & 0xFFFFFFFF
        zone = ((rng_ << (32 - rng_.bit_length())) & 0xFFFFFFFF) - 1
        while True:
            m = next_u32() * rng_
            if (m & 0xFFFFFFFF) <= zone:
                return lo + (m >> 32)

    def uniform(n):  # Uniform::new(0, n).sample
        zone = 0xFFFFFFFF - ((2**32 - n) % n)
        while True:
            m = next_u32() * n
            if (m & 0xFFFFFFFF) <= zone:
                return m >> 32

    j = 0 if length < 500_000 else 1
    if amount < 163:
        c0, c1 = (f32(1.6), f32(8.0) / f32(45.0)), (f32(10.0), f32(70.0) / f32(9.0))
        a = f32(amount)
        alg = "inplace" if amount > 11 and f32(length) < (c1[j] + c0[j] * a) * a else "floyd"
    else:
        c = (f32(270.0), f32(330.0) / f32(9.0))
        alg = "inplace" if f32(length) < c[j] * f32(amount) else "rejection"
    if alg == "floyd":
        idx = []
        for jj in range(length - amount, length):
            t = incl(0, jj)
            if t not in idx:
                idx.append(t)
            elif amount < 50:  # the fully shuffled variant: j goes in before t
                idx.insert(idx.index(t), jj)
            else:
                idx.append(jj)
        if amount >= 50:
            for i in range(amount - 1, 0, -1):
                k = incl(0, i)
                idx[i], idx[k] = idx[k], idx[i]
    elif alg == "inplace":
        allv = list(range(length))
        for i in range(amount):
            k = incl(i, length - 1)
            allv[i], allv[k] = allv[k], allv[i]
        idx = allv[:amount]
    else:
        idx, seen = [], set()
        for _ in range(amount):
            pos = uniform(length)
            while pos in seen:
                pos = uniform(length)
            seen.add(pos)
            idx.append(pos)
    return alg, idx


# (cells, nminus, amount): Floyd below 12, Floyd with the final shuffle (>= 50), in place, rejection (>= 163 of
# a long row), the whole distribution (amount clamped to the cells), and the N- cells only
SUBSAMPLE_CASES = [(300, 20, 5), (300, 20, 11), (12, 3, 11), (40, 0, 30), (2000, 100, 60), (3000, 0, 120), (400, 50, 300), (60000, 1000, 200),
                   (30, 10, 100), (0, 40, 7), (1000, 0, 1000)]


@pytest.mark.parametrize("n_plus,nminus,amount", SUBSAMPLE_CASES)
def test_subsample_reference_host_oracle_python_agree(host, oracle_mod, n_plus, nminus, amount):
    rng = np.random.default_rng(n_plus + amount)
    nplus = rng.integers(1, 90, max(n_plus, 1)).astype(np.uint16)[:n_plus]
    seed, stream = 42, 420 + 3
    for start in (0, 1, 63, 64, 1000):  # word positions: fresh, odd, a 4-block buffer boundary, mid-stream
        wh = C.c_uint64(start)
        out = np.zeros(max(1, n_plus), np.uint16)
        onp, onm = C.c_uint64(), C.c_uint64()
        assert host.ecdna_host_subsample_reference(nplus.ctypes.data if n_plus else None, n_plus, nminus, amount,
                                                   seed, stream, C.byref(wh), out.ctypes.data, C.byref(onp),
                                                   C.byref(onm)) == 0
        cells, wo = oracle_mod.compat_subsample(nplus, nminus, amount, seed, stream, start)
        assert wh.value == wo
        assert sorted(out[: onp.value].tolist()) == sorted(int(c) for c in cells if c) and onm.value == int(
            np.sum(cells == 0))
        assert onp.value + onm.value == min(amount, n_plus + nminus)
        ch = oracle_mod.ChaCha(seed, stream)
        for _ in range(start):
            ch.next_u32()
        used = [0]

        def nxt():
            used[0] += 1
            return ch.next_u32()

        alg, idx = _index_sample_py(nxt, n_plus + nminus, min(amount, n_plus + nminus))
        want = [0 if i < nminus else int(nplus[i - nminus]) for i in idx]
        assert cells.tolist() == want, alg
        assert wo == start + used[0]


def test_subsample_reference_chains_words(host, oracle_mod):
    """Consecutive subsamples of one replicate continue the stream where the previous one stopped (the reference's
    `for nb_cells in samples` loop reuses one rng): the word position advances by exactly the words drawn."""
    nplus = np.arange(1, 501, dtype=np.uint16)
    w = 777
    for amount in (10, 100, 200):
        _, w2 = oracle_mod.compat_subsample(nplus, 20, amount, 7, 71, w)
        assert w2 > w
        wh = C.c_uint64(w)
        out = np.zeros(500, np.uint16)
        onp, onm = C.c_uint64(), C.c_uint64()
        host.ecdna_host_subsample_reference(nplus.ctypes.data, 500, 20, amount, 7, 71, C.byref(wh), out.ctypes.data,
                                            C.byref(onp), C.byref(onm))
        assert wh.value == w2
        w = w2


def test_oracle_compat_reports_stream_positions(oracle_mod):
    """The compat oracle's per-replicate stream position: a replicate that drew nothing stands at 0; a pure-birth
    replicate from one cell to 2 cells drew exactly one Exp1 (two words per next_u64 unless the ziggurat rejects)
    plus its segregation and pick words; positions grow with the run."""
    from ecdna_evo_amd import abi

    spec = abi.RunSpec(seed=5, n_replicates=64, max_cells=200, flags=0)
    r = oracle_mod.run(spec, mode="compat")
    assert r.rng_words.shape == (64,) and np.all(r.rng_words > 0)
    assert np.all(r.rng_words % 1 == 0)
    big = oracle_mod.run(abi.RunSpec(seed=5, n_replicates=64, max_cells=400, flags=0), mode="compat")
    assert np.all(big.rng_words >= r.rng_words)  # the same streams, run further


def test_rendezvous_all_or_none(tmp_path):
    """the --pooled rendezvous with the RCCL reduction stubbed (tests/native/rendezvous_check.cpp): all
    shards OK -> every thread runs the collective; one shard failing -> none does, the failed one keeps its own error
    and the others report the peer failure (ecdna::host::kPeerFailed), never hanging."""
    exe = tmp_path / "rendezvous_check"
    src = os.path.join(REPO, "tests", "native", "rendezvous_check.cpp")
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-I", os.path.join(REPO, "ecdna-evo_amd", "host"), src,
                    "-o", str(exe)], check=True)

    def run(flags):
        out = subprocess.run([str(exe), flags], capture_output=True, text=True, timeout=30, check=True).stdout
        calls, rcs = out.strip().split()
        return int(calls.split("=")[1]), [int(x) for x in rcs.split("=")[1].split(",")]

    assert run("1") == (1, [0])
    assert run("1111") == (4, [0, 0, 0, 0])
    calls, rc = run("1101")
    assert calls == 0 and rc == [-1000, -1000, -2, -1000]
    calls, rc = run("0000")
    assert calls == 0 and rc == [-2, -2, -2, -2]
