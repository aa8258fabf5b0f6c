"""Known-answer and distribution tests of the oracle's RNG primitives (CPU only).

Philox4x32-10: the Random123 known-answer vectors (the same constants rocRAND uses,
/opt/rocm/include/rocrand/rocrand_philox4x32_10.h). ChaCha: RFC 7539 block vectors (20 rounds);
the reference's ChaCha8Rng is the same block function with 8 rounds (rand_chacha 0.3.1,
Cargo.lock:813-821). rand/rand_distr samplers: checked against their target laws.
"""
import math
import os

import numpy as np
import pytest
from scipy import stats


def test_philox_known_answers(oracle_mod):
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, want in kat:
        assert oracle_mod.philox(ctr, key) == want


def _philox_py(ctr, key):
    """Independent pure-Python Philox4x32-10 (Salmon et al. 2011)."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c = list(ctr)
    k0, k1 = key
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF, ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF,
             p0 & 0xFFFFFFFF]
    return c


def test_philox_matches_python_restatement(oracle_mod):
    rng = np.random.default_rng(1)
    for _ in range(200):
        ctr = [int(x) for x in rng.integers(0, 2**32, 4)]
        key = [int(x) for x in rng.integers(0, 2**32, 2)]
        assert oracle_mod.philox(ctr, key) == _philox_py(ctr, key)


def test_softlog_accuracy(oracle_mod):
    """Draw mapping v6: the f32 soft log of u = ((w >> 9) + 0.5) 2^-23 is within 2^-22 relative of
    -ln u (measured: 1.1 ulp over 2e5 random words), strictly positive, and at most 24 ln 2 (w < 512)."""
    ws = [0, 1, 2, 3, 511, 512, 2**31 - 1, 2**31, 2**32 - 1, 0x5A827999, 0x6A09E667]
    ws += [int(x) for x in np.random.default_rng(2).integers(0, 2**32, 3000)]
    for w in ws:
        want = -math.log(((w >> 9) + 0.5) / 2**23)
        got = oracle_mod.softlog_neg(w)
        assert abs(got - want) <= 2.0**-22 * want, (w, got, want)
        assert 0.0 < got <= 24 * math.log(2) * (1 + 2.0**-22)


def test_chacha20_rfc7539_block(oracle_mod):
    # RFC 7539 §2.3.2: key 00..1f, block counter 1, nonce 00:00:00:09:00:00:00:4a:00:00:00:00
    key = [int.from_bytes(bytes(range(i, i + 4)), "little") for i in range(0, 32, 4)]
    state = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + key + [1, 0x09000000, 0x4A000000, 0]
    out = oracle_mod.chacha_block(state, 20)
    assert out[:4] == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3]
    assert out[-1] == 0x4E3C50A2
    # RFC 7539 A.1 test vector #1: all-zero key, counter and nonce
    state = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + [0] * 12
    out = oracle_mod.chacha_block(state, 20)
    assert out[:2] == [0xADE0B876, 0x903DF1A0]


def _pcg32_key(seed):
    MUL, INC = 6364136223846793005, 11634580027462260723
    key, s = [], seed
    for _ in range(8):
        s = (s * MUL + INC) & (2**64 - 1)
        xs = (((s >> 18) ^ s) >> 27) & 0xFFFFFFFF
        rot = s >> 59
        key.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF)
    return key


def test_seed_from_u64_pcg32(oracle_mod):
    # rand_core 0.6.4 SeedableRng::seed_from_u64 (Cargo.lock:823-829), restated independently.
    for seed in (0, 1, 26, 42, 2**63 + 5):
        assert oracle_mod.chacha_key_from_u64(seed) == _pcg32_key(seed)
    assert oracle_mod.chacha_key_from_u64(42)[:2] == [0x7BA18FA4, 0x0A3D3258]


def test_chacha8_stream_layout(oracle_mod):
    """ChaCha8Rng: 4-block buffer of consecutive counters, stream in words 14-15, next_u64 low word first
    (also across the refill boundary at index 63)."""
    seed, stream = 42, 420
    key = _pcg32_key(seed)
    base = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + key
    words = []
    for ctr in range(16):
        words += oracle_mod.chacha_block(base + [ctr, 0, stream & 0xFFFFFFFF, stream >> 32], 8)
    r = oracle_mod.ChaCha(seed, stream)
    got = [r.next_u32() for _ in range(200)]
    assert got == words[:200]
    r = oracle_mod.ChaCha(seed, stream)
    for _ in range(63):
        r.next_u32()
    x = r.next_u64()  # straddles the 64-word buffer
    assert x == words[63] | (words[64] << 32)
    assert r.next_u32() == words[65]


def test_gen_range_widening_multiply(oracle_mod):
    r1, r2 = oracle_mod.ChaCha(7, 70), oracle_mod.ChaCha(7, 70)
    for n in [1, 2, 3, 7, 1000, 2**33 + 17]:
        for _ in range(50):
            zone = ((n << (64 - n.bit_length())) & (2**64 - 1)) - 1
            while True:
                v = r2.next_u64()
                m = v * n
                if (m & (2**64 - 1)) <= zone:
                    want = m >> 64
                    break
            assert r1.gen_range(n) == want


def test_exp1_ziggurat_law(oracle_mod):
    r = oracle_mod.ChaCha(3, 30)
    x = np.array([r.exp1() for _ in range(60000)])
    assert stats.kstest(x, "expon").pvalue > 1e-3
    assert abs(x.mean() - 1.0) < 0.02


@pytest.mark.parametrize("n", [2, 6, 18, 40, 200, 2000, 65534])
def test_binomial_half_law(oracle_mod, n):
    """rand_distr Binomial(n, 1/2): BINV for n*p < 10, BTPE above — chi-square against the exact pmf."""
    r = oracle_mod.ChaCha(11, n)
    N = 40000
    x = np.array([r.binomial(n, 0.5) for _ in range(N)])
    assert x.min() >= 0 and x.max() <= n
    sd = math.sqrt(n) / 2
    lo, hi = int(max(0, n / 2 - 4 * sd)), int(min(n, n / 2 + 4 * sd))
    edges = np.unique(np.linspace(lo, hi + 1, min(hi - lo + 2, 25)).astype(int))
    obs = np.histogram(np.clip(x, lo, hi), bins=edges)[0]
    cdf = stats.binom.cdf(edges - 1, n, 0.5)
    exp = np.diff(cdf) * N
    exp[0] += stats.binom.cdf(lo - 1, n, 0.5) * N
    exp[-1] += stats.binom.sf(hi, n, 0.5) * N
    keep = exp > 5
    chi = ((obs[keep] - exp[keep]) ** 2 / exp[keep]).sum()
    assert stats.chi2.sf(chi, keep.sum() - 1) > 1e-4, (n, chi)


def test_log_tables_match_generator():
    """The exponential draw's log table (draw mapping v6, f32) is the generator's output, identical in the
    product (ecdna-evo_amd/csrc/ssa_logtab.h) and in the oracle (oracle/ssa_logtab.h)."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(repo, "tools", "gen_logtab.py"), "--check"],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr


def test_softlog_near_one_keeps_relative_accuracy(oracle_mod):
    """u -> 1 (w near 2^32): -ln u is tiny (down to 2^-24); the j = 127 table entry {1, 0} avoids cancellation."""
    for w in range(2**32 - 2**15, 2**32, 67):
        want = -math.log1p(-(2**23 - (w >> 9) - 0.5) / 2**23)
        got = oracle_mod.softlog_neg(w)
        assert abs(got - want) <= 2.0**-22 * want, (w, got, want)
