"""Draw mapping v7 / v8 on the CPU: the exact law of the channel pick and of the time draw (v8 = v7
with the time step as a product with the correctly rounded reciprocal of a0).

Channel (v7). The propensities are the reference's own f32 products rate_i * pop_i (src/main.rs:67, 139); their
cumulative sums c_0 <= c_1 <= c_2 <= A are formed in f64, and the channel is the number of c_i <= target with
target = RN64(u A), u = (w1 + 0.5) 2^-32 from all 32 bits of the event's word w1. The target is non-decreasing in w1,
so the words drawing channel i form one interval, found here by binary search over the oracle's own channel function
(oracle_channel, the code path of its stepper). Hence the exact probability of every channel under the mapping:
within 2^-32 (plus f64 rounding) of lambda_i / sum(lambda). The previous mapping (v6: u = ((w1 >> 9) + 0.5) 2^-23 and
f32 cumulative sums) is restated in numpy for contrast: it could not draw a channel below ~2^-24 of the
total, and biased small ones (one N- cell among 1e6 N+ cells: -4.6 %; among 1e7: +19 %; among 1.7e7: never).

Time draw (v6 = v7 = v8). tau = softlog(w0) / a0 (v8: softlog(w0) * RN32(1 / a0), within one ulp of
the quotient) with softlog(w0) = -ln u0, u0 = ((w0 >> 9) + 0.5) 2^-23,
so the draw Exp(1) * a0 takes one of 2^23 values, each with probability 2^-23. All 2^23 soft-log values are enumerated
through the oracle (the same f32 operations as the kernel) and compared with Exp(1): the KS distance, the mean, the
second moment and the tail masses P(X > x). (The total variation distance between a discrete law and Exp(1) is 1 for
any discretization, so it does not measure the draw; the KS distance does.) The reference draws Exp1 by the
ziggurat from 64-bit words and casts to f32 (rand_distr 0.4.3)."""
import math
import os
import shutil
import subprocess
from fractions import Fraction

import numpy as np
import pytest

f32 = np.float32
TWO32 = 1 << 32
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ------------------------------------------------------------------------------------------------ channel, v7

def test_channel_uniform_is_exact_and_inside_the_open_interval():
    for w in (0, 1, 511, 512, 2**31, 2**32 - 512, 2**32 - 1):
        u = math.fsum([w * 2.0**-32, 2.0**-33])  # = fma(w, 2^-32, 2^-33): w + 0.5 has 33 significant bits
        assert Fraction(u) == Fraction(2 * w + 1, 2**33)
        assert 2.0**-33 <= u <= 1 - 2.0**-33


def test_target_stays_inside_zero_and_the_total():
    """u at its extremes times any f64 total in the stepper's range (f32 propensities of rates in [2^-60, 2^60] times
    u32 populations) rounds strictly inside (0, A): neither a zero-propensity last channel (c_2 == A) nor a
    zero-propensity first channel (c_0 == 0) is ever drawn."""
    umax, umin = 1 - 2.0**-33, 2.0**-33
    rng = np.random.default_rng(7)
    A = np.ldexp(rng.uniform(1.0, 2.0, 20000), rng.integers(-60, 95, 20000))
    pow2 = np.ldexp(1.0, np.arange(-60, 95))
    for a in (A, pow2, np.nextafter(pow2, np.inf), np.nextafter(pow2, 0)):
        assert np.all(umax * a < a)
        assert np.all(umin * a > 0)


def _bounds(oracle_mod, rates, nm, np_, bd):
    """first word w drawing a channel >= i, for i = 1, 2, 3 (the channel is non-decreasing in w)."""
    out = []
    for i in (1, 2, 3):
        lo, hi = 0, TWO32  # invariant: ch(lo - 1) < i <= ch(hi) (hi = 2^32: past the last word)
        while lo < hi:
            mid = (lo + hi) // 2
            if oracle_mod.channel(rates, nm, np_, bd, mid) >= i:
                hi = mid
            else:
                lo = mid + 1
        out.append(lo)
    return out


def _lambdas(rates, nm, np_, bd):
    """the reference's f32 propensities rate_i * pop_i over [n-, n+, n-, n+] (src/main.rs:67, 139) as exact rationals"""
    lam = [f32(rates[0]) * f32(nm), f32(rates[1]) * f32(np_)]
    lam += [f32(rates[2]) * f32(nm), f32(rates[3]) * f32(np_)] if bd else [f32(0), f32(0)]
    return [Fraction(float(x)) for x in lam]


STATES = [  # (rates b0 b1 d0 d1, n-, n+, birth_death)
    ((1.0, 1.0, 0.0, 0.0), 1, 1_000_000, False),
    ((1.0, 1.0, 0.0, 0.0), 1, 10_000_000, False),
    ((1.0, 1.0, 0.0, 0.0), 1, 17_000_000, False),  # one N- cell among 1.7e7+ N+ cells
    ((1.0, 1.0, 0.0, 0.0), 1_000_000, 1, False),
    ((1.0, 1.0, 0.0, 0.0), 5, 3, False),
    ((1.0, 1.5, 0.3, 0.3), 1, 1_000_000, True),
    ((1.0, 1.5, 0.3, 0.3), 1, 10_000_000, True),  # DeathNMinus between two large channels
    ((1.0, 1.5, 0.3, 0.3), 10_000_000, 1, True),
    ((1.0, 1.5, 0.3, 0.3), 3_000, 7_000, True),
    ((1.0, 1.0, 0.9, 0.9), 1_000, 999_000, True),  # C5's turnover near its cap
    ((1.0, 1.0, 1e-9, 1.0), 1, 1, True),  # rate ratio 1e-9
    ((1e-9, 1.0, 1.0, 1.0), 1, 1, True),
    ((1.0, 1.0, 1.0, 1e-9), 1_000, 1_000, True),
    ((0.0, 1.5, 0.3, 0.3), 5, 5, True),  # zero rates: their channel never fires
    ((1.0, 0.0, 0.3, 0.3), 5, 5, True),
    ((1.0, 1.5, 0.0, 0.3), 5, 5, True),
    ((1.0, 1.5, 0.3, 0.0), 5, 5, True),
    ((1.0, 1.5, 0.3, 0.3), 0, 5, True),  # no N- cells
    ((1.0, 1.5, 0.3, 0.3), 5, 0, True),  # no N+ cells
    ((2.0**-60, 2.0**60, 2.0**-60, 2.0**60), 1, 1, True),  # the ABI's rate range ends
]


@pytest.mark.parametrize("rates,nm,np_,bd", STATES)
def test_channel_law_is_exact_to_2_pow_minus_32(oracle_mod, rates, nm, np_, bd):
    """P(channel i) = (words drawing i) / 2^32 is within 2^-32 (+ f64 rounding of the sums and the target) of
    lambda_i / sum(lambda); a channel of zero propensity has no word; every channel above 2^-32 has one."""
    b = _bounds(oracle_mod, rates, nm, np_, bd)
    counts = [b[0], b[1] - b[0], b[2] - b[1], TWO32 - b[2]]
    lam = _lambdas(rates, nm, np_, bd)
    tot = sum(lam)
    for i in range(4):
        p = lam[i] / tot
        got = Fraction(counts[i], TWO32)
        assert abs(got - p) <= Fraction(1, TWO32) + Fraction(1, 2**45), (i, counts, float(p))
        if lam[i] == 0:
            assert counts[i] == 0, (i, counts)
        if p >= Fraction(1, 2**31):
            assert counts[i] > 0, (i, counts)


def _v6_channel_probs(rates, nm, np_, bd):
    """the previous mapping (v6), restated: u = ((w1 >> 9) + 0.5) 2^-23 (f32), target = RN32(u a0), f32 cumulative sums;
    each of the 2^23 values of u stands for 512 words."""
    fm, fp = f32(nm), f32(np_)
    a = [f32(rates[0]) * fm, f32(rates[1]) * fp]
    a += [f32(rates[2]) * fm, f32(rates[3]) * fp] if bd else [f32(0), f32(0)]
    c0 = a[0]
    c1 = f32(c0 + a[1])
    c2 = f32(c1 + a[2])
    a0 = f32(c2 + a[3])
    u = (np.arange(1 << 23, dtype=np.float32) * f32(2.0**-23) + f32(2.0**-24)).astype(np.float32)
    t = (u * a0).astype(np.float32)
    ch = (t >= c0).astype(np.int64) + (t >= c1) + (t >= c2)
    return np.bincount(ch, minlength=4) / float(1 << 23)


def test_v6_channel_bias_that_v7_removes(oracle_mod):
    """ADVICE r04's cases: one N- cell among n+ N+ cells at b0 = b1 (pure birth). v6 drew ProliferateNMinus with
    8 2^-23 (-4.6 %) at n+ = 1e6, 2^-23 (+19 %) at 1e7 and never at 1.7e7; birth-death at n+ = 1e7 also lost
    DeathNMinus (0.3 / 1.8e7) in the f32 cumulative sum. v7 is within 2^-32 of every one."""
    want = {1_000_000: -0.046, 10_000_000: 0.19, 17_000_000: -1.0}
    for np_, rel in want.items():
        p_true = 1.0 / (np_ + 1.0)
        p6 = _v6_channel_probs((1.0, 1.0, 0.0, 0.0), 1, np_, False)[0]
        assert abs((p6 - p_true) / p_true - rel) < 0.01, (np_, p6, p_true)
        b = _bounds(oracle_mod, (1.0, 1.0, 0.0, 0.0), 1, np_, False)
        assert abs(b[0] / TWO32 - p_true) <= 2.0**-32
    p6 = _v6_channel_probs((1.0, 1.5, 0.3, 0.3), 1, 10_000_000, True)
    assert p6[2] == 0.0  # DeathNMinus lost in f32
    b = _bounds(oracle_mod, (1.0, 1.5, 0.3, 0.3), 1, 10_000_000, True)
    p_dm = 0.3 / (1.0 + 1.5e7 + 0.3 + 3e6)
    assert abs((b[2] - b[1]) / TWO32 - p_dm) <= 2.0**-32


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc absent")
def test_kernel_header_channel_matches_the_oracle(tmp_path, oracle_mod):
    """The stepper header's chan_target (ecdna-evo_amd/csrc/ssa_device.hpp, host-callable) with the steppers'
    propensity sequence, compiled for the host and compared with oracle_channel over 1.7M cases: random rates in
    the accepted range (and zeros), populations 0 .. 2^32 - 1, and the words either side of every boundary
    (tests/native/device_math_check.cpp). Guards the kernels' channel arithmetic on a machine without a GPU. Then the
    header's rcp_newton (the time step's reciprocal, draw mapping v8) against RN32(1 / d)."""
    exe = tmp_path / "device_math_check"
    subprocess.run(["hipcc", "-x", "hip", "--offload-host-only", "-std=c++17", "-O1", "-I",
                    os.path.join(REPO, "ecdna-evo_amd", "csrc"), os.path.join(REPO, "tests", "native",
                                                                              "device_math_check.cpp"),
                    "-L", os.path.join(REPO, "oracle", "_build"), "-lecdna_oracle",
                    "-Wl,-rpath," + os.path.join(REPO, "oracle", "_build"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("mismatches=0")
    # the time step's reciprocal (draw mapping v8): the Newton step gives RN32(1 / d) from either faithful start, for
    # every d of a binade and 2M random d over [2^-60, 2^95), except from RD at mantissa 0x7fffff (counted as known;
    # the GPU's rcp is RU there: tools/rcp_check.hip, tests/test_gpu_rcp.py)
    rcp = dict(kv.split("=") for kv in out.stdout.split("\n")[0].split())
    assert int(rcp["rcp_cases"]) >= 2 * (2**23 + 2_000_000) and int(rcp["rcp_off"]) == 0, out.stdout
    assert int(rcp["rcp_known"]) >= 1


def test_time_step_operands_stay_normal():
    """Soft log in [2^-24, 24 ln 2] times RN32(1 / a0), a0 = RN32(A) in [2^-60, 2^94] (draw mapping v8): the
    reciprocal, the Newton residual and the product are all normal f32 numbers (>= 2^-126) and finite, the range over
    which rcp_rn is RN32(1 / d) (checked for every f32 in [2^-60, 2^95) on the GPU)."""
    tiny = np.finfo(np.float32).tiny
    n_min, n_max = 2.0**-24, 24 * np.log(2.0)
    d_min, d_max = 2.0**-60, 2.0**94
    assert n_min / d_max >= tiny and n_max / d_min < np.finfo(np.float32).max
    assert 1.0 / d_max >= tiny and 1.0 / d_min < np.finfo(np.float32).max
    assert n_min * 2.0**-24 >= tiny
    # the largest total propensity: four rates of 2^60 times u32 populations
    assert 4 * 2.0**60 * (2.0**32 - 1) <= d_max


# ------------------------------------------------------------------------------------------------ time draw

@pytest.fixture(scope="module")
def softlog_law(oracle_mod):
    """the 2^23 values of the time draw (one per value of w0 >> 9), ascending, each with probability 2^-23"""
    v = oracle_mod.softlog_many(np.arange(1 << 23, dtype=np.uint32) << 9).astype(np.float64)
    assert np.all(np.diff(v) <= 0)  # -ln u is decreasing in u, and so is the soft log
    return v[::-1].copy()


# the bounds DESIGN.md §3 quotes for the time draw of mappings v6 / v7 (measured: KS 9.45e-8 = 1.59 2^-24 at x = 0.51,
# mean - 1 = -4.16e-8, E[X^2] - 2 = -1.50e-6)
KS_BOUND = 1.0e-7
MEAN_BOUND = 5.0e-8


def test_time_draw_ks_distance_to_exp1(softlog_law):
    """sup_x |F(x) - (1 - e^-x)| over the discrete law: at each value the CDF jumps by 2^-23 across the exponential CDF,
    so the distance is at least half a jump (2^-24, what exact -ln of the cells' midpoints gives); rounding the values
    to f32 moves the jumps (1.37 2^-24 for correctly rounded -ln) and the soft log's <= 1.1 ulp error a little more:
    1.59 2^-24 = 9.45e-8."""
    s = softlog_law
    n = len(s)
    g = -np.expm1(-s)  # Exp(1) CDF at the jump points
    j = np.arange(n, dtype=np.float64)
    ks = max(np.max(np.abs(j / n - g)), np.max(np.abs((j + 1) / n - g)))
    assert ks <= KS_BOUND, ks
    assert ks >= 2.0**-24  # (not less than the half jump: the draw's resolution is 2^-23)


def test_time_draw_moments_and_tail(softlog_law):
    s = softlog_law
    mean = s.mean()
    m2 = np.mean(s * s)
    assert abs(mean - 1.0) <= MEAN_BOUND, mean - 1.0
    assert abs(m2 - 2.0) <= 2e-6, m2 - 2.0  # (the top cell, u < 2^-23, carries its mass at 16.64: -1.5e-6)
    # tail masses P(X > x) against e^-x: within one jump (2^-23) everywhere, and cut above the largest value
    n = len(s)
    for x in (1.0, 5.0, 10.0, 14.0, 15.0, 16.0, 16.5):
        p = (n - np.searchsorted(s, x, side="right")) / n
        assert abs(p - math.exp(-x)) <= 2.0**-23, (x, p, math.exp(-x))
    top = s[-1]
    assert 16.63 < top < 16.64  # -ln(2^-24) = 16.636: the tail is cut there, P(Exp(1) > 16.636) = 2^-24
    assert abs(math.exp(-top) - 2.0**-24) < 1e-12
