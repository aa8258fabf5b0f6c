"""The reference-semantics (compat) mapping's transcendental functions and constant tables.

The reference calls glibc's log and exp (Rust f64::ln / f64::exp) inside rand_distr's Exp1 ziggurat and BTPE
binomial. The compat mapping defines them as the CORRECTLY ROUNDED functions, restated on the CPU
(oracle/ssa_compat.c) and the GPU (ecdna-evo_amd/csrc/refdraws.hpp: log_cr / exp_cr / exp_approx) with the same operations, so the two
agree bit for bit. These tests pin:
  * compat_log / compat_exp against exact decimal arithmetic (correct rounding), and
  * against glibc (what the Rust reference calls): equal except where glibc itself misrounds (it guarantees
    0.52 ulp, not correct rounding), there by exactly one ulp;
  * the ziggurat tables against rand's generator as restated in tools/gen_compat_tables.py, and the
    generated headers (product and oracle copies) against the generator.
"""
import math
import os
import random
import subprocess
import sys
from decimal import Decimal, getcontext

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ulps(a: float, b: float) -> int:
    return abs(int(np.float64(a).view(np.int64)) - int(np.float64(b).view(np.int64)))


def _inputs_log(rng, n):
    xs = [rng.random() for _ in range(n)]                              # gen::<f64>() (ziggurat tail), BTPE v
    xs += [rng.uniform(0.5, 3.0) for _ in range(n)]                    # BTPE ratios f1/x1, z/w, ...
    xs += [1.0 + rng.uniform(-1e-3, 1e-3) for _ in range(n)]           # near ln 1 = 0
    xs += [math.ldexp(rng.random() + 0.5, rng.randint(-1070, 1020)) for _ in range(n)]  # whole range
    xs += [5e-324, 2.2250738585072014e-308, 1.0, 2.0, 0.5, 1.41796875, 1.41796875 - 2**-52, 0.70898437500001]
    return [x for x in xs if x > 0]


def test_compat_log_is_correctly_rounded(oracle_mod):
    getcontext().prec = 60
    rng = random.Random(7)
    for x in _inputs_log(rng, 1500):
        assert oracle_mod.compat_log(x) == float(Decimal(x).ln()), x
    assert oracle_mod.compat_log(0.0) == -math.inf and oracle_mod.compat_log(math.inf) == math.inf
    assert math.isnan(oracle_mod.compat_log(-1.0))


def test_compat_exp_is_correctly_rounded(oracle_mod):
    getcontext().prec = 60
    rng = random.Random(8)
    ys = [-rng.uniform(0, 7.7) for _ in range(3000)]                   # the ziggurat's pdf(x) = e^-x, x < R
    ys += [rng.uniform(-22, 22) for _ in range(1500)] + [rng.uniform(-1e-3, 1e-3) for _ in range(1500)]
    ys += [0.0, -7.697117470131050, 1e-300, -1e-300]
    for y in ys:
        assert oracle_mod.compat_exp(y) == float(Decimal(y).exp()), y


def test_exp_filter_error_bound(oracle_mod):
    """The GPU's wedge test decides lhs < exp_cr(-x) with a plain-double e^-x whenever lhs is further than
    2^-40 (relative) from it (csrc/refdraws.hpp lt_exp_cr); that is exact provided the plain value is within
    2^-41 of e^y. Its restatement is within 2^-48 here, over the ziggurat's range and beyond."""
    getcontext().prec = 60
    rng = random.Random(9)
    ys = [-rng.uniform(0, 7.7) for _ in range(6000)] + [-rng.uniform(0, 22) for _ in range(2000)]
    ys += [0.0, -7.697117470131050, -1e-300, -22.0]
    worst = 0.0
    for y in ys:
        exact = Decimal(y).exp()
        err = abs((Decimal(oracle_mod.compat_exp_approx(y)) - exact) / exact)
        worst = max(worst, float(err))
    assert worst < 2.0 ** -48, worst


def test_log_filter_error_bound(oracle_mod):
    """BTPE's region-3/4 step truncates x +- ln(v) / lambda (csrc/refdraws.hpp trunc_log_ratio) from a plain-double
    ln v wherever the result is clear of an integer by 2^-30; exact provided log_approx is within ~2^-38 lambda of
    ln v (lambda >= 2^-7). Its restatement is within 2^-45 (absolute) over BTPE's inputs v in [2^-52, 1) (multiples of
    2^-52: float_1_2(bits) - 1), the smallest and the values next to 1 included."""
    getcontext().prec = 60
    rng = random.Random(13)
    vs = [rng.randrange(1, 1 << 52) * 2.0 ** -52 for _ in range(6000)]
    vs += [rng.randrange(1, 1 << 20) * 2.0 ** -52 for _ in range(1000)]  # far tail
    vs += [2.0 ** -52, 1.0 - 2.0 ** -52, 0.5, 0.5 - 2.0 ** -52, 0.70898, 0.708984375, 0.99, 2.0 ** -26]
    worst = 0.0
    for v in vs:
        err = abs(Decimal(oracle_mod.compat_log_approx(v)) - Decimal(v).ln())
        worst = max(worst, float(err))
    assert worst < 2.0 ** -45, worst


@pytest.mark.parametrize("n", [20, 22, 24, 30, 40, 41 * 2, 64, 128, 256, 1000, 4096, 65534])
def test_btpe_explicit_ratio_filter_error_bound(n):
    """BTPE's explicit acceptance v > f (k = |y - m| <= 20; csrc/refdraws.hpp) is decided first from
    fa = prod(n + 1 - i) / prod(i) (or its inverse) wherever v is clear of it by 2^-40 relative: exact provided fa and
    the loop's f (f *= a / i - s per factor, f /= ... for y < m; the reference's operations, restated with Python's
    IEEE doubles) are each within 2^-41 of the real ratio C(n, y) / C(n, m). Both are, for every y with |y - m| <= 20
    in [0, n] and the BTPE m of Binomial(n, 1/2)."""
    from fractions import Fraction

    p = q = 0.5
    s = p / q
    a = s * (n + 1.0)
    m = int(n * p + p)  # (f_m = n p + p, m = f_m as i64)
    worst_f, worst_fa = 0.0, 0.0
    for y in range(max(0, m - 20), min(n, m + 20) + 1):
        f, num, den = 1.0, 1.0, 1.0
        exact = Fraction(1)
        lo, hi = (m, y) if m < y else (y, m)
        for i in range(lo + 1, hi + 1):
            if m < y:
                f *= a / float(i) - s
            else:
                f /= a / float(i) - s
            num *= n + 1.0 - float(i)
            den *= float(i)
            exact *= Fraction(n + 1 - i, i)
        if m > y:
            exact = 1 / exact
        fa = num / den if m < y else (den / num if m > y else 1.0)
        worst_f = max(worst_f, abs(float((Fraction(f) - exact) / exact)))
        worst_fa = max(worst_fa, abs(float((Fraction(fa) - exact) / exact)))
    assert worst_f < 2.0 ** -41 and worst_fa < 2.0 ** -41, (worst_f, worst_fa)


def test_binv_cdf_filter_agrees_with_the_loop():
    """BINV (rand_distr's n p < 10 branch, n = 2 .. 18): the GPU counts x = #{y : P_y < u} over the running sums P_y of
    the loop's r values (csrc/refdraws.hpp binv_cdf / binv_half) and keeps x only where u is clear of P_x and P_x+1 by
    2^-40 (and x <= n); else it runs the loop. Restated with Python's IEEE doubles: wherever the filter decides it
    equals the reference's loop, over 40,000 uniforms per n (random, and next to every P_y)."""
    rng = random.Random(17)
    s = 0.5 / 0.5
    for n in range(2, 20, 2):
        a = (n + 1) * s
        P, r, acc = [0.0], 2.0 ** -n, 0.0
        for y in range(1, 21):
            acc += r
            P.append(acc)
            r *= a / float(y) - s

        def loop(u):
            r, x = 2.0 ** -n, 0
            while u > r:
                u -= r
                x += 1
                if x > 110:
                    return None  # (restart)
                r *= a / float(x) - s
            return x

        us = [rng.getrandbits(53) * 2.0 ** -53 for _ in range(40_000)]
        us += [math.nextafter(p_, d) for p_ in P[1:] for d in (0.0, 2.0)] + [p_ + e for p_ in P[1:] for e in (2.0 ** -39, -2.0 ** -39)]
        decided = 0
        for u in us:
            if not 0.0 <= u < 1.0:
                continue
            x = sum(1 for y in range(1, 20) if P[y] < u)
            if x <= n and u - P[x] > 2.0 ** -40 and P[x + 1] - u > 2.0 ** -40:
                decided += 1
                assert loop(u) == x, (n, u, x, loop(u))
        assert decided > 0.99 * 40_000


@pytest.mark.parametrize("fn,gen", [
    ("log", lambda r: r.random() or 0.5),
    ("log", lambda r: r.uniform(0.5, 3.0)),
    ("exp", lambda r: -r.uniform(0, 7.7)),
])
def test_compat_math_agrees_with_glibc(oracle_mod, fn, gen):
    """glibc's log/exp (what Rust's f64::ln / f64::exp call on Linux) round correctly almost always: the compat
    functions equal them except on the rare inputs glibc misrounds (within its 0.52 ulp bound), and there
    they differ by one ulp and are the correctly rounded value."""
    getcontext().prec = 60
    rng = random.Random(11)
    f_c = oracle_mod.compat_log if fn == "log" else oracle_mod.compat_exp
    f_g = math.log if fn == "log" else math.exp
    n, diff = 100_000, 0
    for _ in range(n):
        x = gen(rng)
        a, b = f_c(x), f_g(x)
        if a != b:
            diff += 1
            assert _ulps(a, b) == 1, (x, a, b)
            exact = Decimal(x).ln() if fn == "log" else Decimal(x).exp()
            assert abs(Decimal(a) - exact) < abs(Decimal(b) - exact), (x, a, b)
    assert diff / n < 2e-3, diff


def _gen():
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gen_compat_tables

    return gen_compat_tables


def test_ziggurat_tables_follow_rands_generator():
    """rand_distr 0.4.3 ziggurat_tables.rs: ZIG_EXP_X / ZIG_EXP_F as rand's ziggurat_tables.py generates them
    (R = 7.69711747013104972, V = 0.0039496598225815571993, 256 layers, '%.18f' literals)."""
    g = _gen()
    r, x, f = g.zig_exp_tables()
    assert len(x) == len(f) == 257 and x[1] == r and x[256] == 0.0
    assert r == float("7.697117470131050077") and x[0] == float("8.697117470131052741")
    assert all(x[i] > x[i + 1] for i in range(256)) and all(f[i] < f[i + 1] for i in range(256))
    # every layer has area V: x_i (f(x_{i+1}) - f(x_i)) = V (up to the '%.18f' rendering), base strip R f(R) + tail
    v = 0.0039496598225815571993
    for i in range(1, 255):
        assert abs(x[i] * (f[i + 1] - f[i]) - v) < 1e-12, i
    assert abs(x[0] * f[1] - v) < 1e-15


def test_generated_compat_headers_are_current():
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_compat_tables.py"), "--check"],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
