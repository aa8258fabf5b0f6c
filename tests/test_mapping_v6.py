"""Draw mapping v6: the f32 channel and time-step arithmetic, checked on the CPU.

The channel draws u1 = ((w1 >> 9) + 0.5) 2^-23 (exact in f32) and picks the first cumulative propensity above
target = RN32(u1 a0). A channel of zero propensity must never be drawn; for the last channel that needs
target < a0 for every admissible a0, which holds because u1 <= 1 - 2^-24. The time step divides a soft log in
[2^-24, 24 ln 2] by a0 in [2^-60, 2^94] (ABI v8 rates), a range in which every intermediate of the kernel's
division is a normal f32 (the condition of its range argument)."""
import numpy as np

f32 = np.float32


def chan_u(w):
    return f32(w >> 9) * f32(2.0**-23) + f32(2.0**-24)  # exact: a 23-bit integer scaled, plus half an ulp


def test_channel_uniform_is_exact_and_below_one():
    for w in (0, 1, 511, 512, 2**31, 2**32 - 512, 2**32 - 1):
        u = chan_u(w)
        assert float(u) == ((w >> 9) + 0.5) / 2**23
        assert float(u) <= 1 - 2.0**-24
        assert float(u) >= 2.0**-24


def test_target_stays_below_a0_for_every_admissible_a0():
    """u1 at its maximum times any f32 a0 in the stepper's range rounds strictly below a0: a last channel of zero
    propensity (cC == a0) is never selected (powers of two, the worst case for rounding up, included)."""
    umax = chan_u(2**32 - 1)
    rng = np.random.default_rng(6)
    mant = rng.integers(0, 2**23, 20000, dtype=np.uint32)
    expo = rng.integers(127 - 60, 127 + 94, 20000, dtype=np.uint32)
    a0 = ((expo << 23) | mant).view(np.float32)
    pow2 = np.array([2.0**e for e in range(-60, 95)], dtype=np.float32)
    for a in (a0, pow2, np.nextafter(pow2, np.float32(np.inf)), np.nextafter(pow2, np.float32(0))):
        target = (umax * a).astype(np.float32)
        assert np.all(target < a)


def test_time_step_operands_stay_normal():
    """Soft log in [2^-24, 24 ln 2] over a0 in [2^-60, 2^94]: quotient, reciprocal and the Newton residual scale
    (n * 2^-24) are all normal f32 numbers (>= 2^-126) and finite."""
    tiny = np.finfo(np.float32).tiny
    n_min, n_max = 2.0**-24, 24 * np.log(2.0)
    d_min, d_max = 2.0**-60, 2.0**94
    assert n_min / d_max >= tiny and n_max / d_min < np.finfo(np.float32).max
    assert 1.0 / d_max >= tiny and 1.0 / d_min < np.finfo(np.float32).max
    assert n_min * 2.0**-24 >= tiny
    # the largest total propensity: four rates of 2^60 times u32 populations
    assert 4 * 2.0**60 * (2.0**32 - 1) <= d_max
