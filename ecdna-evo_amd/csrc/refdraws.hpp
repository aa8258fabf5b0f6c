// refdraws.hpp — device side of the reference-semantics draw mapping (ECDNA_FLAG_REFERENCE_DRAWS,
// DESIGN.md §4.1): the random-number stack the reference's hot path runs on, restated for gfx950.
//
//   rand_chacha 0.3.1 ChaCha8Rng (Cargo.lock:813-821): 8 rounds, 64-bit block counter in state words
//     12-13, stream in words 14-15; key = rand_core 0.6.4 seed_from_u64 (PCG32 expansion, on the host);
//     stream = seed * 10 + replicate id (src/main.rs:56-58, 213-215). rand_core's BlockRng hands out the
//     words of consecutive blocks in order (next_u64 = two consecutive words, low first, also across a
//     refill), so one 16-word block at a time gives the same stream as rand_chacha's 4-block buffer.
//   rand 0.8.5: gen_range(0..n) (widening multiply, zone = (n << lz(n)) - 1), gen::<f64>() (53 high bits).
//   rand_distr 0.4.3: Exp1 by the 256-layer ziggurat (tables: compat_tables.h), Exp(l) = Exp1 as f32 *
//     (1 / l); Binomial by BINV (n p < 10) or BTPE.
//   log / exp: the correctly rounded double-double functions of the compat mapping (the reference calls
//     glibc's; oracle/ssa_compat.c restates these same operations, tests/test_compat_math.py pins them).
//
// Every floating-point operation is an IEEE add/sub/mul/div/fma in the order the oracle writes it; the file
// is compiled with -ffp-contract=off and pins contraction off, so the GPU reproduces oracle/ssa_compat.c
// bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "compat_tables.h"

#pragma clang fp contract(off)

namespace ecdna {
namespace refdraws {

// ---------------------------------------------------------------- double-double arithmetic
struct dd {
    double hi, lo;
};

__device__ __forceinline__ dd two_sum(double a, double b) {
    const double s = a + b, bb = s - a;
    return dd{s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd fast_sum(double a, double b) {  // |a| >= |b| or a == 0
    const double s = a + b;
    return dd{s, b - (s - a)};
}
__device__ __forceinline__ dd add(dd a, dd b) {
    const dd s = two_sum(a.hi, b.hi);
    const double e = s.lo + (a.lo + b.lo);
    return fast_sum(s.hi, e);
}
__device__ __forceinline__ dd mul(dd a, dd b) {
    const double p = a.hi * b.hi;
    const double e = __builtin_fma(a.hi, b.hi, -p) + (a.hi * b.lo + a.lo * b.hi);
    return fast_sum(p, e);
}
__device__ __forceinline__ dd lift(double a) { return dd{a, 0.0}; }

// ln x, correctly rounded (oracle_compat_log in oracle/ssa_compat.c: the same operations). clog: the
// ECDNA_CLOG table {c_j, hi, lo} for j = 91..181 (LDS or global).
__device__ __forceinline__ double log_cr(double x, const double* clog) {
    if (!(x > 0.0)) return x == 0.0 ? -__builtin_inf() : __builtin_nan("");
    if (x == __builtin_inf()) return x;
    int64_t e = 0;
    uint64_t u = (uint64_t)__double_as_longlong(x);
    if ((u >> 52) == 0) {  // subnormal
        x = x * 0x1p54;
        u = (uint64_t)__double_as_longlong(x);
        e = -54;
    }
    e += (int64_t)(u >> 52) - 1023;
    double f = __longlong_as_double((long long)((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
    if (f >= 1.41796875) {
        f = f * 0.5;
        e += 1;
    }
    const int j = (int)(f * 128.0 + 0.5);
    const double* t = clog + 3 * (j - ECDNA_CLOG_J0);
    const double c = t[0];
    const double ph = f * c, pl = __builtin_fma(f, c, -ph);
    const dd r = two_sum(ph - 1.0, pl);
    double q = -1.0 / 14.0;
    q = __builtin_fma(r.hi, q, 1.0 / 13.0);
    q = __builtin_fma(r.hi, q, -1.0 / 12.0);
    q = __builtin_fma(r.hi, q, 1.0 / 11.0);
    q = __builtin_fma(r.hi, q, -1.0 / 10.0);
    q = __builtin_fma(r.hi, q, 1.0 / 9.0);
    q = __builtin_fma(r.hi, q, -1.0 / 8.0);
    q = __builtin_fma(r.hi, q, 1.0 / 7.0);
    dd P = lift(q);
    P = add(dd{-ECDNA_CINV6_HI, -ECDNA_CINV6_LO}, mul(r, P));
    P = add(dd{ECDNA_CINV5_HI, ECDNA_CINV5_LO}, mul(r, P));
    P = add(lift(-0.25), mul(r, P));
    P = add(dd{ECDNA_CINV3_HI, ECDNA_CINV3_LO}, mul(r, P));
    P = add(lift(-0.5), mul(r, P));
    P = add(lift(1.0), mul(r, P));
    const dd l1p = mul(r, P);
    const double ed = (double)e;
    const double eh = ed * ECDNA_CLN2_HI;
    const dd eln2 = fast_sum(eh, __builtin_fma(ed, ECDNA_CLN2_HI, -eh) + ed * ECDNA_CLN2_LO);
    dd s = add(eln2, dd{t[1], t[2]});
    s = add(s, l1p);
    return s.hi + s.lo;
}

// ln x for x in (0, 1) in plain double arithmetic (log_cr's reduction and table head, a degree-7 polynomial in r,
// |r| <= 2^-8): within 2^-45 of ln x, absolute (|ln x| <= 37 here, so e ln 2 and the final sum carry the largest
// roundings, 2^-47 each). Not correctly rounded: only used to decide integer truncations clear of their boundary
// (trunc_log_ratio), as exp_approx decides lt_exp_cr.
__device__ __forceinline__ double log_approx(double x, const double* clog) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    int64_t e = (int64_t)(u >> 52) - 1023;
    double f = __longlong_as_double((long long)((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull));
    if (f >= 1.41796875) {
        f = f * 0.5;
        e += 1;
    }
    const int j = (int)(f * 128.0 + 0.5);
    const double* t = clog + 3 * (j - ECDNA_CLOG_J0);
    const double r = __builtin_fma(f, t[0], -1.0);
    double q = __builtin_fma(r, -1.0 / 7.0, 1.0 / 6.0);  // (signs folded: ln(1 + r) = r - r^2 (1/2 - r (1/3 - ...)))
    q = __builtin_fma(r, -q, 1.0 / 5.0);
    q = __builtin_fma(r, -q, 1.0 / 4.0);
    q = __builtin_fma(r, -q, 1.0 / 3.0);
    q = __builtin_fma(r, -q, 1.0 / 2.0);
    const double l1p = __builtin_fma(-r * r, q, r);
    return __builtin_fma((double)e, ECDNA_CLN2_HI, t[1] + l1p);
}

// f64_to_i64(base + sign * log_cr(v) / lambda), BTPE's region 3 (sign = +1) and region 4 (sign = -1) step, decided
// with log_approx times inv_lambda = RN(1 / lambda) wherever the result's truncation is clear of an integer boundary by
// 2^-30 (the approximation and the exact path differ by at most ~2^-45 / lambda + a few ulp of the product and the sum:
// lambda >= 2^-7 for n <= 65534), else with the correctly rounded log and the division: the exact path's value, bit for bit, without its double-double polynomial (~150 f64
// instructions) on the common path. v == 0 (probability 2^-52) takes the exact path.
__device__ __forceinline__ int64_t trunc_log_ratio(double base, double sign, double v, double lambda, double inv_lambda,
                                                   const double* clog);

// e^y, correctly rounded for |y| <= 22 (oracle_compat_exp: the same operations). cexp: {hi, lo} of 2^(j/64).
__device__ __forceinline__ double exp_cr(double y, const double* cexp) {
    if (y != y) return y;
    if (y > 709.0) return __builtin_inf();
    if (y < -745.0) return 0.0;
    const double kd = __builtin_rint(y * ECDNA_CEXP_INV_L);
    const int64_t k = (int64_t)kd;
    const double rh = y - kd * ECDNA_CEXP_L_HI;
    const double pl = kd * ECDNA_CEXP_L_LO, ple = __builtin_fma(kd, ECDNA_CEXP_L_LO, -pl);
    dd r = two_sum(rh, -pl);
    r = fast_sum(r.hi, r.lo - ple);
    double q = 1.0 / 39916800.0;
    q = __builtin_fma(r.hi, q, 1.0 / 3628800.0);
    q = __builtin_fma(r.hi, q, 1.0 / 362880.0);
    q = __builtin_fma(r.hi, q, 1.0 / 40320.0);
    q = __builtin_fma(r.hi, q, 1.0 / 5040.0);
    dd P = lift(q);
    P = add(dd{ECDNA_CFACT6_HI, ECDNA_CFACT6_LO}, mul(r, P));
    P = add(dd{ECDNA_CFACT5_HI, ECDNA_CFACT5_LO}, mul(r, P));
    P = add(dd{ECDNA_CFACT4_HI, ECDNA_CFACT4_LO}, mul(r, P));
    P = add(dd{ECDNA_CFACT3_HI, ECDNA_CFACT3_LO}, mul(r, P));
    P = add(lift(0.5), mul(r, P));
    P = add(lift(1.0), mul(r, P));
    const dd er = add(lift(1.0), mul(r, P));
    const int64_t jj = k & 63, qq = (k - jj) / 64;
    const dd v = mul(dd{cexp[2 * jj], cexp[2 * jj + 1]}, er);
    return __builtin_ldexp(v.hi + v.lo, (int)qq);
}

// e^y for -22 <= y <= 0 in plain double arithmetic (the 2^(j/64) table head and a degree-6 polynomial):
// within about 2^-49 of e^y, relative (the head's rounding, r's reduction, six Horner roundings, the final
// product); not correctly rounded, so only used to decide comparisons against exp_cr clear of the boundary
__device__ __forceinline__ double exp_approx(double y, const double* cexp) {
    const double kd = __builtin_rint(y * ECDNA_CEXP_INV_L);
    const int64_t k = (int64_t)kd;
    const double r = (y - kd * ECDNA_CEXP_L_HI) - kd * ECDNA_CEXP_L_LO;
    double q = __builtin_fma(r, 1.0 / 720.0, 1.0 / 120.0);
    q = __builtin_fma(r, q, 1.0 / 24.0);
    q = __builtin_fma(r, q, 1.0 / 6.0);
    q = __builtin_fma(r, q, 0.5);
    q = __builtin_fma(r, q, 1.0);
    q = __builtin_fma(r, q, 1.0);
    const int64_t jj = k & 63, qq = (k - jj) / 64;
    return __builtin_ldexp(cexp[2 * jj] * q, (int)qq);
}

// lhs < exp_cr(y) for -22 <= y <= 0, the same result: exp_approx decides whenever lhs is further than
// 2^-40 (relative) from it, far beyond both functions' errors (exp_cr is within 2^-53 of e^y); otherwise
// the correctly rounded value does (about once in 2^40 comparisons)
__device__ __forceinline__ bool lt_exp_cr(double lhs, double y, const double* cexp) {
    const double a = exp_approx(y, cexp);
    if (lhs < a * (1.0 - 0x1p-40)) return true;
    if (lhs > a * (1.0 + 0x1p-40)) return false;
    return lhs < exp_cr(y, cexp);
}

// Rust's `f as i64`: saturating, NaN -> 0
__device__ __forceinline__ int64_t f64_to_i64(double x) {
    if (x != x) return 0;
    if (x >= 0x1p63) return INT64_MAX;
    if (x < -0x1p63) return INT64_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t trunc_log_ratio(double base, double sign, double v, double lambda, double inv_lambda,
                                                   const double* clog) {
    if (v > 0.0) {  // (the quotient as a product with the host's RN(1 / lambda): within 2^-52 relative more, ~2^-37 in all)
        const double ta = base + sign * (log_approx(v, clog) * inv_lambda);
        const double d = ta - __builtin_rint(ta);
        if (__builtin_fabs(d) > 0x1p-30 && __builtin_fabs(ta) < 0x1p52) return (int64_t)ta;
    }
    return f64_to_i64(base + sign * (log_cr(v, clog) / lambda));
}

// bits >> 12 as the mantissa of a value in [1, 2) (rand's into_float_with_exponent(0))
__device__ __forceinline__ double float_1_2(uint64_t bits) {
    return __longlong_as_double((long long)(0x3FF0000000000000ull | (bits >> 12)));
}

// ---------------------------------------------------------------- ChaCha8
#define ECDNA_QR(a, b, c, d)             \
    a += b;                              \
    d ^= a;                              \
    d = __builtin_rotateleft32(d, 16);   \
    c += d;                              \
    b ^= c;                              \
    b = __builtin_rotateleft32(b, 12);   \
    a += b;                              \
    d ^= a;                              \
    d = __builtin_rotateleft32(d, 8);    \
    c += d;                              \
    b ^= c;                              \
    b = __builtin_rotateleft32(b, 7);

// The ChaCha8 block (rand_chacha 0.3.1, 8 rounds) of (key, 64-bit block counter, stream) into 16 LDS words dst[i *
// stride]: the input words plus the permuted words, as rand_chacha's refill hands them out.
__device__ __forceinline__ void chacha8_block_to_lds(const uint32_t* key, uint32_t* dst, uint32_t stride, uint64_t counter,
                                                     uint32_t s_lo, uint32_t s_hi) {
    const uint32_t in[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                             key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                             (uint32_t)counter, (uint32_t)(counter >> 32), s_lo, s_hi};
    uint32_t x[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) x[i] = in[i];
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        ECDNA_QR(x[0], x[4], x[8], x[12]);
        ECDNA_QR(x[1], x[5], x[9], x[13]);
        ECDNA_QR(x[2], x[6], x[10], x[14]);
        ECDNA_QR(x[3], x[7], x[11], x[15]);
        ECDNA_QR(x[0], x[5], x[10], x[15]);
        ECDNA_QR(x[1], x[6], x[11], x[12]);
        ECDNA_QR(x[2], x[7], x[8], x[13]);
        ECDNA_QR(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) dst[i * stride] = x[i] + in[i];
}

#ifndef ECDNA_REF_INNER_CALL
#define ECDNA_REF_INNER_CALL 1
#endif
#if ECDNA_REF_INNER_CALL
__device__ __attribute__((noinline)) void chacha8_block_to_lds_call(const uint32_t* key, uint32_t* dst, uint32_t stride,
                                                                    uint64_t counter, uint32_t s_lo, uint32_t s_hi) {
    chacha8_block_to_lds(key, dst, stride, counter, s_lo, s_hi);
}
#endif

// Ring words per lane (a power of two, >= 32): ECDNA_REF_RING. ECDNA_REF_SYNC_TOPUP: when the wave-uniform top-up
// runs a refill for some lane, every lane with room for a block takes one too (the wave issues the refill's
// instructions either way), so later events find fewer lanes short of words.
// (C3 reference-draws line, same box: ring 32 1,898 ms; ring 64 1,883; ring 64 with the synchronized top-up 1,700;
// and the out-of-line inner refill 1,668; profiles/r06c_ab_ref.txt)
#ifndef ECDNA_REF_RING
#define ECDNA_REF_RING 64u
#endif
#ifndef ECDNA_REF_SYNC_TOPUP
#define ECDNA_REF_SYNC_TOPUP 1
#endif
static_assert(ECDNA_REF_RING >= 32u && (ECDNA_REF_RING & (ECDNA_REF_RING - 1u)) == 0u, "ring: a power of two >= 32");
constexpr uint32_t kRingWords = ECDNA_REF_RING;

// The per-lane generator: key (uniform, 8 words from the host's seed_from_u64), 64-bit block counter and
// stream, and a ring of kRingWords / 16 16-word blocks per lane in LDS ([word][lane]: a wave's accesses hit distinct
// banks). Words come out in stream order whatever the refill timing. Lanes consume words at different
// rates, so a refill inside next_u32 would run (masked) for the whole wave at nearly every draw site;
// instead top_up(), called once per event at a wave-uniform point, generates the next block for lanes with
// fewer than 16 words buffered, and next_u32 refills on demand only when a lane's event outruns that (rare
// rejection loops).
struct ChaCha8 {
    const uint32_t* key;   // 8 words
    uint32_t* buf;         // LDS, ring word w (0 .. kRingWords - 1) of this lane at buf[w * stride]
    uint32_t stride;
    uint64_t counter;      // next block
    uint32_t s_lo, s_hi;   // stream
    uint32_t head, tail;   // words read / generated (tail - head = buffered, 0 .. kRingWords)
#ifdef ECDNA_CYCLE_STATS
    // (development counters, ssa_refdraws.hip: refills inside an event, Exp1 retries, BTPE and BINV draws)
    uint32_t dbg[4] = {0u, 0u, 0u, 0u};
#define ECDNA_REF_DBG(rng, i) ((rng).dbg[i] += 1u)
#else
#define ECDNA_REF_DBG(rng, i) ((void)0)
#endif

    __device__ __forceinline__ void reset() {
        counter = 0;
        head = tail = 0;
    }
    __device__ __forceinline__ void refill() {  // one block into ring words tail .. tail + 15 (mod kRingWords)
        chacha8_block_to_lds(key, buf + (tail & (kRingWords - 16u)) * stride, stride, counter, s_lo, s_hi);
        counter += 1;
        tail += 16u;
    }
    // the same from a rare site (an event that outran the top-up): one out-of-line copy of the block function for
    // every such site (ECDNA_REF_INNER_CALL; inlined at each of them, the kernel carried ~23 copies of its ~400
    // instructions)
    __device__ __forceinline__ void refill_rare() {
#if ECDNA_REF_INNER_CALL
        chacha8_block_to_lds_call(key, buf + (tail & (kRingWords - 16u)) * stride, stride, counter, s_lo, s_hi);
        counter += 1;
        tail += 16u;
#else
        refill();
#endif
    }
    __device__ __forceinline__ void top_up() {
#if ECDNA_REF_SYNC_TOPUP
        if (__ballot(tail - head < 16u) != 0ull) {  // (wave-uniform) some lane is short: every lane with room refills
            if (tail - head <= kRingWords - 16u) refill();
        }
#else
        if (tail - head < 16u) refill();
#endif
    }
    __device__ __forceinline__ uint32_t next_u32() {
        if (head == tail) {
            ECDNA_REF_DBG(*this, 0);
            refill_rare();
        }
        return buf[(head++ & (kRingWords - 1u)) * stride];
    }
    __device__ __forceinline__ uint64_t next_u64() {
        const uint32_t lo = next_u32();
        const uint32_t hi = next_u32();
        return ((uint64_t)hi << 32) | lo;
    }
    // rand 0.8.5 Standard for f64: 53 high bits of next_u64, scaled by 2^-53
    __device__ __forceinline__ double gen_f64() { return (double)(next_u64() >> 11) * 0x1p-53; }
    // rand 0.8.5 gen_range(0..n), n >= 1 (UniformInt::sample_single_inclusive over usize)
    __device__ __forceinline__ uint64_t gen_range(uint64_t n) {
        const uint64_t zone = (n << __builtin_clzll(n)) - 1ull;
        for (;;) {
            const uint64_t v = next_u64();
            const uint64_t lo = v * n;
            if (lo <= zone) return __umul64hi(v, n);
        }
    }
};
#undef ECDNA_QR

// rand_distr 0.4.3 Exp1 (ziggurat, rand_distr utils.rs with symmetric = false): x / f tables and the log /
// exp tables in LDS
__device__ __forceinline__ double exp1(ChaCha8& rng, const double* zx, const double* zf, const double* clog,
                                       const double* cexp) {
    for (;;) {
        const uint64_t bits = rng.next_u64();
        const int i = (int)(bits & 0xffu);
        const double u = float_1_2(bits) - (1.0 - 0x1p-53);
        const double x = u * zx[i];
        if (x < zx[i + 1]) return x;
        ECDNA_REF_DBG(rng, 1);
        if (i == 0) return ECDNA_ZIG_EXP_R - log_cr(rng.gen_f64(), clog);
        // (the wedge test against the correctly rounded e^-x, decided by lt_exp_cr's filter; x < R < 22)
        if (lt_exp_cr(zf[i + 1] + (zf[i] - zf[i + 1]) * rng.gen_f64(), -x, cexp)) return x;
    }
}

__device__ __forceinline__ double stirling(double a) {
    const double a2 = a * a;
    return (13860. - (462. - (132. - (99. - 140. / a2) / a2) / a2) / a2) / a / 166320.;
}

// BTPE constants of Binomial(n, 1/2), one row per copy number k = n / 2 (host: ssa_api.cpp btpe_setup, the
// same operations as the oracle's setup): npq, m, p1, x_m, x_l, x_r, c, p2, lambda_l, lambda_r, p3, p4
constexpr int kBtpeRow = 16;  // doubles per row (128 B)
enum { BT_NPQ, BT_M, BT_P1, BT_XM, BT_XL, BT_XR, BT_C, BT_P2, BT_LL, BT_LR, BT_P3, BT_P4, BT_ILL, BT_ILR };

// BINV (the n p < 10 branch of rand_distr 0.4.3 Binomial with p = 1/2: n = 2, 4, ..., 18). The reference's loop
// subtracts r_0 = 2^-n, r_1, r_2, ... from u (r_x = r_{x-1} (a / x - s), a = (n + 1) s, s = p / q = 1) and returns the
// first x with u_x <= r_x. The r_x do not depend on u: binv_cdf forms them by the loop's own IEEE operations, and their
// running sums P_y = r_0 + ... + r_{y-1} (within 20 2^-53 of the real sums), row n / 2 - 1, y = 0 .. 20 (padded past
// n + 1 with the last sum). The loop's u_x is u - P_x up to x roundings (x 2^-53 < 2^-47), so it stops at
// x* = #{y >= 1 : P_y < u} whenever u is clear of P_x* and P_x*+1 by 2^-40 (the earlier sums lie further below u):
// binv_half counts that branch-free and runs the reference's loop itself only otherwise (about 2^-35 of the draws, and
// u past P_n+1, where the loop would run to its restart). Same result, bit for bit, without the serial loop (up to ~15
// dependent steps for the slowest lane of a wave) on the common path.
constexpr int kBinvRows = 9, kBinvCols = 21;
__device__ __forceinline__ void binv_cdf(double* tab, uint32_t tid, uint32_t nthreads) {
    for (uint32_t row = tid; row < (uint32_t)kBinvRows; row += nthreads) {
        const uint32_t n = 2u * (row + 1u);
        const double s = 0.5 / 0.5;
        const double a = (double)(n + 1u) * s;
        double r = __builtin_ldexp(1.0, -(int)n), acc = 0.0;
        tab[row * kBinvCols] = 0.0;
        for (uint32_t y = 1; y < (uint32_t)kBinvCols; ++y) {
            acc += r;                              // P_y
            tab[row * kBinvCols + y] = acc;
            r *= a / (double)y - s;                // r_y (0 from y = n + 1 on)
        }
    }
}

// rand_distr 0.4.3 Binomial::sample for p = 1/2 (n = 2k even, 2 <= n <= 65534): BINV for n p < 10, else BTPE.
__device__ __forceinline__ bool binomial_half_is_binv(uint32_t n) { return (double)n * 0.5 < 10.0; }

// BINV (n p < 10, n <= 18): s = p / q = 1, r0 = q^n = 2^-n exactly. binv: the binv_cdf table.
__device__ __forceinline__ uint32_t binv_half(ChaCha8& rng, uint32_t n, const double* binv) {
    ECDNA_REF_DBG(rng, 3);
    double u = rng.gen_f64();
    {
        const double* const P = binv + (n / 2u - 1u) * kBinvCols;
        uint32_t x = 0;
#pragma unroll
        for (int y = 1; y < kBinvCols - 1; ++y) x += P[y] < u ? 1u : 0u;
        if (x <= n && u - P[x] > 0x1p-40 && P[x + 1u] - u > 0x1p-40) return x;
    }
    // the reference's loop (the draws close to a sum, and past the last one)
    const double s = 0.5 / 0.5;
    const double a = (double)(n + 1u) * s;
    for (;;) {
        double r = __builtin_ldexp(1.0, -(int)n);
        uint32_t x = 0;
        bool restart = false;
        while (u > r) {
            u -= r;
            x += 1;
            if (x > 110u) {
                restart = true;
                break;
            }
            r *= a / (double)x - s;
        }
        if (!restart) return x;
        u = rng.gen_f64();
    }
}

// BTPE (n p >= 10)
__device__ __forceinline__ uint32_t btpe_half(ChaCha8& rng, uint32_t n, const double* btpe, const double* clog) {
    const double p = 0.5, q = 0.5;
    ECDNA_REF_DBG(rng, 2);
    const int64_t SQUEEZE = 20;
    const double* b = btpe + (uint64_t)(n >> 1) * kBtpeRow;
    const double nd = (double)n, npq = b[BT_NPQ], p1 = b[BT_P1], x_m = b[BT_XM], x_l = b[BT_XL], x_r = b[BT_XR];
    const double c = b[BT_C], p2 = b[BT_P2], lambda_l = b[BT_LL], lambda_r = b[BT_LR], p3 = b[BT_P3], p4 = b[BT_P4];
    const double inv_lambda_l = b[BT_ILL], inv_lambda_r = b[BT_ILR];
    const int64_t m = (int64_t)b[BT_M];
    int64_t y;
    for (;;) {
        const double u = (float_1_2(rng.next_u64()) - 1.0) * p4;
        double v = float_1_2(rng.next_u64()) - 1.0;
        if (!(u > p1)) {
            y = f64_to_i64(x_m - p1 * v + u);
            break;
        }
        if (!(u > p2)) {
            const double x = x_l + (u - p1) / c;
            v = v * c + 1.0 - __builtin_fabs(x - x_m) / p1;
            if (v > 1.) continue;
            y = f64_to_i64(x);
        } else if (!(u > p3)) {
            y = trunc_log_ratio(x_l, 1.0, v, lambda_l, inv_lambda_l, clog);  // f64_to_i64(x_l + log_cr(v) / lambda_l)
            if (y < 0) continue;
            v *= (u - p2) * lambda_l;
        } else {
            y = trunc_log_ratio(x_r, -1.0, v, lambda_r, inv_lambda_r, clog);  // f64_to_i64(x_r - log_cr(v) / lambda_r)
            if (y > 0 && (uint64_t)y > (uint64_t)n) continue;
            v *= (u - p3) * lambda_r;
        }
        const int64_t k = y > m ? y - m : m - y;
        if (!(k > SQUEEZE && (double)k < 0.5 * npq - 1.)) {
            const double s = p / q;
            const double a = s * (nd + 1.);
            // (filter) f is the ratio C(n, y) / C(n, m) = prod (n + 1 - i) / i over i in (m, y] (or its inverse for
            // y < m), formed below by one f64 division per factor. For k <= 20 the decision v > f is taken first
            // from that ratio as one quotient of two products of exact integers (within ~2^-47 of the real ratio,
            // as is the loop's f: 3 roundings per factor), wherever v is clear of it by 2^-40 relative; else by
            // the loop's own f. Same decision bit for bit, without ~20 f64 divisions on the common path.
            if (k <= 20) {
                double num = 1.0, den = 1.0;
                for (int64_t i = (m < y ? m : y) + 1; i <= (m < y ? y : m); ++i) {
                    num *= nd + 1. - (double)i;
                    den *= (double)i;
                }
                const double fa = m < y ? num / den : (m > y ? den / num : 1.0);
                if (v > fa * (1.0 + 0x1p-40)) continue;
                if (v < fa * (1.0 - 0x1p-40)) break;
            }
            double f = 1.0;
            if (m < y) {
                int64_t i = m;
                do {
                    i += 1;
                    f *= a / (double)i - s;
                } while (i != y);
            } else if (m > y) {
                int64_t i = y;
                do {
                    i += 1;
                    f /= a / (double)i - s;
                } while (i != m);
            }
            if (v > f) continue;
            break;
        }
        const double kf = (double)k;
        const double rho = (kf / npq) * ((kf * (kf / 3. + 0.625) + 1. / 6.) / npq + 0.5);
        const double t = -0.5 * kf * kf / npq;
        const double alpha = log_cr(v, clog);
        if (alpha < t - rho) break;
        if (alpha > t + rho) continue;
        const double x1 = (double)(y + 1);
        const double f1 = (double)(m + 1);
        const double z = (double)(f64_to_i64(nd) + 1 - m);
        const double w = (double)(f64_to_i64(nd) - y + 1);
        if (alpha > x_m * log_cr(f1 / x1, clog) + (nd - (double)m + 0.5) * log_cr(z / w, clog) +
                        (double)(y - m) * log_cr(w * p / (x1 * q), clog) + stirling(f1) + stirling(z) -
                        stirling(x1) - stirling(w))
            continue;
        break;
    }
    return (uint32_t)y;
}

__device__ __forceinline__ uint32_t binomial_half(ChaCha8& rng, uint32_t n, const double* btpe, const double* clog,
                                                  const double* binv) {
    return binomial_half_is_binv(n) ? binv_half(rng, n, binv) : btpe_half(rng, n, btpe, clog);
}

}  // namespace refdraws
}  // namespace ecdna
