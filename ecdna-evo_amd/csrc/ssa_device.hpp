// ssa_device.hpp — device-side building blocks of the SSA stepper (gfx950).
//
// The draw mapping is the engine's own definition; the CPU
// oracle (oracle/ssa_oracle.c) restates it independently and the parity tests
// require bit-identical results. Every f32 / f64 operation here is a correctly
// rounded IEEE add/sub/mul/div/fma in a fixed order; the file is compiled with
// -ffp-contract=off and additionally pins contraction off below, so no FMA
// fusion can change a rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ssa_logtab.h"

#pragma clang fp contract(off)

namespace ecdna {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;

// Philox4x32-10. The key is wave-uniform (the run's seed), so the key schedule lives in SGPRs;
// each round is two 32x32->64 multiplies (v_mad_u64_u32) and four XORs per lane (gfx9 has no v_xor3).
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += kPhiloxW0;
            k1 += kPhiloxW1;
        }
        // keep the round keys a per-call chain of scalar adds: hoisted out of the event loop they
        // are 18 loop-invariant SGPRs, which spill to VGPR lanes (v_readlane in every event)
        asm volatile("" : "+s"(k0), "+s"(k1));
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c.x;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * c.z;
        c = make_uint4((uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
                       (uint32_t)p0);
    }
    return c;
}

// Philox4x32-10 with the 20 round keys precomputed per lane in VGPRs (philox_round_keys): no key
// schedule on the SALU and no SALU-write -> VALU-read hazard waits inside the rounds. Same function.
struct PhiloxKeys {
    uint32_t k0[10], k1[10];
};

__device__ __forceinline__ PhiloxKeys philox_round_keys(uint32_t k0, uint32_t k1) {
    PhiloxKeys r;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        uint32_t a = k0 + (uint32_t)i * kPhiloxW0, b = k1 + (uint32_t)i * kPhiloxW1;
        asm volatile("v_mov_b32 %0, %1" : "=v"(r.k0[i]) : "s"(a));  // pin to VGPRs
        asm volatile("v_mov_b32 %0, %1" : "=v"(r.k1[i]) : "s"(b));
    }
    return r;
}

// a ^ b ^ c as one gfx950 v_bitop3_b32 (truth table 0x96) instead of two v_xor_b32. B3: the compiler builtin, whose
// hazards the compiler sees (an inline asm block is opaque: each is followed by a conservative s_nop before the next
// v_mad_u64_u32, and the scheduler works around it). Same instruction, same result; only the schedule differs: the
// builtin is faster where waves drain or run alone (C4 shard -4 %, C5 shard -2 %) and 1 % slower on the issue-bound
// C3 kernel (profiles/r05zb_bitop3_ab.txt), so the bin stepper picks it per instance (kB3).
template <bool B3 = false>
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    if (B3) return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

template <bool B3 = false>
__device__ __forceinline__ uint4 philox4x32_10(uint4 c, const PhiloxKeys& rk) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)kPhiloxM0 * c.x;
        const uint64_t p1 = (uint64_t)kPhiloxM1 * c.z;
        c = make_uint4(xor3<B3>((uint32_t)(p1 >> 32), c.y, rk.k0[r]), (uint32_t)p1,
                       xor3<B3>((uint32_t)(p0 >> 32), c.w, rk.k1[r]), (uint32_t)p0);
    }
    return c;
}

// The bin store's event block is Philox((e, 0, rid_lo, rid_hi)): round 0's c.z product and the words it is XORed with
// depend only on the replicate, and so do round 1's c.x product (c.x = round 0's output 0) and the key words XORed into
// round 1's outputs 0 and 2. They are formed once per replicate; an event's round 1 is then one product and three
// two-input XORs (the e-dependent part), against two products and two three-input XORs. Same function.
struct PhiloxEventPre {
    uint32_t x1k;  // round-0 output 1 ^ k0[1]
    uint32_t x2;   // rid_hi ^ k1[0] (round-0 output 2 is hi(M0 e) ^ x2)
    uint32_t y2k;  // hi(M0 * round-0 output 0) ^ k1[1]
    uint32_t y3;   // lo(M0 * round-0 output 0): round-1 output 3
};

__device__ __forceinline__ PhiloxEventPre philox_event_pre(uint32_t rid_lo, uint32_t rid_hi, const PhiloxKeys& rk) {
    const uint64_t p1 = (uint64_t)kPhiloxM1 * rid_lo;
    const uint32_t x0 = (uint32_t)(p1 >> 32) ^ rk.k0[0];  // round-0 output 0 (c.y = 0)
    const uint64_t q0 = (uint64_t)kPhiloxM0 * x0;          // round 1's c.x product
    PhiloxEventPre p;
    p.x1k = (uint32_t)p1 ^ rk.k0[1];
    p.x2 = rid_hi ^ rk.k1[0];
    p.y2k = (uint32_t)(q0 >> 32) ^ rk.k1[1];
    p.y3 = (uint32_t)q0;
    return p;
}

// == philox4x32_10(make_uint4(e, 0, rid_lo, rid_hi), rk) for the pre formed from (rid_lo, rid_hi)
template <bool B3 = false>
__device__ __forceinline__ uint4 philox_event(uint32_t e, const PhiloxEventPre& pre, const PhiloxKeys& rk) {
    const uint64_t p0 = (uint64_t)kPhiloxM0 * e;                        // round 0's c.x product
    const uint64_t q1 = (uint64_t)kPhiloxM1 * ((uint32_t)(p0 >> 32) ^ pre.x2);  // round 1's c.z product
    uint4 c = make_uint4((uint32_t)(q1 >> 32) ^ pre.x1k, (uint32_t)q1, pre.y2k ^ (uint32_t)p0, pre.y3);
#pragma unroll
    for (int r = 2; r < 10; ++r) {
        const uint64_t q0 = (uint64_t)kPhiloxM0 * c.x;
        const uint64_t q1r = (uint64_t)kPhiloxM1 * c.z;
        c = make_uint4(xor3<B3>((uint32_t)(q1r >> 32), c.y, rk.k0[r]), (uint32_t)q1r,
                       xor3<B3>((uint32_t)(q0 >> 32), c.w, rk.k1[r]), (uint32_t)q0);
    }
    return c;
}

// -ln u for u = ((w >> 9) + 0.5) 2^-23, draw mapping v6, in f32: d = (w >> 8) | 1 is odd and below
// 2^24, so (float)d is exact, = m 2^ex with m in [0.5, 1) and u = d 2^-24; the top 7 fraction bits j of m pick
// {C, LN} = {RN32(1/mid_j), RN32(-ln C)} (ssa_logtab.h, staged in LDS; LN is the log of the stored C, so ln m =
// ln(m C) + LN exactly whatever C's rounding; entry 127 = {1, 0}, so u -> 1 keeps its relative accuracy);
// r = fma(m, C, -1) (|r| <= 2^-8); ln(1 + r) by a degree-4 series in explicit fmas (truncation |r|^5 / 5 <= 2^-42);
// -ln u = -(LN + ln(1 + r) + k ln 2), k = ex - 24 in [-23, 0], with ln 2 as an exact head (k LN2_HI is exact) and a
// tail. oracle_softlog_neg (oracle/ssa_oracle.c) performs the same IEEE f32 operations in the same order, so CPU
// and GPU agree bit for bit. (v2-v5 formed the same function in f64 from all 32 bits of w: MI355X issues f64
// arithmetic at half the f32 rate, and the stepper is issue-bound.)
struct SoftlogParts {
    float2 cl;
    float m;
    int k;
};

// the table load (begin) and the arithmetic after it (end), so that a loop can issue the load one iteration ahead
__device__ __forceinline__ SoftlogParts softlog_begin(uint32_t w, const float2* tab) {
    const uint32_t bits = __float_as_uint((float)((w >> 8) | 1u));  // exact
    SoftlogParts p;
    p.k = (int)(bits >> 23) - 150;                                 // ex - 24, ex = biased exponent - 126
    p.m = __uint_as_float((bits & 0x007fffffu) | 0x3f000000u);      // m in [0.5, 1)
    p.cl = tab[(bits >> 16) & 127u];
    return p;
}

__device__ __forceinline__ float softlog_end(const SoftlogParts& p) {
    const float r = fmaf(p.m, p.cl.x, -1.0f);
    float q = fmaf(r, -0.25f, 0x1.555556p-2f);  // -1/4, RN32(1/3)
    q = fmaf(r, q, -0.5f);
    const float l = fmaf(r * r, q, r);  // ln(1 + r)
    const float kf = (float)p.k;
    return -fmaf(kf, ECDNA_LN2_HI, fmaf(kf, ECDNA_LN2_LO, p.cl.y + l));
}

__device__ __forceinline__ float softlog_neg(uint32_t w, const float2* tab) { return softlog_end(softlog_begin(w, tab)); }

// The channel's target, draw mapping v7: u = (w + 0.5) 2^-32 from all 32 bits of w1, exact in f64 (one
// fma: w + 0.5 has 33 significant bits), times the f64 total propensity A (RN64). u <= 1 - 2^-33, so the target stays
// below A and a last channel of zero propensity is never drawn; u >= 2^-33 and A >= 2^-60 keep it above 0, so a first
// channel of zero propensity is never drawn either. (v6 took 23 bits of w1 and f32 cumulative sums: a channel below
// ~2^-24 of the total could not fire)
//
// Formed as ((w + 0.5) A) 2^-32: one conversion, one add of the inline constant 0.5 and two multiplies (the second by
// a power of two, exact: the product stays far above the f64 underflow), no f64 constant to materialise in registers;
// RN((w + 0.5) A) 2^-32 = RN((w + 0.5) 2^-32 A), the oracle's u A, bit for bit. (Host-callable: the CPU tests check it
// against the oracle's channel function, tests/native/device_math_check.cpp.)
__host__ __device__ __forceinline__ double chan_target(uint32_t w, double a) { return ((double)w + 0.5) * a * 0x1p-32; }

// RN32(1 / d) from the hardware reciprocal and one Newton step: y = fma(fma(-d, r, 1), r, r), r = v_rcp_f32(d). For
// every f32 d of the stepper's divisors (total propensities in [2^-60, 2^94]: every rate 0 or in [2^-60, 2^60], which
// ecdna_ssa_ctx_create requires, u32 populations; reference-draws rates, the same range) y is the correctly rounded
// reciprocal: checked on the GPU for all 1.3e9 f32 values in [2^-60, 2^95) (tools/rcp_check.hip, tests/test_gpu_rcp.py:
// no mismatch). On the CPU (tests/native/device_math_check.cpp) the step from either faithful r (RD or RU of 1 / d)
// gives RN(1 / d) for every d of a binade but one mantissa, 0x7fffff from RD (1 / d within 2^-49 of a midpoint), where
// the hardware's r is RU. Draw mapping v8: the time step is RN32(softlog * RN32(1 / a0)), a product with
// the correctly rounded reciprocal (v7 divided: the correctly rounded quotient took two more residual corrections, four
// more instructions per event; the product differs from the quotient by at most one ulp). rcp_newton is the step from
// a given r (host-callable: the CPU check feeds it RD and RU).
__host__ __device__ __forceinline__ float rcp_newton(float d, float r) { return fmaf(fmaf(-d, r, 1.0f), r, r); }

__device__ __forceinline__ float rcp_rn(float d) { return rcp_newton(d, __builtin_amdgcn_rcpf(d)); }

// x << (s & 31) as one v_lshlrev_b32, which reads only the low five bits of its amount (C++ leaves a shift by
// 32 or more undefined, so the compiler would keep an explicit mask)
__device__ __forceinline__ uint32_t shl_lo5(uint32_t x, uint32_t s) {
    uint32_t r;
    asm("v_lshlrev_b32 %0, %1, %2" : "=v"(r) : "v"(s), "v"(x));
    return r;
}

// (x & m) | y and (x << s) | y as one VALU each (the compiler splits them when it merges neighbouring ORs)
__device__ __forceinline__ uint32_t and_or(uint32_t x, uint32_t m, uint32_t y) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "i"(m), "v"(y));
    return r;
}
__device__ __forceinline__ uint32_t lshl_or(uint32_t x, uint32_t s, uint32_t y) {
    uint32_t r;
    asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "i"(s), "v"(y));
    return r;
}

// 32 x 32 -> 64-bit product as one v_mad_u64_u32 (the compiler widens a u32 * u64 into two)
__device__ __forceinline__ uint64_t mul_u32_wide(uint32_t a, uint32_t b) {
    uint64_t d, carry;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(d), "=s"(carry) : "v"(a), "v"(b));
    return d;
}

// The log table in constant memory; each workgroup stages it into LDS (divergent per-lane index).
__constant__ const float kLogTab[2 * ECDNA_LOGTAB_N] = ECDNA_LOGTAB_INIT;

__device__ __forceinline__ void stage_logtab(float2* lds) {
    for (uint32_t i = threadIdx.x; i < ECDNA_LOGTAB_N; i += blockDim.x)
        lds[i] = make_float2(kLogTab[2 * i], kLogTab[2 * i + 1]);
    __syncthreads();
}

// Stream words of one event (draw mapping v5): [w2, w3, spare0 .. spare(nsp-1), blk1.x,
// blk1.y, blk1.z, blk1.w, blk2.x, ...], blk j = Philox(e, j, rid). The spares are words of earlier events'
// blocks that no draw used, a two-slot stack (newest first). Only the rare paths (Lemire rejection, copy
// numbers beyond what w3 and the spares cover, NoUneven redraws) reach the Philox blocks.
// pos = words consumed so far; w2 counts as consumed by the cell pick (pos starts at 1).
struct WordStream {
    uint32_t w2, w3;
    uint32_t s0, s1, nsp;
    uint32_t e, rid_lo, rid_hi, k0, k1;
    uint32_t pos;
    uint32_t blk_id;
    uint4 blk;

    // value selects (not member-address selects, which would demote the stream to memory)
    static __device__ __forceinline__ uint32_t sel(bool c, uint32_t a, uint32_t b) {
        return b ^ ((a ^ b) & (0u - (uint32_t)c));
    }

    __device__ __forceinline__ uint32_t next() {
        const uint32_t p = pos++;
        if (p < 2) return sel(p == 0, w2, w3);
        if (p - 2 < nsp) return sel(p == 2, s0, s1);
        const uint32_t q = p - 2 - nsp;
        const uint32_t j = (q >> 2) + 1;
        if (j != blk_id) {
            blk = philox4x32_10(make_uint4(e, j, rid_lo, rid_hi), k0, k1);
            blk_id = j;
        }
        const bool odd = (q & 1u) != 0;
        return sel((q & 2u) != 0, sel(odd, blk.w, blk.z), sel(odd, blk.y, blk.x));
    }

    // the low `take` bits (0 <= take <= 32)
    static __device__ __forceinline__ uint32_t low_bits(uint32_t take) { return (uint32_t)((1ull << take) - 1ull); }

    // popcount of the next n stream bits (n >= 1): k1 ~ Binomial(n, 1/2) exactly. The same words in the
    // same order as ceil(n / 32) calls of next() (the low bits of the last one), but past the base words
    // and spares the Philox blocks come from a lane-uniform loop, one block per iteration with its four
    // words popcounted branch-free. (Word by word, next() generates a block whenever ANY lane of the
    // wave crosses a block boundary, and lanes sit at different stream offsets: large copy numbers then
    // ran a Philox block for almost every word.) block(c): Philox4x32-10 of counter c under the run's key.
    // kReuse: keep a block already in `blk` (the stepper's K = 64 / u32 max-ILP instances form block 1 ahead);
    // elsewhere every block is formed here, as before (no compare on their path)
    template <bool kReuse, class Block>
    __device__ __forceinline__ uint32_t binomial_half_with(uint32_t n, const Block& block) {
        uint32_t c = 0;
        while (n && pos < 2u + nsp) {  // w3 and the spares (at most three words; no Philox block here)
            const uint32_t p = pos++;
            const uint32_t w = p < 2u ? sel(p == 0u, w2, w3) : sel(p == 2u, s0, s1);
            const uint32_t take = min(n, 32u);
            c += __popc(w & low_bits(take));
            n -= take;
        }
        while (n) {
            const uint32_t q = pos - 2u - nsp;  // stream offset inside the block region
            const uint32_t j = (q >> 2) + 1u;
            if (!kReuse || j != blk_id) {  // (kReuse: block 1 formed ahead, or this block by the Lemire loop)
                blk = block(make_uint4(e, j, rid_lo, rid_hi));
                blk_id = j;
            }
            const uint32_t t0 = q & 3u;
            const uint32_t w[4] = {blk.x, blk.y, blk.z, blk.w};
#pragma unroll
            for (uint32_t t = 0; t < 4u; ++t) {
                const uint32_t take = t >= t0 ? min(n, 32u) : 0u;
                c += __popc(w[t] & low_bits(take));
                n -= take;
                pos += take ? 1u : 0u;
            }
        }
        return c;
    }

    // The no-uneven rule's redraws for 2 <= n <= 32 (SEG_BINOMIAL_NO_UNEVEN: resample k1 while it is 0 or n,
    // src/segregation.rs:157-174), after `tries` rejected draws: the same words in the same order as repeated
    // binomial_half(n) calls (one word per try), but the accepted word is found branch-free over the base
    // words and then four words at a time over Philox blocks, one block per iteration of a lane loop (a word
    // is rejected with probability 2^(1-n) <= 1/2: word by word the wave looped once per try of its unluckiest
    // lane, each try a full binomial_half). `fail`: max_tries draws, all uneven (ECDNA_REP_ERR_REJECTION).
    template <class Block>
    __device__ __forceinline__ uint32_t redraw_even_small_with(uint32_t n, uint32_t tries, uint32_t max_tries,
                                                               bool& fail, const Block& block) {
        const uint32_t m = low_bits(n);
        uint32_t res = 0;
        bool found = false;
        const auto try_word = [&](uint32_t w, bool take) {
            const uint32_t c = __popc(w & m);
            const bool acc = take && c != 0u && c != n;
            res = acc ? c : res;
            found = found || acc;
            tries += take ? 1u : 0u;
        };
#pragma unroll
        for (uint32_t p = 1; p < 4u; ++p) {  // w3 (position 1) and the spares (2, 3)
            const bool take = !found && p >= pos && p < 2u + nsp && tries < max_tries;
            try_word(p == 1u ? w3 : sel(p == 2u, s0, s1), take);
            pos = take ? p + 1u : pos;
        }
        while (!found && tries < max_tries) {
            const uint32_t q = pos - 2u - nsp;
            const uint32_t j = (q >> 2) + 1u;
            blk = block(make_uint4(e, j, rid_lo, rid_hi));
            blk_id = j;
            const uint32_t t0 = q & 3u;
            const uint32_t w[4] = {blk.x, blk.y, blk.z, blk.w};
#pragma unroll
            for (uint32_t t = 0; t < 4u; ++t) {
                const bool take = !found && t >= t0 && tries < max_tries;
                try_word(w[t], take);
                pos += take ? 1u : 0u;
            }
        }
        fail = !found;
        return res;
    }

    __device__ __forceinline__ uint32_t redraw_even_small(uint32_t n, uint32_t tries, uint32_t max_tries, bool& fail) {
        return redraw_even_small_with(n, tries, max_tries, fail, [&](uint4 c4) { return philox4x32_10(c4, k0, k1); });
    }

    template <bool B3 = false>
    __device__ __forceinline__ uint32_t redraw_even_small(uint32_t n, uint32_t tries, uint32_t max_tries, bool& fail,
                                                          const PhiloxKeys& rk) {
        return redraw_even_small_with(n, tries, max_tries, fail, [&](uint4 c4) { return philox4x32_10<B3>(c4, rk); });
    }

    // with the key schedule formed per block (k0, k1)
    __device__ __forceinline__ uint32_t binomial_half(uint32_t n) {
        return binomial_half_with<false>(n, [&](uint4 c4) { return philox4x32_10(c4, k0, k1); });
    }

    // with the kernel's VGPR round keys. (A reference, never a nullable pointer: a null test of the keys'
    // private-memory address does not fold on AMDGPU, where private null is not address 0, and the test alone
    // kept the 20 keys in scratch, reloaded at every Philox round of every kernel that had it.)
    template <bool kReuse = false, bool B3 = false>
    __device__ __forceinline__ uint32_t binomial_half(uint32_t n, const PhiloxKeys& rk) {
        return binomial_half_with<kReuse>(n, [&](uint4 c4) { return philox4x32_10<B3>(c4, rk); });
    }
};

// The spare stack after an event that consumed `used` stream words (0 when no cell was picked), draw mapping
// v5: the unused base words are pushed, newest on top (the oldest falls off the two slots): w2 then w3 when
// used == 0, w3 when used == 1; used == 2 leaves the stack; used >= 3 consumed used - 2 words after w3, the
// top spares first. Branch-free selects (v3 kept the oldest two in list order: ~15 more VALU per event; v4's
// single spare sent 3.5x more events to a second Philox block, a net loss at C3).
__device__ __forceinline__ void spares_update(uint32_t used, uint32_t w2, uint32_t w3, uint32_t& s0, uint32_t& s1,
                                              uint32_t& nsp) {
    const bool u0 = used == 0u, le1 = used <= 1u, pop = used >= 3u;  // (three compares: u1 = le1 & !u0)
    const uint32_t n1 = s1, n0 = s0;
    s1 = u0 ? w2 : (le1 ? n0 : n1);
    s0 = le1 ? w3 : (pop ? n1 : n0);
    // 2 pushes (used 0), 1 push (used 1), none (used 2), used - 2 pops: min(max(nsp + 2 - used, 0), 2)
    const uint32_t grown = nsp + 2u;
    nsp = min(grown > used ? grown - used : 0u, 2u);
}

}  // namespace ecdna
