// ssa_device.hpp — device-side building blocks of the SSA stepper (gfx950).
//
// The draw mapping is the engine's own definition; the CPU
// oracle (oracle/ssa_oracle.c) restates it independently and the parity tests
// require bit-identical results. Every f64 operation here is a correctly
// rounded IEEE add/sub/mul/div in a fixed order; the file is compiled with
// -ffp-contract=off and additionally pins contraction off below, so no FMA
// fusion can change a rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace ecdna {

constexpr uint32_t kPhiloxM0 = 0xD2511F53u;
constexpr uint32_t kPhiloxM1 = 0xCD9E8D57u;
constexpr uint32_t kPhiloxW0 = 0x9E3779B9u;
constexpr uint32_t kPhiloxW1 = 0xBB67AE85u;

// Philox4x32-10. The key is wave-uniform (the run's seed), so the key schedule lives in SGPRs;
// each round is two 32x32->64 multiplies and four XORs per lane.
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

// -ln((w + 0.5) 2^-32): same operations, same order as oracle_softlog_neg (oracle/ssa_oracle.c).
__device__ __forceinline__ double softlog_neg(uint32_t w) {
    const uint64_t m = 2ull * (uint64_t)w + 1ull;
    int ex = 63 - __clzll((long long)m);
    const double d = (double)m;
    const double scale = __longlong_as_double((long long)((uint64_t)(1023 - ex) << 52));
    double f = d * scale;
    if (f > 0x1.6a09e667f3bcdp+0) {
        f = f * 0.5;
        ex += 1;
    }
    const double s = (f - 1.0) / (f + 1.0);
    const double z = s * s;
    double r = 0x1.af286bca1af28p-5;
    r = r * z + 0x1.e1e1e1e1e1e1ep-5;
    r = r * z + 0x1.1111111111111p-4;
    r = r * z + 0x1.3b13b13b13b14p-4;
    r = r * z + 0x1.745d1745d1746p-4;
    r = r * z + 0x1.c71c71c71c71cp-4;
    r = r * z + 0x1.2492492492492p-3;
    r = r * z + 0x1.999999999999ap-3;
    r = r * z + 0x1.5555555555555p-2;
    const double s2 = s + s;
    const double lnf = s2 + (s2 * z) * r;
    return (double)(33 - ex) * 0x1.62e42fefa39efp-1 - lnf;
}

// Extra words of one event: [w2, w3, blk1.x..w, blk2.x..w, ...], blk j = Philox(e, j, rid).
// Only the rare paths (Lemire rejection, copy numbers > 16, NoUneven redraws) go past w3.
struct WordStream {
    uint32_t w2, w3;
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
        const uint32_t q = p - 2;
        const uint32_t j = (q >> 2) + 1;
        if (j != blk_id) {
            blk = philox4x32_10(make_uint4(e, j, rid_lo, rid_hi), k0, k1);
            blk_id = j;
        }
        const bool odd = (q & 1u) != 0;
        return sel((q & 2u) != 0, sel(odd, blk.w, blk.z), sel(odd, blk.y, blk.x));
    }

    // popcount of the next n stream bits (n >= 1): k1 ~ Binomial(n, 1/2) exactly.
    __device__ __forceinline__ uint32_t binomial_half(uint32_t n) {
        uint32_t c = 0;
        while (n >= 32) {
            c += __popc(next());
            n -= 32;
        }
        if (n) c += __popc(next() & ((1u << n) - 1u));
        return c;
    }
};

}  // namespace ecdna
