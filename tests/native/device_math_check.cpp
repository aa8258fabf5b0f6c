// TEST INFRASTRUCTURE ONLY — host-side check of the stepper header's host-callable draw-mapping pieces
// (ecdna-evo_amd/csrc/ssa_device.hpp) against the CPU oracle's channel function (oracle/ssa_oracle.c:136,
// oracle_channel), built with hipcc and run on the CPU by tests/test_mapping_v7.py.
//
// The propensity / cumulative-sum sequence below is the one the steppers inline (ssa_kernels.hip, ssa_stepper
// "propensities" block): f32 products rate * f32(pop), f64 cumulative sums, then chan_target(w1, A) against the
// boundaries. chan_target itself is the header's function, so a change of its scale or rounding that the oracle
// does not share shows here, without a GPU.
// Then the time step's reciprocal (draw mapping v8): rcp_newton(d, r), the Newton step rcp_rn applies to the hardware's
// v_rcp_f32, from both faithful starts r (RD and RU of 1 / d) against RN32(1 / d), for every d in [1, 2) and for
// random d over [2^-60, 2^95): the step is exact from either start except from RD at mantissa 0x7fffff (1 / d within
// 2^-49 of a rounding midpoint), where the GPU's rcp gives RU (tools/rcp_check.hip checks every d on the GPU).
// Prints "rcp_cases=<n> rcp_off=<k>" and "cases=<n> mismatches=<m>"; exits 1 on any mismatch.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "ssa_device.hpp"

extern "C" int oracle_channel(const float rates[4], uint64_t nminus, uint64_t nplus, int birth_death, uint32_t w1);

namespace {

uint64_t g_state = 0x9E3779B97F4A7C15ull;
uint64_t next_u64() {  // splitmix64
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

float rand_rate() {  // 0 or log-uniform in [2^-60, 2^60], the range ecdna_ssa_ctx_create accepts
    const uint64_t r = next_u64();
    if ((r & 7u) == 0u) return 0.0f;
    const double ex = -60.0 + 120.0 * (double)(r >> 11) * 0x1p-53;
    return (float)exp2(ex);
}

uint32_t rand_pop() {
    const uint64_t r = next_u64();
    switch (r & 3u) {
        case 0: return 0u;
        case 1: return (uint32_t)((r >> 8) & 15u);
        case 2: return (uint32_t)((r >> 8) & 0xFFFFu);
        default: return (uint32_t)(r >> 32);
    }
}

int kernel_channel(const float r[4], uint32_t nm, uint32_t np, bool bd, uint32_t w1) {
    const float fnm = (float)nm, fnp = (float)np;
    const double cA = (double)(r[0] * fnm);
    const double cB = cA + (double)(r[1] * fnp);
    double cC = cB, A = cB;
    if (bd) {
        cC = cB + (double)(r[2] * fnm);
        A = cC + (double)(r[3] * fnp);
    }
    if (!((float)A > 0.0f)) return -1;
    const double target = ecdna::chan_target(w1, A);
    if (bd) return target < cA ? 0 : (target < cB ? 1 : (target < cC ? 2 : 3));
    return target < cA ? 0 : 1;
}

// RN32(1 / d): the f64 quotient rounded to f32 (1 / d is never within 2^-53 relative of an f32 rounding boundary)
float rn_recip(float d) { return (float)(1.0 / (double)d); }

// (cases, mismatches other than the known one) of rcp_newton from RD and RU of 1 / d
void check_recip(float d, long& cases, long& bad, long& known) {
    const double inv = 1.0 / (double)d;
    const float yt = (float)inv;
    const float rd = (double)yt <= inv ? yt : nextafterf(yt, 0.0f);
    const float ru = (double)yt >= inv ? yt : nextafterf(yt, INFINITY);
    for (const float r : {rd, ru}) {
        ++cases;
        if (ecdna::rcp_newton(d, r) == yt) continue;
        uint32_t u;
        memcpy(&u, &d, 4);
        if ((u & 0x7fffffu) == 0x7fffffu && r == rd) {
            ++known;
            continue;
        }
        if (++bad <= 5) fprintf(stderr, "rcp mismatch: d %a r %a -> %a, RN %a\n", d, r, ecdna::rcp_newton(d, r), yt);
    }
}

}  // namespace

int main() {
    long rc = 0, rbad = 0, rknown = 0;
    for (uint32_t m = 0; m < (1u << 23); ++m) {
        float d;
        const uint32_t u = 0x3f800000u | m;
        memcpy(&d, &u, 4);
        check_recip(d, rc, rbad, rknown);
    }
    for (int i = 0; i < 2000000; ++i) {  // other binades: [2^-60, 2^95)
        const uint64_t r = next_u64();
        const uint32_t u = ((uint32_t)(67u + (r >> 32) % 155u) << 23) | (uint32_t)(r & 0x7fffffu);
        float d;
        memcpy(&d, &u, 4);
        check_recip(d, rc, rbad, rknown);
    }
    printf("rcp_cases=%ld rcp_off=%ld rcp_known=%ld\n", rc, rbad, rknown);
    long cases = 0, bad = 0;
    for (int i = 0; i < 200000; ++i) {
        const float r[4] = {rand_rate(), rand_rate(), rand_rate(), rand_rate()};
        const uint32_t nm = rand_pop(), np = rand_pop();
        const bool bd = (i & 1) != 0;
        // w1: random, the extremes, and the words either side of each boundary
        uint32_t ws[12];
        int nw = 0;
        ws[nw++] = (uint32_t)next_u64();
        ws[nw++] = 0u;
        ws[nw++] = 0xFFFFFFFFu;
        const float fnm = (float)nm, fnp = (float)np;
        const double c0 = (double)(r[0] * fnm), c1 = c0 + (double)(r[1] * fnp);
        const double c2 = c1 + (bd ? (double)(r[2] * fnm) : 0.0);
        const double A = c2 + (bd ? (double)(r[3] * fnp) : 0.0);
        if (A > 0.0) {
            for (double c : {c0, c1, c2}) {
                const double w = floor(c / A * 0x1p32 - 0.5);
                for (int d = -1; d <= 1; ++d) {
                    const double x = w + d;
                    if (x >= 0.0 && x <= 4294967295.0 && nw < 12) ws[nw++] = (uint32_t)x;
                }
            }
        }
        for (int k = 0; k < nw; ++k) {
            const int want = oracle_channel(r, nm, np, bd ? 1 : 0, ws[k]);
            const int got = kernel_channel(r, nm, np, bd, ws[k]);
            ++cases;
            if (want != got) {
                if (++bad <= 5)
                    fprintf(stderr, "mismatch: rates %a %a %a %a nm %u np %u bd %d w1 %u: oracle %d header %d\n",
                            r[0], r[1], r[2], r[3], nm, np, bd ? 1 : 0, ws[k], want, got);
            }
        }
    }
    printf("cases=%ld mismatches=%ld\n", cases, bad + rbad);
    return (bad || rbad) ? 1 : 0;
}
