// ssa_refdraws.hip — the SSA stepper under the reference's own draw structure (ECDNA_FLAG_REFERENCE_DRAWS;
// DESIGN.md §4.1): a correctness path that reproduces, per replicate, the sequence of random draws the Rust
// reference makes, so a GPU run can be compared seed for seed with the reference semantics
// (oracle/ssa_compat.c restates the same on the CPU and the parity tests require bit-identical results).
//
// One replicate per lane, cells in a u16 row in HBM in swap_remove order (the row store; the bin store's
// canonical order is a different arrangement, so it has no seed-for-seed counterpart in the reference). Per
// event, in the reference's order:
//   * sosa 3.0.3 loop (call sites src/main.rs:92-99, 166-173; reconstructed): stop checks
//     (iterations, cells, f32 time), then the FIRST-REACTION method over update_state's population vector
//     [n-, n+(, n-, n+)] (src/process.rs:187-196, 339-344) with f32 rates (src/main.rs:67, 139): channel i
//     draws tau_i = Exp(rate_i * pop_i) unless its propensity is 0 (no draw), the first minimum wins;
//   * advance_step (src/process.rs:147-184, 291-336): ProliferateNPlus picks a uniform N+ cell with
//     gen_range + swap_remove (ecdna-lib), segregates 2k copies with rand_distr's Binomial(2k, 1/2) under the
//     CLI's Segregation rule (src/segregation.rs:110-194) and pushes the daughters
//     (src/proliferation.rs:25-111); DeathNPlus removes a uniform cell (src/proliferation.rs:125-133); the N-
//     events count (src/proliferation.rs:113-117, 135-139);
//   * process.time += tau in f32 (src/process.rs:184, 336).
// RNG: ChaCha8Rng::seed_from_u64(seed) on stream seed * 10 + r (src/main.rs:56-58), refdraws.hpp.
#include "refdraws.hpp"
#include "ssa_device.hpp"
#include "ssa_launch.h"

#pragma clang fp contract(off)

namespace ecdna {

namespace {
__constant__ const double kZigX[257] = ECDNA_ZIG_EXP_X_INIT;
__constant__ const double kZigF[257] = ECDNA_ZIG_EXP_F_INIT;
__constant__ const double kCLog[3 * ECDNA_CLOG_N] = ECDNA_CLOG_INIT;
__constant__ const double kCExp[128] = ECDNA_CEXP_INIT;
constexpr uint64_t kFnv0 = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvP = 0x100000001b3ull;
constexpr uint32_t kRefBlock = 256;
}  // namespace

#ifndef ECDNA_REF_MIN_WAVES
#define ECDNA_REF_MIN_WAVES 1
#endif

// Development cycle counters of the reference-draws stepper (built with -DECDNA_CYCLE_STATS only;
// tools/cycle_stats_ref.py), per wave, summed over waves: shader-clock cycles in [0] the replicate boundary (finish +
// claim), [1] the per-event ChaCha8 top-up, [2] the stop checks and the first-reaction draws (Exp1 per positive
// channel), [3] the cell pick (gen_range + row read; ProliferateNPlus only), [4] the segregation (BTPE under the Binomial
// rules; all of it under the others), [6] BINV (the Binomial rules), [5] the rest of the event (other channels' updates, the row update, the commit); counts, summed over lanes: [8] lane
// loop iterations, [10] lane refills in the top-up, [11] lane refills inside an event (next_u32 on an empty ring), [12]
// Exp1 loop trips beyond the first, [13] binomial draws by BTPE, [14] by BINV; [9] wave-iterations (per wave); [15]
// whole-kernel cycles (per wave). The cycle attribution is per WAVE: a mark, executed by the wave whenever any lane is
// active (also inside divergent branches), charges the time since the wave's previous mark to its region, through a
// per-wave clock in LDS that the wave's first active lane keeps (a mark waits for the wave's LDS operations: a rough
// attribution of latency, an exact one of the wave's serial time).
#ifdef ECDNA_CYCLE_STATS
__device__ unsigned long long g_cycle_stats_ref[16];
#define RCYC_DECL                                                                                              \
    __shared__ unsigned long long rcyc_w_[kRefBlock / 64][8];                                                 \
    unsigned long long rcy_[16] = {};                                                                         \
    const unsigned long long rcy_start_ = clock64();                                                          \
    const uint32_t rcy_wave_ = threadIdx.x >> 6;                                                              \
    if ((threadIdx.x & 63u) == 0u) {                                                                          \
        for (int q = 0; q < 7; ++q) rcyc_w_[rcy_wave_][q] = 0ull;                                             \
        rcyc_w_[rcy_wave_][7] = rcy_start_;                                                                   \
    }
#define RCYC_MARK(i)                                                                                           \
    do {                                                                                                       \
        const unsigned long long n_ = clock64();                                                               \
        const uint32_t l_ = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));                \
        if (l_ == (uint32_t)__builtin_amdgcn_readfirstlane(l_)) {                                             \
            rcyc_w_[rcy_wave_][i] += n_ - rcyc_w_[rcy_wave_][7];                                              \
            rcyc_w_[rcy_wave_][7] = n_;                                                                       \
        }                                                                                                      \
    } while (0)
#define RCYC_ADD(i, v) (rcy_[i] += (unsigned long long)(v))
#define RCYC_FLUSH()                                                                                           \
    do {                                                                                                       \
        __builtin_amdgcn_s_waitcnt(0xc07f);                                                                    \
        for (int q = 0; q < 4; ++q) rcy_[11 + q] = rng.dbg[q];                                                 \
        for (int q = 8; q < 15; ++q) rcy_[q] = wave_sum_u64(rcy_[q]);                                          \
        if ((threadIdx.x & 63u) == 0u) {                                                                       \
            for (int q = 0; q < 7; ++q) rcy_[q] = rcyc_w_[rcy_wave_][q];                                       \
            rcy_[15] = clock64() - rcy_start_;                                                                 \
            for (int q = 0; q < 16; ++q)                                                                       \
                __hip_atomic_fetch_add(&g_cycle_stats_ref[q], rcy_[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
        }                                                                                                      \
    } while (0)
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}
#else
#define RCYC_DECL
#define RCYC_MARK(i) ((void)0)
#define RCYC_ADD(i, v) ((void)0)
#define RCYC_FLUSH() ((void)0)
#endif
template <bool BD, int SEG>
__global__ void __launch_bounds__(kRefBlock, ECDNA_REF_MIN_WAVES) ssa_stepper_refdraws(const StepperArgs a) {
    __shared__ uint32_t ccbuf[refdraws::kRingWords * kRefBlock];
    __shared__ double zx[257], zf[257], clog[3 * ECDNA_CLOG_N], cexp[128];
    __shared__ double binv[refdraws::kBinvRows * refdraws::kBinvCols];
    // the sampler tables, staged in LDS (per-lane divergent indices)
    for (uint32_t i = threadIdx.x; i < 257u; i += blockDim.x) {
        zx[i] = kZigX[i];
        zf[i] = kZigF[i];
    }
    for (uint32_t i = threadIdx.x; i < 3u * ECDNA_CLOG_N; i += blockDim.x) clog[i] = kCLog[i];
    for (uint32_t i = threadIdx.x; i < 128u; i += blockDim.x) cexp[i] = kCExp[i];
    refdraws::binv_cdf(binv, threadIdx.x, blockDim.x);
    __syncthreads();
    const uint32_t tid = threadIdx.x;
    const bool hash_on = (a.flags & ECDNA_FLAG_EVENT_HASH) != 0;
    constexpr int K = BD ? 4 : 2;

    refdraws::ChaCha8 rng;
    RCYC_DECL;
    rng.key = a.ref_key;
    rng.buf = ccbuf + tid;
    rng.stride = kRefBlock;

    // Persistent lanes: a lane whose replicate stops writes it out and claims the next one inside the same
    // loop, so lanes never idle while the rest of their wave finishes longer replicates (replicate lengths
    // vary widely: extinctions are short).
    bool active = false;
    uint32_t li = 0;
    uint16_t* row = a.rows;
    float rates[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    uint32_t np = 0, nm = 0;
    // the row's last cell (row[np - 1]), cached: swap_remove reads it at every N+ event, and a read straight from HBM
    // sat on the event's chain (round 6: the cycle counters put ~40 % of a C3 wave's time after the segregation). A
    // division pushes its daughters, so the new tail is known; after a death it is reloaded at the top of the next
    // event, where the load's latency hides behind the first-reaction draws. The row in HBM stays complete.
    uint32_t tail = 0;
    bool tail_ok = false;
    uint64_t h = kFnv0;
    float t = 0.0f;
    uint32_t e = 0, stop = 0, err = 0, sj = 0, uneven_n = 0;
    uint32_t cnt[4] = {0u, 0u, 0u, 0u};

    auto finish = [&]() {
        ecdna_rep_summary_t* s = a.summaries + li;
        s->nminus = nm;
        s->nplus = np;
        s->iters = e;
#pragma unroll
        for (int c = 0; c < 4; ++c) s->events_by_type[c] = cnt[c];
        s->uneven = uneven_n;
        s->time = (double)t;
        s->event_hash = hash_on ? h : 0ull;
        s->stop_reason = stop;
        s->error = err;
        // where the stream stands (words handed out: blocks generated minus those still buffered), for the
        // reference's subsampling with the same rng after the run (src/main.rs:110-123)
        if (a.rng_words) a.rng_words[li] = rng.counter * 16ull - (uint64_t)(rng.tail - rng.head);
        active = false;
    };

    // one advance_step; sets stop (and err) instead of applying the event when the replicate ends
    auto event = [&]() {
        if (e >= a.max_iter) {
            stop = ECDNA_STOP_MAX_ITER;
            return;
        }
        if ((uint64_t)nm + np >= a.stop_cells) {
            stop = ECDNA_STOP_MAX_CELLS;
            return;
        }
        if (t >= a.max_time32) {
            stop = ECDNA_STOP_MAX_TIME;
            return;
        }
        if (!tail_ok && np > 0) {  // (after a death, or at the replicate's start)
            tail = row[np - 1];
            tail_ok = true;
        }
        // first-reaction method, channel order [PN-, PN+, DN-, DN+]
        const uint32_t pop[4] = {nm, np, nm, np};
        int ch = -1;
        float best = __builtin_inff();
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const float lambda = rates[c] * (float)pop[c];
            if (!(lambda > 0.0f)) continue;
            // 1 / lambda, the correctly rounded f32 quotient: rcp_rn (ssa_device.hpp) is RN32(1 / d) for every f32 d in
            // [2^-60, 2^95), and lambda = rate * pop is in [2^-60, 2^92] (the ABI's rate range, u32 populations)
            const float inv = rcp_rn(lambda);
            const float tau = (float)refdraws::exp1(rng, zx, zf, clog, cexp) * inv;
            if (ch < 0 || tau < best) {
                best = tau;
                ch = c;
            }
        }
        RCYC_MARK(2);
        if (ch < 0) {
            stop = ECDNA_STOP_ABSORBING;
            return;
        }
        if (a.n_snap) {  // advance_step's snapshot rule (src/process.rs:122-145), before the event
            const uint64_t total = (uint64_t)nm + np;
            while (sj < a.n_snap) {
                bool any = false;
                for (uint32_t q = sj; q < a.n_snap; ++q) any |= a.snap_cells[q] == total;
                if (!any) break;
                ecdna_snapshot_t* m = a.snap_meta + (uint64_t)li * a.n_snap + sj;
                m->time = (double)t;
                m->nminus = nm;
                m->nplus = np;
                m->taken = 1u;
                m->reserved = 0u;
                if (a.snap_rows) {
                    uint16_t* dst = a.snap_rows + ((uint64_t)li * a.n_snap + sj) * a.snap_stride;
                    for (uint32_t j = 0; j < np; ++j) dst[j] = row[j];
                }
                ++sj;
            }
        }
        uint64_t x = (uint64_t)ch;
        if (ch == ECDNA_EV_PROLIF_NMINUS) {
            nm += 1;
        } else if (ch == ECDNA_EV_DEATH_NMINUS) {
            nm -= 1;
        } else if (ch == ECDNA_EV_DEATH_NPLUS) {
            const uint32_t i = (uint32_t)rng.gen_range(np);
            if (i != np - 1) row[i] = (uint16_t)tail;  // swap_remove(i)
            np -= 1;
            tail_ok = false;
            x |= (uint64_t)i << 20;
        } else {  // ProliferateNPlus
            const uint32_t i = (uint32_t)rng.gen_range(np);
            const uint32_t k = i == np - 1 ? tail : row[i];
            RCYC_MARK(3);
            if (k > 32767u) {  // checked_mul panic (src/proliferation.rs:63-67)
                err = ECDNA_REP_ERR_OVERFLOW;
                stop = ECDNA_STOP_ERROR;
                return;
            }
            const uint32_t n = 2u * k;
            uint32_t k1 = 0;
            int un = 0;  // 0 False, 1 True, 2 TrueWithoutNMinusIncrease
            if (SEG == ECDNA_SEG_DETERMINISTIC) {
                k1 = n / 2u;
            } else if (SEG == ECDNA_SEG_BINOMIAL_NO_UNEVEN) {
                int tries = 0;
                do {
                    k1 = refdraws::binomial_half(rng, n, a.ref_btpe, clog, binv);
                } while ((k1 == 0u || k1 == n) && ++tries < 4096);
                if (k1 == 0u || k1 == n) {
                    err = ECDNA_REP_ERR_REJECTION;
                    stop = ECDNA_STOP_ERROR;
                    return;
                }
            } else {
#ifdef ECDNA_CYCLE_STATS  // (the two samplers as separate regions: [6] BINV, [4] BTPE)
                const bool binv_n = refdraws::binomial_half_is_binv(n);
                if (binv_n) k1 = refdraws::binv_half(rng, n, binv);
                RCYC_MARK(6);
                if (!binv_n) k1 = refdraws::btpe_half(rng, n, a.ref_btpe, clog);
#else
                k1 = refdraws::binomial_half(rng, n, a.ref_btpe, clog, binv);
#endif
                if (k1 == 0u || k1 == n) un = SEG == ECDNA_SEG_BINOMIAL_NO_NMINUS ? 2 : 1;
            }
            RCYC_MARK(4);
            if (un == 0 && np + 1u > a.cell_cap) {
                err = ECDNA_REP_ERR_CELL_CAP;
                stop = ECDNA_STOP_ERROR;
                return;
            }
            if (i != np - 1) row[i] = (uint16_t)tail;  // pick_remove_random_nplus: swap_remove(i)
            np -= 1;
            if (un == 0) {
                row[np++] = (uint16_t)k1;
                row[np++] = (uint16_t)(n - k1);
                tail = n - k1;
            } else {
                if (un == 1) nm += 1;
                row[np++] = (uint16_t)n;
                tail = n;
                uneven_n += 1;
            }
            x |= ((uint64_t)k1 << 2) | ((uint64_t)i << 20);
        }
        cnt[ch] += 1;
        e += 1;
        t = t + best;
        if (hash_on) h = (h ^ x) * kFnvP;
    };

    for (;;) {
        RCYC_ADD(8, 1);
        if (!active) {  // claim the next replicate (and set it up)
            li = atomicAdd(a.head, 1u);
            if (li >= a.n) break;
            const uint64_t rid = a.rid0 + (uint64_t)li * a.rid_stride;
            row = a.rows + (uint64_t)li * a.row_stride;
            const uint64_t set = rid / a.reps_per_set;
            const float4 r4 = a.rates[set];
            rates[0] = r4.x;
            rates[1] = r4.y;
            rates[2] = r4.z;
            rates[3] = r4.w;
            const uint16_t* src = a.init_copies;
            np = a.init_nplus;
            if (a.init_offsets) {
                src = a.init_copies + a.init_offsets[set];
                np = a.init_offsets[set + 1] - a.init_offsets[set];
            }
            for (uint32_t j = 0; j < np; ++j) row[j] = src[j];
            nm = (uint32_t)(a.init_nminus_set ? a.init_nminus_set[set] : a.init_nminus);
            tail_ok = false;
            const uint64_t stream = a.seed * 10ull + rid;  // src/main.rs:56-58
            rng.reset();
            rng.s_lo = (uint32_t)stream;
            rng.s_hi = (uint32_t)(stream >> 32);
            h = kFnv0;
            t = 0.0f;
            e = stop = err = sj = uneven_n = 0;
#pragma unroll
            for (int c = 0; c < 4; ++c) cnt[c] = 0u;
            active = true;
            if (np == 0 && nm == 0) {  // ensure!(!distribution.is_empty()) src/process.rs:88, 232
                err = ECDNA_REP_ERR_EMPTY;
                stop = ECDNA_STOP_ERROR;
                finish();
                continue;
            }
        }
        RCYC_MARK(0);
#ifdef ECDNA_CYCLE_STATS
        {
            const bool need = rng.tail - rng.head < 16u;
            const uint32_t l_ = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
            RCYC_ADD(9, l_ == (uint32_t)__builtin_amdgcn_readfirstlane(l_) ? 1u : 0u);  // (summed over lanes: per wave)
            RCYC_ADD(10, need ? 1u : 0u);
        }
#endif
        rng.top_up();  // (one refill site per iteration for the wave; see refdraws::ChaCha8)
        RCYC_MARK(1);
        event();
        RCYC_MARK(5);
        if (stop) finish();
    }
    RCYC_FLUSH();
}

#ifdef ECDNA_CYCLE_STATS
// Development: read (and reset) the reference-draws stepper's cycle counters (tools/cycle_stats.py ref)
extern "C" int ecdna_dev_cycle_stats_ref(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cycle_stats_ref), sizeof(g_cycle_stats_ref)) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_cycle_stats_ref), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

#define ECDNA_REF_SEG(BD)                                                                                    \
    {(const void*)ssa_stepper_refdraws<BD, 0>, (const void*)ssa_stepper_refdraws<BD, 1>,                      \
     (const void*)ssa_stepper_refdraws<BD, 2>, (const void*)ssa_stepper_refdraws<BD, 3>}
static const void* const kRefTable[2][4] = {ECDNA_REF_SEG(false), ECDNA_REF_SEG(true)};

const void* refdraws_kernel(int birth_death, int segregation) {
    return kRefTable[birth_death ? 1 : 0][segregation & 3];
}

int refdraws_block() { return (int)kRefBlock; }

hipError_t launch_refdraws(const StepperArgs& a, int birth_death, int segregation, uint32_t blocks,
                           hipStream_t stream) {
    StepperArgs copy = a;
    void* args[] = {&copy};
    return hipLaunchKernel(refdraws_kernel(birth_death, segregation), dim3(blocks), dim3(kRefBlock), args, 0, stream);
}

}  // namespace ecdna
