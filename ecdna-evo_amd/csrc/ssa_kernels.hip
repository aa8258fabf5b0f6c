// ssa_kernels.hip — the MI355X (gfx950) many-replicate Gillespie SSA stepper
// and the copy-number histogram pass.
//
// One replicate per lane. A lane runs the whole sosa::simulate loop
// (external crate sosa 3.0.3; call sites src/main.rs:92-99, 166-173) for its
// replicate: stop checks, propensities of update_state's population vector
// (src/process.rs:187-196, 339-344), one Philox4x32-10 block per event, the
// direct-method channel pick, the event of advance_step
// (src/process.rs:147-184, 291-336) — Exponential::increase_nplus with its
// swap_remove pick and Segregate rule (src/proliferation.rs:25-111,
// src/segregation.rs:110-194), increase_nminus / CellDeath
// (src/proliferation.rs:113-140) — and the time accumulation
// (src/process.rs:184, 336). When its replicate stops, the lane writes the
// summary and pulls the next replicate id from a work counter (persistent
// grid), so early extinctions in birth–death runs do not idle the lane.
//
// Memory: every replicate owns a u16 row of row_stride cells in HBM
// (replicate-major, 128-B aligned). An event touches at most one random cell
// (the swap_remove pick) plus the row's tail; the tail VALUE is cached in a
// register (the reference re-reads it through Vec::swap_remove), so a
// ProliferateNPlus costs one random 2-B load and up to three 2-B stores.
#include <stdlib.h>

#include "ssa_device.hpp"
#include "ssa_launch.h"

#pragma clang fp contract(off)

namespace ecdna {

constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;
constexpr uint32_t kNoUnevenMaxTries = 4096;

// LDS tail window (WIN): the last cells of each lane's row — the stack end that swap_remove reads
// and the daughter pushes write — live in LDS, cells [wb, np); cells [0, wb) live in HBM. Ring
// slot = position % kWin, laid out [slot][lane] so a wave's 2-B accesses spread over the banks.
// The window is flushed / refilled in aligned 16-cell (32-B, one HBM write sector) blocks, so the
// pushes cost ~1/16 of a write request instead of one each. Invariant: 1 <= np - wb <= kWin
// whenever np > 0; wb is a multiple of kFlush.
// Explicitly global (address space 1) 2-B load: pointers read from the kernel-argument struct are
// generic, and the optimizer would otherwise fuse the LDS and HBM reads of cell_get into a flat load.
__device__ __forceinline__ uint32_t gload_u16(const uint16_t* p) {
    return *(const __attribute__((address_space(1))) uint16_t*)p;
}

constexpr uint32_t kWin = 32;
constexpr uint32_t kFlush = 16;

template <bool BD, int SEG, bool WIN>
__global__ void __launch_bounds__(kStepperBlock) ssa_stepper(const StepperArgs a) {
    __shared__ uint16_t win[WIN ? kWin + 1 : 1][kStepperBlock];  // + 1 spare row
    __shared__ float2 logtab[ECDNA_LOGTAB_N];
    stage_logtab(logtab);
    const uint32_t tid = threadIdx.x;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    const bool f32t = (a.flags & ECDNA_FLAG_TIME_F32) != 0;
    const bool hash_on = (a.flags & ECDNA_FLAG_EVENT_HASH) != 0;

    bool active = false, have = false;
    uint32_t li = 0;
    uint64_t rid = 0;
    uint16_t* row = a.rows;  // (not nullptr: keeps the pointer provably global, no flat_* accesses)
    uint32_t nm = 0, np = 0, tail = 0, wb = 0;
    uint32_t sp0 = 0, sp1 = 0, nsp = 0;  // spare stream words (draw mapping v3)
    bool tail_ok = false;  // (HBM-only variant: tail value cached; the window variant always has it)
    // cell access through the window (WIN) or straight to HBM
    auto slot = [&](uint32_t pos) -> uint16_t& { return win[WIN ? (pos & (kWin - 1)) : 0][tid]; };
    // LDS side unconditional (a spare row absorbs stores outside the window), HBM side under the
    // branch: symmetric conditional accesses would be merged into one flat_load / flat_store.
    auto cell_get = [&](uint32_t pos) -> uint32_t {
        if (!WIN) return row[pos];
        uint32_t v = slot(pos);
        if (pos < wb) v = gload_u16(row + pos);
        return v;
    };
    auto cell_put = [&](uint32_t pos, uint32_t v) {
        if (!WIN) {
            row[pos] = (uint16_t)v;
            return;
        }
        const bool in_win = pos >= wb;
        win[in_win ? (pos & (kWin - 1)) : kWin][tid] = (uint16_t)v;
        if (!in_win) {
            row[pos] = (uint16_t)v;
        }
    };
    auto flush_block = [&]() {  // cells [wb, wb + 16) -> HBM as two 16-B stores; wb += 16
        uint32_t p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = (uint32_t)slot(wb + 2 * j) | ((uint32_t)slot(wb + 2 * j + 1) << 16);
        uint4* dst = reinterpret_cast<uint4*>(row + wb);
        dst[0] = make_uint4(p[0], p[1], p[2], p[3]);
        dst[1] = make_uint4(p[4], p[5], p[6], p[7]);
        wb += kFlush;
    };
    auto refill_block = [&]() {  // wb -= 16; cells [wb, wb + 16) HBM -> LDS
        wb -= kFlush;
        const uint4* src = reinterpret_cast<const uint4*>(row + wb);
        const uint4 x0 = src[0], x1 = src[1];
        const uint32_t p[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            slot(wb + 2 * j) = (uint16_t)(p[j] & 0xffffu);
            slot(wb + 2 * j + 1) = (uint16_t)(p[j] >> 16);
        }
    };
    float b0 = 0.f, b1 = 0.f, d0 = 0.f, d1 = 0.f;
    double t = 0.0;
    float t32 = 0.f;
    // Per-type event counts: only DeathNMinus (BD) and uneven splits are counted per event; the other
    // three follow at the end from the event total and the population changes (src/proliferation.rs:
    // an even split adds one N+ cell, an uneven one none (plus an N- cell unless NoNminus), a death
    // removes one): dnp = pp - un - dp, dnm = pm - dm + un(with an N- daughter), e = pm + pp + dm + dp.
    uint32_t e = 0, n_dm = 0, n_un = 0, np0 = 0, nm0 = 0;
    uint64_t h = kFnvOffset;
    uint32_t stop = 0, err = 0;
    uint32_t sj = 0;  // snapshots popped so far (the deque's front index)

    for (;;) {
        if (!active) {
            if (have) {
                if (WIN)
                    for (uint32_t j = wb; j < np; ++j) row[j] = slot(j);  // whole row back in HBM
                ecdna_rep_summary_t* s = a.summaries + li;
                s->nminus = nm;
                s->nplus = np;
                s->iters = e;
                {
                    const uint32_t un1 = SEG == ECDNA_SEG_BINOMIAL_NO_NMINUS ? 0u : n_un;  // uneven with an N- daughter
                    const uint32_t n_pm = nm - nm0 + n_dm - un1;                          // (mod 2^32)
                    const uint32_t pp_minus_dp = np - np0 + n_un;
                    const uint32_t pp_plus_dp = e - n_pm - n_dm;
                    const uint32_t n_pp = (pp_plus_dp + pp_minus_dp) >> 1;
                    s->events_by_type[0] = n_pm;
                    s->events_by_type[1] = n_pp;
                    s->events_by_type[2] = n_dm;
                    s->events_by_type[3] = pp_plus_dp - n_pp;
                    s->uneven = n_un;
                }
                s->time = f32t ? (double)t32 : t;
                s->event_hash = hash_on ? h : 0ull;
                s->stop_reason = stop;
                s->error = err;
            }
            uint32_t i = atomicAdd(a.head, 1u);
            if (i >= a.n) break;
            if (a.order) i = a.order[i];
            have = true;
            active = true;
            li = i;
            rid = a.rid0 + (uint64_t)i * a.rid_stride;
            row = a.rows + (uint64_t)i * a.row_stride;
            const uint64_t set = rid / a.reps_per_set;
            const float4 r = a.rates[set];
            b0 = r.x;
            b1 = r.y;
            d0 = r.z;
            d1 = r.w;
            const uint16_t* src = a.init_copies;
            uint32_t cnt = a.init_nplus;
            if (a.init_offsets) {
                src = a.init_copies + a.init_offsets[set];
                cnt = a.init_offsets[set + 1] - a.init_offsets[set];
            }
            wb = (WIN && cnt) ? ((cnt - 1) / kFlush) * kFlush : 0;
            if (WIN) {
                for (uint32_t j = 0; j < wb; ++j) row[j] = src[j];
                for (uint32_t j = wb; j < cnt; ++j) slot(j) = src[j];
            } else {
                for (uint32_t j = 0; j < cnt; ++j) row[j] = src[j];
            }
            np = cnt;
            nm = (uint32_t)(a.init_nminus_set ? a.init_nminus_set[set] : a.init_nminus);
            tail_ok = false;
            if (WIN && cnt) tail = src[cnt - 1];
            t = 0.0;
            t32 = 0.f;
            e = n_dm = n_un = 0;
            np0 = np;
            nm0 = nm;
            nsp = 0;
            h = kFnvOffset;
            stop = 0;
            err = 0;
            sj = 0;
            if (np == 0 && nm == 0) {  // ensure!(!distribution.is_empty()) src/process.rs:88, 232
                err = ECDNA_REP_ERR_EMPTY;
                stop = ECDNA_STOP_ERROR;
                active = false;
                continue;
            }
        }

        // propensities rate_i * population_i over [n-, n+(, n-, n+)] in f32 (the reference's own, src/main.rs:67, 139),
        // their cumulative sums in f64 (draw mapping v7); the time step divides by a0 = RN32(A)
        const float fnm = (float)nm, fnp = (float)np;
        const double cA = (double)(b0 * fnm);
        const double cB = cA + (double)(b1 * fnp);
        double cC = cB, A = cB;
        if (BD) {
            cC = cB + (double)(d0 * fnm);
            A = cC + (double)(d1 * fnp);
        }
        const float a0 = (float)A;

        // stop checks, in the order of DESIGN.md §3.1 (selects, last write = first check)
        {
            const bool t_over = f32t ? (t32 >= a.max_time32) : (t >= a.max_time);
            uint32_t s = (a0 > 0.0f) ? 0u : (uint32_t)ECDNA_STOP_ABSORBING;
            s = t_over ? (uint32_t)ECDNA_STOP_MAX_TIME : s;
            s = ((uint64_t)nm + np >= a.stop_cells) ? (uint32_t)ECDNA_STOP_MAX_CELLS : s;
            s = (e >= a.max_iter) ? (uint32_t)ECDNA_STOP_MAX_ITER : s;
            if (s) {
                stop = s;
                active = false;
                continue;
            }
        }

        // snapshots, checked at the top of advance_step before the event is applied
        // (src/process.rs:122-145): while ANY remaining snapshot equals n- + n+, pop the FRONT one
        // and save the current state into its slot.
        if (a.n_snap) {
            const uint64_t total = (uint64_t)nm + np;
            while (sj < a.n_snap) {
                bool any = false;
                for (uint32_t q = 0; q < a.n_snap; ++q) any |= (q >= sj) && (a.snap_cells[q] == total);
                if (!any) break;
                ecdna_snapshot_t* m = a.snap_meta + (uint64_t)li * a.n_snap + sj;
                m->time = f32t ? (double)t32 : t;
                m->nminus = nm;
                m->nplus = np;
                m->taken = 1u;
                m->reserved = 0u;
                if (a.snap_rows) {
                    uint16_t* dst = a.snap_rows + ((uint64_t)li * a.n_snap + sj) * a.snap_stride;
                    const uint32_t hbm_end = WIN ? (wb < np ? wb : np) : np;
                    for (uint32_t j = 0; j < hbm_end; ++j) dst[j] = row[j];
                    if (WIN)
                        for (uint32_t j = hbm_end; j < np; ++j) dst[j] = slot(j);
                }
                ++sj;
            }
        }

        if (!WIN && !tail_ok && np > 0) {  // reload the cached tail value (after a DeathNPlus)
            tail = cell_get(np - 1);
            tail_ok = true;
        }

        const uint32_t rid_lo = (uint32_t)rid, rid_hi = (uint32_t)(rid >> 32);
        const uint4 w = philox4x32_10(make_uint4(e, 0u, rid_lo, rid_hi), k0, k1);
        const double target = chan_target(w.y, A);
        uint32_t ch;
        if (BD)
            ch = target < cA ? 0u : (target < cB ? 1u : (target < cC ? 2u : 3u));
        else
            ch = target < cA ? 0u : 1u;
#ifdef ECDNA_INJECT_EMPTY_NPLUS  // (fault-injection builds only, tools/inject_check.py: an N+ event with no N+ cell)
        if (np == 0u) ch = BD ? 3u : 1u;
#endif

        WordStream ws;
        ws.w2 = w.z;
        ws.w3 = w.w;
        ws.s0 = sp0;
        ws.s1 = sp1;
        ws.nsp = nsp;
        ws.e = e;
        ws.rid_lo = rid_lo;
        ws.rid_hi = rid_hi;
        ws.k0 = k0;
        ws.k1 = k1;
        ws.pos = 1;
        ws.blk_id = 0;
        ws.blk = make_uint4(0, 0, 0, 0);

        uint32_t idx = 0, k = 0;
        if (ch & 1u) {
            // uniform N+ cell: Lemire multiply-shift on w2, exact rejection from the stream
            uint64_t m = (uint64_t)w.z * np;
            uint32_t lo = (uint32_t)m;
            if (lo < np) {
                const uint32_t thr = (0u - np) % np;
                while (lo < thr) {
                    m = (uint64_t)ws.next() * np;
                    lo = (uint32_t)m;
                }
            }
            idx = (uint32_t)(m >> 32);
            // the indexing invariant (ECDNA_REP_ERR_INTERNAL, ABI v11): an N+ event needs an N+ cell, and the pick
            // stays below n+ (np == 0 gives idx 0 here). Unreachable under draw mapping v7; a broken channel would
            // otherwise wrap np and index off the row (the r05e illegal address). The oracle returns the same code.
            if (idx >= np) {
                err = ECDNA_REP_ERR_INTERNAL;
                stop = ECDNA_STOP_ERROR;
                active = false;
                continue;
            }
            if (ch == 1u) {
                if (idx == np - 1)
                    k = tail;
                else
                    k = cell_get(idx);
            }
        }

        // Exponential::increase_nplus (src/proliferation.rs:25-111): its draws and error checks
        uint32_t n = 0, k1v = 0;
        uint32_t un = 0;  // 0 False, 1 True, 2 TrueWithoutNMinusIncrease
        if (ch == 1u) {
            if (k > 32767u) {  // checked_mul panic (src/proliferation.rs:63-67)
                err = ECDNA_REP_ERR_OVERFLOW;
                stop = ECDNA_STOP_ERROR;
                active = false;
                continue;
            }
            n = 2u * k;
            if (SEG == ECDNA_SEG_DETERMINISTIC) {
                k1v = k;
            } else {
                if (ws.pos == 1 && n <= 32u) {
                    k1v = __popc(n == 32u ? w.w : (w.w & ((1u << n) - 1u)));
                    ws.pos = 2;
                } else if (ws.pos == 1 && n <= 64u && nsp >= 1u) {  // w3 and the first spare word
                    k1v = __popc(w.w) + __popc(n == 64u ? sp0 : (sp0 & ((1u << (n - 32u)) - 1u)));
                    ws.pos = 3;
                } else {
                    k1v = ws.binomial_half(n);
                }
                if (SEG == ECDNA_SEG_BINOMIAL_NO_UNEVEN) {
                    uint32_t tries = 1;
                    bool rej = false;
                    if (n <= 32u && (k1v == 0u || k1v == n)) {
                        k1v = ws.redraw_even_small(n, tries, kNoUnevenMaxTries, rej);
                    } else {
                        while (k1v == 0u || k1v == n) {
                            if (tries == kNoUnevenMaxTries) {
                                rej = true;
                                break;
                            }
                            k1v = ws.binomial_half(n);
                            ++tries;
                        }
                    }
                    if (rej) {
                        err = ECDNA_REP_ERR_REJECTION;
                        stop = ECDNA_STOP_ERROR;
                        active = false;
                        continue;
                    }
                } else if (k1v == 0u || k1v == n) {
                    un = (SEG == ECDNA_SEG_BINOMIAL_NO_NMINUS) ? 2u : 1u;
                }
            }
            if (un == 0u && np + 1u > a.cell_cap) {
                err = ECDNA_REP_ERR_CELL_CAP;
                stop = ECDNA_STOP_ERROR;
                active = false;
                continue;
            }
        }

        // waiting time
        const float tau = softlog_neg(w.x, logtab) * rcp_rn(a0);  // (draw mapping v8)

        uint64_t x = ch;
        if (ch == 1u) {
            // swap_remove(idx); the slot already holds the tail's copy number about 7 % of the time at
            // C3 (sum of p_k^2), and random HBM stores are the stepper's binding limit
            if (idx != np - 1 && k != tail) cell_put(idx, tail);
            // the pushes land at np - 1 and np, inside the window (np - wb >= 1 before, <= 32 after a flush)
            if (un == 0u) {
                if (WIN) slot(np - 1) = (uint16_t)k1v; else cell_put(np - 1, k1v);  // push k1, push k2
                if (WIN && np - wb == kWin) flush_block();
                if (WIN) slot(np) = (uint16_t)(n - k1v); else cell_put(np, n - k1v);
                np += 1;
                tail = n - k1v;
            } else {
                if (WIN) slot(np - 1) = (uint16_t)n; else cell_put(np - 1, n);  // push k1 + k2
                tail = n;
                nm += (un == 1u) ? 1u : 0u;
                n_un += 1;
            }
            x |= ((uint64_t)k1v << 2) | ((uint64_t)idx << 20);
        } else if (BD && ch == 3u) {  // CellDeath::decrease_nplus (src/proliferation.rs:126-133)
            if (idx != np - 1) cell_put(idx, tail);
            np -= 1;
            if (WIN) {
                if (np > 0 && np == wb) refill_block();  // keep the window non-empty
                if (np > 0) tail = slot(np - 1);
            } else {
                tail_ok = (np > 0) && (idx == np - 1);
            }
            x |= (uint64_t)idx << 20;
        }
        spares_update((ch & 1u) ? ws.pos : 0u, w.z, w.w, sp0, sp1, nsp);
        // increase_nminus / decrease_nminus (src/proliferation.rs:113-117, 135-139) and the counters
        nm = nm + (ch == 0u ? 1u : 0u) - (ch == 2u ? 1u : 0u);
        if (BD) n_dm += ch == 2u ? 1u : 0u;
        e += 1;
        if (f32t)
            t32 = t32 + tau;
        else
            t = t + (double)tau;
        if (hash_on) h = (h ^ x) * kFnvPrime;
    }
}

// ---------------------------------------------------------------- bin store (ECDNA_FLAG_BIN_STORE)
//
// DESIGN.md §3.3 / §5. A lane's N+ cells are counts c[k] of cells with k copies, k = 1..K with
// K = 8 * NG, held in LDS, plus a row B (HBM, the replicate's row) of the cells with k > K. The uniform
// cell pick indexes the canonical order (all k = 1 cells, then k = 2, ..., then B), found by a two-level
// scan: NG group sums (8 bins each), then the 8 bins of the chosen group. Each is one or two 16-B LDS
// reads per lane; updates are fire-and-forget LDS atomic adds on the packed counters. In the common case
// (every copy number involved <= K) an event touches no HBM at all.
//
// LDS per lane: counts NG*8 (u16, or u32 when C32) + NG group sums of the same width. u16 counters are
// laid out [vector][lane] in 16-B vectors so a wave's 16-B reads are contiguous (conflict-free); u32
// counters [counter][lane] (planar), see word_index.
template <int NG, bool C32>
struct BinLayout {
    static constexpr int kK = 8 * NG;                       // binned copy numbers 1..kK
    static constexpr int kPerVec = C32 ? 4 : 8;             // counters per 16-B vector
    static constexpr int kGroupVecs = 8 / kPerVec;          // vectors per group of 8 bins
    static constexpr int kBinVecs = NG * kGroupVecs;
    static constexpr int kSumVecs = (NG + kPerVec - 1) / kPerVec;
};

// ---- replicate rotation helpers (bin store; DESIGN.md §5 "Rotation")
//
// A parked replicate is handed from one CU to another of the SAME XCD (partition = XCC id): the parker's
// plain stores land in the XCD's L2, it waits for them (vmcnt(0)) before publishing PARKED with an
// agent-scope atomic, and the resumer reads the state with sc1 loads (vector L1 bypassed, served by that
// L2) only after its compare-and-swap PARKED -> RUNNING has returned. Flags and counters are only ever
// read through RMW atomics (compare-and-swap with new == expected, which the compiler cannot turn into a
// plain load), so a stale cached copy can never hide a waiting replicate.
constexpr int kCpolSc1 = 16;  // buffer cache policy: sc1 (gfx940+ bit 4)

// The second instruction schedule of the bin stepper (ECDNA_ILP_BUILD: this file compiled again with
// -mllvm -amdgpu-sched-strategy=max-ilp, Makefile): only its bin-stepper table and accessor are defined
// there (template argument SCH = 1 keeps its kernels distinct from this build's SCH = 0 ones). Its
// development counters are its own (static): the tools read the default build's.
#ifndef ECDNA_FF_MAX
#define ECDNA_FF_MAX 16
#endif
#ifndef ECDNA_FF_ENTER8
#define ECDNA_FF_ENTER8 7  // enter when >= this many eighths of the lanes expect an N- event w.p. >= ECDNA_FF_ENTER8 / 8
#endif
#ifndef ECDNA_FF_TEST_EVERY
#define ECDNA_FF_TEST_EVERY 32u  // while a wave is not fast-forwarding, its entry test runs every this many
                                // iterations (C3, which never enters: 8 -> 32 is -1.2 %; C4 / C5 unchanged)
#endif
#ifndef ECDNA_FF_STAY8
#define ECDNA_FF_STAY8 7   // keep going while >= this many eighths of the entered lanes do
#endif
// the entry test runs when a wave-uniform countdown reaches 0 (reset to ECDNA_FF_TEST_EVERY, or to 1 while the wave
// fast-forwards)
static_assert(ECDNA_FF_TEST_EVERY > 0, "ECDNA_FF_TEST_EVERY must be positive");
constexpr uint32_t kFfMax = ECDNA_FF_MAX;  // N- fast-forward: events per full iteration at most

#ifdef ECDNA_ILP_BUILD
#define ECDNA_DEV_STATIC static
#else
#define ECDNA_DEV_STATIC
#endif

#ifdef ECDNA_PAIR_CHECK
// Debug builds (-DECDNA_PAIR_CHECK): paired steps whose helper was out of step with its owner (must stay 0)
ECDNA_DEV_STATIC __device__ unsigned int g_pair_check;
#endif

// Development counters of the rotation (built with -DECDNA_ROT_STATS only; tools/rot_stats.py)
#ifdef ECDNA_ROT_STATS
ECDNA_DEV_STATIC __device__ unsigned long long g_rot_stats[12];
#define ROT_STAT(i, v) __hip_atomic_fetch_add(&g_rot_stats[i], (unsigned long long)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define ROT_STAT(i, v) ((void)0)
#endif

// Development counters of the bin stepper's rare blocks (built with -DECDNA_PATH_STATS only;
// tools/path_stats.py): how many wave-iterations execute each block (the first active lane counts).
#ifdef ECDNA_PATH_STATS
ECDNA_DEV_STATIC __device__ unsigned long long g_path_stats[8];
// counts in registers (the first active lane of the block adds 1, or the active-lane count), summed into
// g_path_stats once per lane at exit
#define PATH_STAT(i) (ps[i] += ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(__builtin_amdgcn_read_exec())) ? 1u : 0u)
#define PATH_STAT_LANES(i)                                                                                      \
    do {                                                                                                        \
        const uint64_t ex_ = __builtin_amdgcn_read_exec();                                                      \
        const uint32_t pc_ = __builtin_amdgcn_readfirstlane((uint32_t)__builtin_popcountll(ex_));              \
        ps[i] += ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex_)) ? pc_ : 0u;                          \
    } while (0)
#define PATH_STATS_DECL uint32_t ps[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u}
#define PATH_STATS_FLUSH()                                                                                      \
    for (int q = 0; q < 8; ++q)                                                                               \
        if (ps[q]) __hip_atomic_fetch_add(&g_path_stats[q], (unsigned long long)ps[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define PATH_STAT(i) ((void)0)
#define PATH_STAT_LANES(i) ((void)0)
#define PATH_STATS_DECL
#define PATH_STATS_FLUSH() ((void)0)
#endif

// Development cycle counters of the bin stepper's loop sections (built with -DECDNA_CYCLE_STATS only;
// tools/cycle_stats.py), per wave, summed over waves: [0] shader-clock cycles from the loop top through the
// replicate boundary, [1] the fast-forward block (entry test included), [2] the full event and the loop
// latch, [3] iterations, [4] fast-forward entries, [5] fast-forward steps, [6] lanes entering the full event,
// [7] whole-kernel cycles; inside the full event (lanes past the stop test) [8] propensities and stop test,
// [9] Philox block and channel, [10] cell pick, [11] segregation, [12] error and capacity checks, [13] time
// step, [14] counter and large-k row updates ([2] then holds the commit and the loop latch). Marks sit at
// wave-uniform points of their region (a mark waits for the wave's LDS operations: a rough attribution);
// the wave's lane 0 flushes.
#ifdef ECDNA_CYCLE_STATS
#ifdef ECDNA_ILP_BUILD
#define ECDNA_CYC_SYM g_cycle_stats_ilp
#else
#define ECDNA_CYC_SYM g_cycle_stats
#endif
ECDNA_DEV_STATIC __device__ unsigned long long ECDNA_CYC_SYM[16];
#define CYC_DECL                                                                                               \
    unsigned long long cy_[16] = {};                                                                           \
    const unsigned long long cy_start_ = clock64();                                                           \
    unsigned long long cy_t_ = cy_start_
#define CYC_MARK(i)                                                                                            \
    do {                                                                                                       \
        const unsigned long long n_ = clock64();                                                               \
        cy_[i] += n_ - cy_t_;                                                                                  \
        cy_t_ = n_;                                                                                            \
    } while (0)
#define CYC_ADD(i, v) (cy_[i] += (unsigned long long)(v))
#define CYC_FLUSH()                                                                                            \
    do {                                                                                                       \
        cy_[7] = clock64() - cy_start_;                                                                        \
        if ((threadIdx.x & 63u) == 0u)                                                                         \
            for (int q = 0; q < 16; ++q)                                                                       \
                __hip_atomic_fetch_add(&ECDNA_CYC_SYM[q], cy_[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   \
    } while (0)
#else
#define CYC_DECL
#define CYC_MARK(i) ((void)0)
#define CYC_ADD(i, v) ((void)0)
#define CYC_FLUSH() ((void)0)
#endif

// The kernel argument block as seen from a rare path: read through a pointer the compiler cannot prove
// loop-invariant, so those loads stay inside the rare block instead of holding scalar registers across
// the event loop (the bin stepper's event path already fills the SGPR file).
using KArgs = const __attribute__((address_space(4))) StepperArgs;
__device__ __forceinline__ KArgs* rare_args() {
    KArgs* p = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

__device__ __forceinline__ uint4 ld_l2_b128(const void* base, uint32_t byte_off) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff,
                                                                         0x00020000);
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kCpolSc1));
}

// Large-k row cell of a replicate that may have run on another CU of this XCD: vector L1 bypassed
__device__ __forceinline__ uint32_t gload_u16_l2(const uint16_t* p) {
    return __hip_atomic_load(const_cast<uint16_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename T>
__device__ __forceinline__ T atomic_read(T* p) {  // memory-side read: CAS(p, 0 -> 0)
    T e = 0;
    __hip_atomic_compare_exchange_strong(p, &e, e, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return e;
}

// Replicate r's state word: from RUNNING (only its owner changes a RUNNING word) to `to`
__device__ __forceinline__ void rot_set(uint32_t* flags, uint32_t r, uint32_t to) {
    __hip_atomic_exchange(flags + r, to, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Claim the next waiting replicate of partition `pp` by walking its items one at a time (the lanes of a
// wave that walk together share one aggregated add on the head): FRESH or PARKED when !fresh_only; FRESH
// only, and only during the partition's first pass, when fresh_only. The count is checked before the
// head moves: a lane that has nothing to claim must not consume (and so skip) another lane's item.
// (C3: per-lane count reads and read-then-CAS 91 ms; one count read per wave round and a blind CAS 88 ms.) Returns 0 when the partition has nothing left to claim, else the state claimed plus one,
// with the replicate in `out` (chunk-local).
__device__ __forceinline__ uint32_t rot_claim(KArgs* ra, uint32_t pp, bool fresh_only, uint32_t& out) {
    RotPart* P = ra->rot_parts + pp;
    const uint32_t n_pad = ra->rot_n_pad;
    uint32_t* const flags = ra->rot_flags;
    const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#pragma unroll 1
    for (;;) {
        // one read of the count per wave round (the first walking lane), before any item is taken
        int w = 0;
        if (lane == __builtin_amdgcn_readfirstlane(lane)) w = atomic_read(fresh_only ? &P->fresh : &P->waiting);
        if (__builtin_amdgcn_readfirstlane(w) <= 0) return 0u;
        const unsigned long long j =
            __hip_atomic_fetch_add(&P->head, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ROT_STAT(fresh_only ? 4 : 1, 1);
        if (fresh_only && j >= n_pad) return 0u;  // past the first pass: no fresh replicate is left
        // partitions interleave the replicates (r mod kRotParts), so a run whose cost varies along the
        // replicate order (an ABC sweep's parameter sets) gives every XCD the same mix
        uint32_t r = pp + kRotParts * (j < (1ull << 32) ? (uint32_t)j % n_pad : (uint32_t)(j % n_pad));
        if (ra->order) {  // item r starts the order's r-th replicate (costliest sets first); past n: padding
            if (r >= ra->n) continue;
            r = ra->order[r];
        }
        // blind compare-and-swap from the likelier waiting state; the value it returns says whether the
        // item is FRESH after all (one more try) or not waiting (RUNNING / DONE: next item)
        uint32_t st = fresh_only ? (uint32_t)ROT_FRESH : (uint32_t)ROT_PARKED;
        if (__hip_atomic_compare_exchange_strong(flags + r, &st, (uint32_t)ROT_RUNNING, __ATOMIC_RELAXED,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
            (!fresh_only && st == ROT_FRESH &&
             __hip_atomic_compare_exchange_strong(flags + r, &st, (uint32_t)ROT_RUNNING, __ATOMIC_RELAXED,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_fetch_add(&P->waiting, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (st == ROT_FRESH) __hip_atomic_fetch_add(&P->fresh, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            out = r;
            ROT_STAT(st == ROT_FRESH ? 2 : 3, 1);
            return st + 1u;
        }
    }
}

// Counter j of a 16-B vector (8 x u16 or 4 x u32)
template <bool C32>
__device__ __forceinline__ uint32_t vec_get(const uint4& v, int j) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    if (C32) return w[j];
    return (w[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
}

// SCH: the build's schedule (no code): 0 occupancy-first, 1 max-ILP (ECDNA_ILP_BUILD), 2 occupancy-first
// capped at 128 VGPRs so that four 256-lane workgroups fit a CU (K = 64 / u16 only, many replicates per lane)
// PAIR (lone waves, DESIGN.md §5 "Paired lanes"): lane l < 32 of every wave owns a replicate, lane l + 32 is its
// helper: in the N- fast-forward both compute a Philox block and soft log with the same instructions, the owner's
// for event e and the helper's for e + 1, and the owner runs both events' state-dependent steps. (Round 5's lane
// quads, four lanes per replicate, were slower at every shard size and are gone, VERDICT r05 #7.)
template <bool BD, int SEG, int NG, bool C32, int BLK, int TF, int SCH, bool PAIR = false>
__global__ void __launch_bounds__(BLK, SCH == 2 ? 4 : 1) ssa_stepper_bins(const StepperArgs a) {
    using L = BinLayout<NG, C32>;
    constexpr uint32_t K = L::kK;
    __shared__ uint4 cnt_v[L::kBinVecs][BLK];  // bin counters
    __shared__ uint4 sum_v[L::kSumVecs][BLK];  // group sums
    __shared__ float2 logtab[ECDNA_LOGTAB_N];
    stage_logtab(logtab);
    const uint32_t tid = threadIdx.x;
    const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
    const PhiloxKeys rk = philox_round_keys(k0, k1);  // event blocks: round keys in VGPRs
    // the Philox blocks' XOR3 as the compiler builtin (ssa_device.hpp xor3) in the K = 64 / 256 and paired instances
    // (C4, C5 shards: waves that drain or run alone); the issue-bound K = 32 kernel (C3) keeps the asm form
    constexpr bool kB3 = NG >= 8 || PAIR;
    PhiloxEventPre pre{0u, 0u, 0u, 0u};  // the replicate-only part of rounds 0 and 1
    PATH_STATS_DECL;
    const uint32_t stop32 = a.stop_cells < 0xffffffffull ? (uint32_t)a.stop_cells : 0xffffffffu;
    // PAIR: a helper serves lane - 32 and never owns a replicate
    const bool helper = PAIR && (threadIdx.x & 63u) >= 32u;
    // the large-k row capacity, held in a VGPR for the event path's one compare (left to the compiler, the event
    // loop's SGPR pressure had it reloaded from the kernel arguments in every iteration, with an lgkmcnt(0) wait
    // that also drained the wave's outstanding LDS reads)
    uint32_t big_cap_v = a.big_cap;
    asm volatile("" : "+v"(big_cap_v));

    // packed counter add: bin b (0-based, copy number b + 1) / group g, by +d (d = +1, -1 or 0, as a
    // two's complement 32-bit word: a 16-bit field never borrows from its neighbour because it is >= 1
    // when decremented)
    // 32-bit word index (u32 math: LDS addresses stay 32-bit) of bin b / group g in the [vector][lane]
    // layout: vector b / kPerVec, word (b % kPerVec) / (counters per word). Indices are masked to their
    // range (b < K, g < NG) so the vector term folds away where it is constant.
    // u32 counters (C32) use the planar layout instead: counter b of a lane at word b * BLK + lane, so
    // an update is one shifted add off a per-lane base and the wave's 4-B atomics hit 64 consecutive
    // words (no bank conflicts); the scans read single words at immediate offsets.
    uint32_t* const cnt_w = reinterpret_cast<uint32_t*>(&cnt_v[0][0]);
    uint32_t* const sum_w = reinterpret_cast<uint32_t*>(&sum_v[0][0]);
    const uint32_t lane4 = tid * 4u;
    auto word_index = [&](uint32_t b) -> uint32_t {
        return C32 ? b * (uint32_t)BLK + tid : (b >> 3) * (BLK * 4u) + lane4 + ((b >> 1) & 3u);
    };
    auto bin_word = [&](uint32_t b) -> uint32_t* { return cnt_w + word_index(b); };
    auto shifted = [&](uint32_t idx, uint32_t d) -> uint32_t { return C32 ? d : (d << ((idx & 1u) * 16)); };
    // bin of copy number k (1..K) += d (d in {1, 0xffffffff, 0}); unconditional LDS atomics, so lanes
    // with nothing to change add 0 instead of branching
    auto bin_add = [&](uint32_t k, uint32_t d) {
        const uint32_t b = (k - 1u) & (K - 1u), g = (b >> 3) & (uint32_t)(NG - 1);
        atomicAdd(cnt_w + word_index(b), shifted(b, d));
        atomicAdd(sum_w + word_index(g), shifted(g, d));
    };
    // the event's three counter updates (C32, planar, 256-lane workgroups): the copy number clamped into 1..K
    // (one v_med3; a lane adding 0 may pass any value, and its add of 0 to some counter of its own changes
    // nothing), the bin's byte offset kc * 1024 + 4 tid - 1024 (one v_lshl_add) and the group sum's from it,
    // (offset >> 13) * 1024 + 4 tid, since offset >> 13 = (kc - 1) >> 3 while 4 tid < 1024: five VALU per update
    // with the select of d, against seven for bin_add's masked indices. Same counters, same adds.
    // K = 64 / u16 ([vector][lane], 256 lanes): with b2 = 2 (kc - 1) and gm = b2 & 0x70 (bit 4 = the group's
    // parity), bin b sits at byte (gm << 8) | (b2 & 12) | 16 tid in half b & 1, its group at byte
    // ((gm >> 3) & 12) | 16 tid in half (b >> 3) & 1; the shifts into the half take b2 << 3 and gm as amounts,
    // of which the VALU reads the low five bits (shl_lo5): eleven VALU per update with the select of d, against
    // thirteen for bin_add's masked indices. Same counters, same adds.
    const uint32_t bin_c = 4u * tid - 4u * BLK, sum_c = 4u * tid, lane16 = 16u * tid;
    auto bin_add_ev = [&](uint32_t k, uint32_t d) {
        if (!C32 && BLK == 256 && NG == 8) {
            const uint32_t kc = min(max(k, 1u), K);
            const uint32_t b2 = 2u * kc - 2u;
            const uint32_t gm = b2 & 0x70u;
            const uint32_t boff = lshl_or(gm, 8u, and_or(b2, 12u, lane16));
            const uint32_t goff = (__builtin_amdgcn_ubfe(b2, 5u, 2u) << 2) + lane16;
            atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(cnt_w) + boff), shl_lo5(d, b2 << 3));
            atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(sum_w) + goff), shl_lo5(d, gm));
            return;
        }
        if (!C32 || BLK != 256) {
            bin_add(k, d);
            return;
        }
        const uint32_t kc = min(max(k, 1u), K);
        const uint32_t off = (kc << 10) + bin_c;
        atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(cnt_w) + off), d);
        uint32_t g = off >> 13;
        asm("" : "+v"(g));  // (keeps shift-then-v_lshl_add: the compiler would re-form it as shift, mask and add)
        atomicAdd(reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(sum_w) + ((g << 10) + sum_c)), d);
    };
    // canonical position i -> copy number, valid for i < ns (other lanes get an unused in-range value).
    // Branch-free subtract/shift form (the compiler's compare + select form took ~40 % more VALU): with
    // d_j = i - (prefix sum through group j), the group is the number of d_j >= 0 and the offset inside
    // it is the smallest such d_j, i.e. the unsigned minimum over {i, d_j} (a negative d_j wraps above
    // every valid i). The same for the 8 bins of the group. Counts stay below 2^31.
    auto bin_find = [&](uint32_t i) -> uint32_t {
        uint32_t d = i, r = i, neg = 0;
        if (C32) {
#pragma unroll
            for (int j = 0; j < NG - 1; ++j) {  // the last group closes the scan
                d -= sum_w[j * BLK + tid];
                neg += d >> 31;
                r = min(r, d);
            }
            const uint32_t g = (uint32_t)(NG - 1) - neg;
            const uint32_t* grp = cnt_w + g * (8u * BLK) + tid;
            uint32_t d2 = r, neg2 = 0;
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                d2 -= grp[j * BLK];
                neg2 += d2 >> 31;
            }
            return g * 8u + (7u - neg2) + 1u;
        }
#pragma unroll
        for (int v = 0; v < L::kSumVecs; ++v) {
            const uint4 sv = sum_v[v][tid];
#pragma unroll
            for (int j = 0; j < L::kPerVec; ++j) {
                if (v * L::kPerVec + j >= NG - 1) break;  // the last group closes the scan
                d -= vec_get<C32>(sv, j);
                neg += d >> 31;
                r = min(r, d);
            }
        }
        const uint32_t g = (uint32_t)(NG - 1) - neg;
        uint32_t d2 = r, neg2 = 0;
#pragma unroll
        for (int v = 0; v < L::kGroupVecs; ++v) {
            const uint4 cv = cnt_v[g * L::kGroupVecs + v][tid];
#pragma unroll
            for (int j = 0; j < L::kPerVec; ++j) {
                if (v * L::kPerVec + j >= 7) break;
                d2 -= vec_get<C32>(cv, j);
                neg2 += d2 >> 31;
            }
        }
        return g * 8u + (7u - neg2) + 1u;
    };
    auto bins_zero = [&]() {
        if (C32) {
#pragma unroll 8
            for (uint32_t b = 0; b < K; ++b) cnt_w[b * BLK + tid] = 0u;
#pragma unroll
            for (uint32_t g = 0; g < (uint32_t)NG; ++g) sum_w[g * BLK + tid] = 0u;
            return;
        }
#pragma unroll
        for (int v = 0; v < L::kBinVecs; ++v) cnt_v[v][tid] = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int v = 0; v < L::kSumVecs; ++v) sum_v[v][tid] = make_uint4(0, 0, 0, 0);
    };
    // canonical row (bins ascending, then B) -> dst; B lives at row[0, nb)
    auto expand = [&](uint16_t* dst, const uint16_t* big, uint32_t nb) {  // rare path: keep it a plain loop
        uint32_t pos = 0;
#pragma unroll 1
        for (uint32_t b = 0; b < K; ++b) {
            const uint32_t c = C32 ? *bin_word(b) : ((*bin_word(b) >> ((b & 1u) * 16)) & 0xffffu);
#pragma unroll 1
            for (uint32_t q = 0; q < c; ++q) dst[pos++] = (uint16_t)(b + 1u);
        }
#pragma unroll 1
        for (uint32_t j = 0; j < nb; ++j) dst[pos + j] = (uint16_t)gload_u16_l2(big + j);
    };

    // TF: 0 = f64 time, no event hash and no snapshots (compile-time), 1 = all three from the runtime arguments
    const bool f32t = TF ? (a.flags & ECDNA_FLAG_TIME_F32) != 0 : false;
    const bool hash_on = TF ? (a.flags & ECDNA_FLAG_EVENT_HASH) != 0 : false;
    const uint32_t n_snap = TF ? a.n_snap : 0u;

    // Drain control (speed only; results depend on replicate ids alone): a SIMD's arbiter favours its
    // older waves, so a replicate started near the end on the youngest wave runs 2-3x
    // longer than on the oldest. The youngest wave slot(s) of each SIMD (HW_ID wave id >= admit_slot)
    // stops taking fresh replicates once fewer than admit_remaining are left.
    unsigned hw_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    const bool young = (hw_id & 15u) >= a.admit_slot;  // (0xffffffff: off)
    bool active = false, have = false;
    uint32_t li = 0;
    uint64_t rid = 0;
    uint16_t* row = a.rows;
    uint32_t nm = 0, ns = 0, nb = 0;
    uint32_t sp0 = 0, sp1 = 0, nsp = 0;                 // spare stream words (draw mapping v3)
    float rb0 = 0.f, rb1 = 0.f, rd0 = 0.f, rd1 = 0.f;  // the replicate's rates
    double t = 0.0;
    float t32 = 0.f;
    // Per-type event counts: only DeathNMinus (BD) and uneven splits are counted per event; the other
    // three follow at the end from the event total and the population changes (src/proliferation.rs:
    // an even split adds one N+ cell, an uneven one none (plus an N- cell unless NoNminus), a death
    // removes one): dnp = pp - un - dp, dnm = pm - dm + un(with an N- daughter), e = pm + pp + dm + dp.
    uint32_t e = 0, n_dm = 0, n_un = 0, np0 = 0, nm0 = 0;
    uint64_t h = kFnvOffset;
    uint32_t stop = 0, err = 0;
    uint32_t sj = 0;

    // bin counters of the lane's replicate -> bags[li] (final, or parked); B stays in the row
    auto store_bag = [&]() {
        uint4* bag = reinterpret_cast<uint4*>(rare_args()->bags) + (uint64_t)li * L::kBinVecs;
        if (C32) {
#pragma unroll 8
            for (uint32_t v = 0; v < (uint32_t)L::kBinVecs; ++v) {
                const uint32_t* c = cnt_w + 4u * v * BLK + tid;
                bag[v] = make_uint4(c[0], c[BLK], c[2 * BLK], c[3 * BLK]);
            }
        } else {
#pragma unroll
            for (int v = 0; v < L::kBinVecs; ++v) bag[v] = cnt_v[v][tid];
        }
    };

    // Replicate rotation (a.rot_parts != nullptr): every 2^rot_tick_log2 loop iterations
    // (a wave-uniform tick) the wave parks its lanes' replicates if enough others of its XCD's partition
    // wait, and the lanes claim waiting ones in the partition's round-robin item order. A lane whose
    // partition has nothing left takes fresh replicates of other partitions and runs them to their end
    // without parking ("pinned": their state never crosses an XCD).
    const bool rot = a.rot_parts != nullptr;  // (kept: the tick test reads it every iteration)
    unsigned xcc_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    const uint32_t part = xcc_id % kRotParts;
    const uint32_t tick_mask = rot ? ((1u << a.rot_tick_log2) - 1u) : 0xffffffffu;
    uint32_t it = 0;
    bool pinned = false;
    // N- fast-forward: the entry test's countdown (wave-uniform: three scalar instructions per iteration, where a mask of
    // an iteration counter or-ed with the mode took eight) and the wave's mode
    uint32_t ff_cd = ECDNA_FF_TEST_EVERY;
    bool ff_mode = false;

#ifdef ECDNA_ROT_STATS
    unsigned long long c_tick = 0, c_bound = 0, c_start = clock64();
#endif
    // PAIR: the loop is wave-uniform. A lane with nothing left to claim (and every helper, which owns no replicate)
    // is `done` and idles under EXEC; the wave leaves when the ballot of lanes not done is empty, so a helper can
    // never leave while its owner still runs (the owners' liveness is explicit, not read from EXEC). Without PAIR a
    // lane leaves the loop as soon as it has nothing left (done stays false and folds away).
    bool done = PAIR && helper;
    CYC_DECL;
    for (;;) {
        CYC_MARK(2);
        CYC_ADD(3, 1);
        if (rot && ((++it & tick_mask) == 0u)) {  // ---- rotation tick (wave-uniform)
#ifdef ECDNA_ROT_STATS
            const unsigned long long c0 = clock64();
#endif
            KArgs* const ra = rare_args();
            RotPart* P = ra->rot_parts + part;
            const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
            int w = 0;
            if (lane == __builtin_amdgcn_readfirstlane(lane)) w = atomic_read(&P->waiting);
            w = __builtin_amdgcn_readfirstlane(w);
            ROT_STAT(w >= ra->rot_park_min ? 5 : 6, 1);
            if (w >= ra->rot_park_min) {
                const bool pk = active && !pinned;
                if (pk) {
                    store_bag();
                    uint4* q = ra->rot_park + (uint64_t)li * kParkVecs;
                    q[0] = make_uint4(nm, ns, nb, e);
                    q[1] = make_uint4(sp0, sp1, nsp, sj);
                    q[2] = make_uint4(n_dm, n_un, np0, nm0);
                    const uint64_t tb = f32t ? (uint64_t)__float_as_uint(t32) : (uint64_t)__double_as_longlong(t);
                    q[3] = make_uint4((uint32_t)tb, (uint32_t)(tb >> 32), (uint32_t)h, (uint32_t)(h >> 32));
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the state is in the XCD's L2
                if (pk) {
                    __hip_atomic_fetch_add(&P->waiting, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // counted before it can be claimed
                    rot_set(ra->rot_flags, li, ROT_PARKED);
                    ROT_STAT(0, 1);
                    active = false;
                    have = false;
                }
            }
#ifdef ECDNA_ROT_STATS
            c_tick += clock64() - c0;
#endif
        }
#ifdef ECDNA_ROT_STATS
        const unsigned long long cb0 = clock64();
        const bool any_bound = __builtin_amdgcn_read_exec() & __ballot(!active);
#endif
        // (a PAIR helper claims nothing: it skips the boundary and takes part in the fast-forward steps below)
        if (!active && !done) {  // ---- replicate boundary (rare): write the finished one, pull the next
            PATH_STAT(2);
            KArgs* const ra = rare_args();
            if (have) {
                store_bag();
                ecdna_rep_summary_t* s = ra->summaries + li;
                s->nminus = nm;
                s->nplus = ns + nb;
                s->iters = e;
                {
                    const uint32_t un1 = SEG == ECDNA_SEG_BINOMIAL_NO_NMINUS ? 0u : n_un;  // uneven with an N- daughter
                    const uint32_t n_pm = nm - nm0 + n_dm - un1;                          // (mod 2^32)
                    const uint32_t pp_minus_dp = (ns + nb) - np0 + n_un;
                    const uint32_t pp_plus_dp = e - n_pm - n_dm;
                    const uint32_t n_pp = (pp_plus_dp + pp_minus_dp) >> 1;
                    s->events_by_type[0] = n_pm;
                    s->events_by_type[1] = n_pp;
                    s->events_by_type[2] = n_dm;
                    s->events_by_type[3] = pp_plus_dp - n_pp;
                    s->uneven = n_un;
                }
                s->time = f32t ? (double)t32 : t;
                s->event_hash = hash_on ? h : 0ull;
                s->stop_reason = stop;
                s->error = err;
                if (rot) rot_set(ra->rot_flags, li, ROT_DONE);
                have = false;
            }
            uint32_t i = 0, kind = ROT_FRESH + 1u;
            if (rot) {
                kind = rot_claim(ra, part, false, i);
                pinned = false;
#pragma unroll 1
                for (uint32_t d = 1; kind == 0u && d < kRotParts; ++d) {  // own partition drained: steal fresh
                    kind = rot_claim(ra, (part + d) % kRotParts, true, i);
                    pinned = kind != 0u;
                }
                if (kind == 0u) {
                    if (!PAIR) break;
                    done = true;
                }
            } else if (young && __hip_atomic_load(ra->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
                                        ra->admit_remaining >= ra->n) {
                if (!PAIR) break;
                done = true;
            } else {
                i = atomicAdd(ra->head, 1u);
                if (i >= ra->n) {
                    if (!PAIR) break;
                    done = true;
                } else if (ra->order) {
                    i = ra->order[i];
                }
            }
            if (!done) {  // a replicate claimed
            have = true;
            active = true;
            li = i;
            rid = ra->rid0 + (uint64_t)i * ra->rid_stride;
            pre = philox_event_pre((uint32_t)rid, (uint32_t)(rid >> 32), rk);
            row = ra->rows + (uint64_t)i * ra->row_stride;
            const uint64_t set = rid / ra->reps_per_set;
            const float4 r = ra->rates[set];
            rb0 = r.x;
            rb1 = r.y;
            rd0 = r.z;
            rd1 = r.w;
            stop = 0;
            err = 0;
            if (kind == ROT_PARKED + 1u) {  // resume: the parker's stores, through the XCD's L2
                const uint32_t bag_bytes = (uint32_t)(L::kBinVecs * 16);
#pragma unroll 1
                for (uint32_t v = 0; v < (uint32_t)L::kBinVecs; ++v) {
                    const uint4 c = ld_l2_b128(ra->bags, i * bag_bytes + v * 16u);
                    if (C32) {
                        uint32_t* d = cnt_w + 4u * v * BLK + tid;
                        d[0] = c.x;
                        d[BLK] = c.y;
                        d[2 * BLK] = c.z;
                        d[3 * BLK] = c.w;
                    } else {
                        cnt_v[v][tid] = c;
                    }
                }
                if (C32) {
#pragma unroll 1
                    for (uint32_t g = 0; g < (uint32_t)NG; ++g) {
                        uint32_t sg = 0;
#pragma unroll
                        for (uint32_t b = 0; b < 8u; ++b) sg += cnt_w[(8u * g + b) * BLK + tid];
                        sum_w[g * BLK + tid] = sg;
                    }
                } else {
#pragma unroll
                    for (int v = 0; v < L::kSumVecs; ++v) sum_v[v][tid] = make_uint4(0, 0, 0, 0);
#pragma unroll 1
                    for (uint32_t g = 0; g < (uint32_t)NG; ++g) {
                        uint32_t sg = 0;
#pragma unroll
                        for (uint32_t b = 8u * g; b < 8u * g + 8u; ++b) sg += (*bin_word(b) >> ((b & 1u) * 16)) & 0xffffu;
                        atomicAdd(sum_w + word_index(g), shifted(g, sg));
                    }
                }
                const uint32_t pb = i * (uint32_t)(kParkVecs * 16);
                const uint4 q0 = ld_l2_b128(ra->rot_park, pb), q1 = ld_l2_b128(ra->rot_park, pb + 16u);
                const uint4 q2 = ld_l2_b128(ra->rot_park, pb + 32u), q3 = ld_l2_b128(ra->rot_park, pb + 48u);
                nm = q0.x;
                ns = q0.y;
                nb = q0.z;
                e = q0.w;
                sp0 = q1.x;
                sp1 = q1.y;
                nsp = q1.z;
                sj = q1.w;
                n_dm = q2.x;
                n_un = q2.y;
                np0 = q2.z;
                nm0 = q2.w;
                const uint64_t tb = (uint64_t)q3.x | ((uint64_t)q3.y << 32);
                t = f32t ? 0.0 : __longlong_as_double((long long)tb);
                t32 = f32t ? __uint_as_float((uint32_t)tb) : 0.f;
                h = (uint64_t)q3.z | ((uint64_t)q3.w << 32);
            } else {
                const uint16_t* src = ra->init_copies;
                uint32_t cnt = ra->init_nplus;
                if (ra->init_offsets) {
                    src = ra->init_copies + ra->init_offsets[set];
                    cnt = ra->init_offsets[set + 1] - ra->init_offsets[set];
                }
                bins_zero();
                ns = 0;
                nb = 0;
#pragma unroll 1
                for (uint32_t j = 0; j < cnt; ++j) {
                    const uint32_t kk = src[j];
                    if (kk <= K) {
                        bin_add(kk, 1u);
                        ++ns;
                    } else {
                        row[nb++] = (uint16_t)kk;
                    }
                }
                nm = (uint32_t)(ra->init_nminus_set ? ra->init_nminus_set[set] : ra->init_nminus);
                t = 0.0;
                t32 = 0.f;
                e = n_dm = n_un = 0;
                np0 = ns + nb;
                nm0 = nm;
                nsp = 0;
                h = kFnvOffset;
                sj = 0;
                // ensure!(!distribution.is_empty()) src/process.rs:88, 232: the error is recorded here and the replicate
                // stops at this iteration's stop test (a0 = 0 there; the reason follows err), so that every lane that
                // reaches the event path without PAIR holds a replicate and the path needs no skip branch
                if (ns + nb == 0 && nm == 0) err = ECDNA_REP_ERR_EMPTY;
            }
            }  // (a replicate claimed)
        }
        if (PAIR && __builtin_amdgcn_ballot_w64(!done) == 0u) break;  // every lane of the wave done (wave-uniform)
#ifdef ECDNA_ROT_STATS
        if (any_bound) c_bound += clock64() - cb0;
#endif
        CYC_MARK(0);
        // ---- N- fast-forward (birth-death; DESIGN.md §5 "N- fast-forward"): an N- event
        // (ProliferateNMinus, DeathNMinus) picks no cell, so its exact work is the propensities, the stop
        // checks, the block, the channel, the time step and the n- / spare / count / hash updates. While
        // most of the wave's lanes draw N- events, they run them here, up to kFfMax per iteration, without
        // the pick, the segregation and the counter updates. A lane leaves at its first N+ event or stop
        // condition, untouched: the full event below draws that same event. Snapshots (checked per
        // event) keep the full loop. The entry test runs every 32nd iteration (ECDNA_FF_TEST_EVERY) while the wave is not
        // fast-forwarding, every iteration while it is (wave-uniform control: ballots at the loop top).
        if (BD && kFfMax && !n_snap && --ff_cd == 0u) {
            const uint32_t npf = ns + nb;  // n+ is fixed during N- events
            const float fpf = (float)npf;
            const double pbf = (double)(rb1 * fpf), pdf = (double)(rd1 * fpf);
            const float pm = rb0 * (float)nm + rd0 * (float)nm;
            const bool heavy = active && pm * 8.0f >= (pm + (float)pbf + (float)pdf) * (float)ECDNA_FF_ENTER8;  // (speed only)
            const uint32_t n_in = (uint32_t)__builtin_popcountll(__ballot(active));
            ff_mode = n_in != 0u && (uint32_t)__builtin_popcountll(__ballot(heavy)) * 8u >= n_in * ECDNA_FF_ENTER8;
            ff_cd = ff_mode ? 1u : ECDNA_FF_TEST_EVERY;
            CYC_ADD(4, ff_mode ? 1u : 0u);
            if (PAIR && ff_mode) {
                // Paired steps (DESIGN.md §5 "Paired lanes"): every lane forms one Philox block and soft log with
                // the same instructions, the owner (lane l) for its event e, the helper (lane l + 32) for the
                // owner's e + 1 from the owner's replicate-only round-0 and round-1 words; the owner pulls the helper's
                // words (v_permlane32_swap) and runs the state-dependent part of e, then of e + 1. Same draws, same
                // arithmetic, same order as the unpaired loop below: results are identical.
                bool go = active;
                PhiloxEventPre hp = pre;
                {
                    const auto x1k = __builtin_amdgcn_permlane32_swap(pre.x1k, pre.x1k, false, false);
                    const auto x2 = __builtin_amdgcn_permlane32_swap(pre.x2, pre.x2, false, false);
                    const auto y2k = __builtin_amdgcn_permlane32_swap(pre.y2k, pre.y2k, false, false);
                    const auto y3 = __builtin_amdgcn_permlane32_swap(pre.y3, pre.y3, false, false);
                    if (helper) hp = PhiloxEventPre{x1k[0], x2[0], y2k[0], y3[0]};  // (lanes >= 32 receive lanes < 32)
                }
                // One paired step: events e and e + 1 of the owner, branch-free. Both events' propensities,
                // stop tests and channels are formed from the state as it would be after e (e + 1 reads n-
                // after e's channel and the time after e's step), and each is committed by a select: e when it
                // is an N- event that passes the stop tests, e + 1 when e was committed and e + 1 passes too;
                // the first event not committed ends the lane's fast-forward, untouched, as in the unpaired
                // loop (the full event below draws it). The step is one basic block, and the next step's Philox
                // blocks and soft-log table loads are issued ahead, while this step's events run (used only if
                // both events commit; otherwise the lane has left). A lone wave pays roughly its instruction
                // count here (forming e + 1 for both possible n- alongside e, to cut the chain, was slower).
                // (one Philox instruction stream for both halves: the counter and the replicate words are selected
                // per lane; two philox_event calls under a per-lane select would run both streams on every lane)
                // ctr: the lane's event counter, e for an owner and its owner's e + 1 for a helper; a step that
                // continues advances both by 2 (a lane that commits fewer leaves, and its next words go unused)
                uint32_t ctr = __builtin_amdgcn_permlane32_swap(e, e, false, false)[0] + 1u;
                ctr = helper ? ctr : e;
                uint4 wb = philox_event<kB3>(ctr, hp, rk);
                SoftlogParts lp = softlog_begin(wb.x, logtab);  // (finished at the top of the step that uses it)
#pragma unroll 1
                for (uint32_t q = 0; q < kFfMax; q += 2) {
                    if ((uint32_t)__builtin_popcountll(__ballot(go)) * 8u < n_in * ECDNA_FF_STAY8) break;  // (uniform)
                    CYC_ADD(5, 1);
                    const float lg = softlog_end(lp);
                    // the helper's block and soft log (event e + 1) to the owner
                    const uint32_t lgb = __float_as_uint(lg);
                    const float lg2 = __uint_as_float(__builtin_amdgcn_permlane32_swap(lgb, lgb, false, false)[1]);
                    const uint32_t y2 = __builtin_amdgcn_permlane32_swap(wb.y, wb.y, false, false)[1];
                    const uint32_t z2 = __builtin_amdgcn_permlane32_swap(wb.z, wb.z, false, false)[1];
                    const uint32_t w2 = __builtin_amdgcn_permlane32_swap(wb.w, wb.w, false, false)[1];
#ifdef ECDNA_PAIR_CHECK
                    // (debug builds) the helper is still in step: its counter is the owner's e + 1. A helper that
                    // left early (EXEC at the loop top narrowed by a compiler change) would hand over stale words;
                    // counted in g_pair_check, and e + 1 is then not committed here (the full event draws it).
                    const uint32_t hctr = __builtin_amdgcn_permlane32_swap(ctr, ctr, false, false)[1];
                    const bool pair_ok = helper || hctr == e + 1u;
                    if (!pair_ok && go) __hip_atomic_fetch_add(&g_pair_check, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
                    constexpr bool pair_ok = true;
#endif
                    const uint4 wa = wb;
                    const float lga = lg;
                    // the next step's words (events e + 2, e + 3), off this step's chain
                    ctr += 2u;
                    wb = philox_event<kB3>(ctr, hp, rk);
                    lp = softlog_begin(wb.x, logtab);
                    // event e (conditions as 0/1 words combined with bitwise ops: no short-circuit branches, so
                    // the step stays one basic block for the scheduler)
                    const float fmA = (float)nm;
                    const double cAA = (double)(rb0 * fmA);
                    const double cBA = cAA + pbf;
                    const double cCA = cBA + (double)(rd0 * fmA);
                    const double AA = cCA + pdf;
                    const float a0A = (float)AA;
                    const bool overA = f32t ? (t32 >= a.max_time32) : (t >= a.max_time);
                    const double targetA = chan_target(wa.y, AA);
                    // the channel as lane masks (ProliferateNMinus !g0, DeathNMinus g1 & !g2); conditions combined
                    // with non-short-circuit & so that the step stays one basic block
                    const bool g0A = targetA >= cAA, g1A = targetA >= cBA, g2A = targetA >= cCA;
                    const bool dmA = g1A & !g2A;
                    const bool cA = go & (e < a.max_iter) & (nm + npf < stop32) & !overA & (a0A > 0.0f) & (!g0A | dmA);
                    const uint32_t nmB = nm + (g0A ? 0u : 1u) - (dmA ? 1u : 0u);
                    const float tauA = lga * rcp_rn(a0A);
                    const double tB = t + (double)tauA;
                    const float t32B = t32 + tauA;
                    // event e + 1, from the state after e
                    const float fmB = (float)nmB;
                    const double cAB = (double)(rb0 * fmB);
                    const double cBB = cAB + pbf;
                    const double cCB = cBB + (double)(rd0 * fmB);
                    const double AB = cCB + pdf;
                    const float a0B = (float)AB;
                    const bool overB = f32t ? (t32B >= a.max_time32) : (tB >= a.max_time);
                    const double targetB = chan_target(y2, AB);
                    const bool g0B = targetB >= cAB, g1B = targetB >= cBB, g2B = targetB >= cCB;
                    const bool dmB = g1B & !g2B;
                    const bool cB = cA & pair_ok & (e + 1u < a.max_iter) & (nmB + npf < stop32) & !overB & (a0B > 0.0f) &
                                    (!g0B | dmB);
                    const uint32_t nmC = nmB + (g0B ? 0u : 1u) - (dmB ? 1u : 0u);
                    const float tauB = lg2 * rcp_rn(a0B);
                    // commit. An N- event consumes no stream word after w1, so its spare update pushes w2 and
                    // w3 onto the stack and leaves exactly those two (spares_update with used = 0).
                    sp0 = cB ? w2 : (cA ? wa.w : sp0);
                    sp1 = cB ? z2 : (cA ? wa.z : sp1);
                    nsp = cA ? 2u : nsp;
                    nm = cB ? nmC : (cA ? nmB : nm);
                    n_dm += ((cA & dmA) ? 1u : 0u) + ((cB & dmB) ? 1u : 0u);
                    e += (cA ? 1u : 0u) + (cB ? 1u : 0u);
                    if (f32t)
                        t32 = cB ? t32B + tauB : (cA ? t32B : t32);
                    else
                        t = cB ? tB + (double)tauB : (cA ? tB : t);
                    if (hash_on) {
                        const uint64_t chA = (uint64_t)g0A + (uint64_t)g1A + (uint64_t)g2A;
                        const uint64_t chB = (uint64_t)g0B + (uint64_t)g1B + (uint64_t)g2B;
                        const uint64_t hA = (h ^ chA) * kFnvPrime;
                        const uint64_t hB = (hA ^ chB) * kFnvPrime;
                        h = cB ? hB : (cA ? hA : h);
                    }
                    go = cB;
                }
            } else if (ff_mode) {
                bool go = active;
#pragma unroll 1
                for (uint32_t q = 0; q < kFfMax; ++q) {
                    if ((uint32_t)__builtin_popcountll(__ballot(go)) * 8u < n_in * ECDNA_FF_STAY8) break;  // (uniform)
                    CYC_ADD(5, 1);
                    if (go) {
                        const float fm2 = (float)nm;
                        const double cA2 = (double)(rb0 * fm2);
                        const double cB2 = cA2 + pbf;
                        const double cC2 = cB2 + (double)(rd0 * fm2);
                        const double A2 = cC2 + pdf;
                        const float a02 = (float)A2;
                        const bool t_over2 = f32t ? (t32 >= a.max_time32) : (t >= a.max_time);
                        if ((e >= a.max_iter) || nm + npf >= stop32 || t_over2 || !(a02 > 0.0f)) {
                            go = false;
                        } else {
                            const uint4 w2 = philox_event<kB3>(e, pre, rk);
                            const double target2 = chan_target(w2.y, A2);
                            // the channel as lane masks: ProliferateNMinus !g0, DeathNMinus g1 & !g2
                            const bool g0 = target2 >= cA2, g1 = target2 >= cB2, g2 = target2 >= cC2;
                            const bool dm = g1 & !g2;
                            if (g0 & !dm) {  // an N+ event: the full event draws it
                                go = false;
                            } else {
                                const float tau2 = softlog_neg(w2.x, logtab) * rcp_rn(a02);
                                spares_update(0u, w2.z, w2.w, sp0, sp1, nsp);
                                nm = nm + (g0 ? 0u : 1u) - (dm ? 1u : 0u);
                                n_dm += dm ? 1u : 0u;
                                e += 1;
                                if (f32t)
                                    t32 = t32 + tau2;
                                else
                                    t = t + (double)tau2;
                                if (hash_on) h = (h ^ ((uint64_t)g0 + (uint64_t)g1 + (uint64_t)g2)) * kFnvPrime;
                            }
                        }
                    }
                }
            }
        }
        CYC_MARK(1);
        CYC_ADD(6, __builtin_popcountll(__ballot(active)));
        if (PAIR && !active) continue;  // (a helper, or an owner with nothing left)
        PATH_STAT(0);
        PATH_STAT_LANES(1);
        const uint32_t np = ns + nb;

        // propensities rate_i * population_i over [n-, n+(, n-, n+)] in f32 (the reference's own, src/main.rs:67, 139),
        // their cumulative sums in f64 (draw mapping v7); the time step divides by a0 = RN32(A)
        // (the four f32 products as two v_pk_mul_f32 of the rate pairs (b-, b+) and (d-, d+) by (n-, n+): the same
        // IEEE products)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const f32x2 pops = {(float)nm, (float)np};
        const f32x2 rbv = {rb0, rb1}, rdv = {rd0, rd1};
        const f32x2 pb = rbv * pops;
        const double cA = (double)pb.x;
        const double cB = cA + (double)pb.y;
        double cC = cB, A = cB;
        if (BD) {
            const f32x2 pd = rdv * pops;
            cC = cB + (double)pd.x;
            A = cC + (double)pd.y;
        }
        const float a0 = (float)A;
        // stop checks: one test here, the reason only when a lane stops
        const bool t_over = f32t ? (t32 >= a.max_time32) : (t >= a.max_time);
        const bool cells_over = nm + np >= stop32;  // (u32: cell counts stay below 2^32)
        if ((e >= a.max_iter) || cells_over || t_over || !(a0 > 0.0f)) {
            stop = err                 ? (uint32_t)ECDNA_STOP_ERROR  // (an empty initial distribution: ERR_EMPTY)
                   : (e >= a.max_iter) ? (uint32_t)ECDNA_STOP_MAX_ITER
                   : cells_over        ? (uint32_t)ECDNA_STOP_MAX_CELLS
                   : t_over            ? (uint32_t)ECDNA_STOP_MAX_TIME
                                       : (uint32_t)ECDNA_STOP_ABSORBING;
            active = false;
        } else {
            if (n_snap) {  // src/process.rs:122-145, as in ssa_stepper
                const uint64_t total = (uint64_t)nm + np;
                while (sj < n_snap) {
                    bool any = false;
                    for (uint32_t q = 0; q < n_snap; ++q) any |= (q >= sj) && (a.snap_cells[q] == total);
                    if (!any) break;
                    ecdna_snapshot_t* m = a.snap_meta + (uint64_t)li * n_snap + sj;
                    m->time = f32t ? (double)t32 : t;
                    m->nminus = nm;
                    m->nplus = np;
                    m->taken = 1u;
                    m->reserved = 0u;
                    if (a.snap_rows) expand(a.snap_rows + ((uint64_t)li * n_snap + sj) * a.snap_stride, row, nb);
                    ++sj;
                }
            }

            CYC_MARK(8);
            const uint32_t rid_lo = (uint32_t)rid, rid_hi = (uint32_t)(rid >> 32);
            const uint4 w = philox_event<kB3>(e, pre, rk);
            // direct method: the channel is the number of cumulative propensities <= target (the first i
            // with target < c_i; the c_i are non-decreasing); (w1 + 0.5) 2^-32 times A, in f64 (chan_target)
            const double target = chan_target(w.y, A);
            // the channel as the three compares' lane masks (no integer channel on the event path; it is formed
            // only for the event hash): ProliferateNMinus !gA, ProliferateNPlus gA & !gB, DeathNMinus gB & !gC,
            // DeathNPlus gC
#ifdef ECDNA_INJECT_EMPTY_NPLUS  // (fault-injection builds only, tools/inject_check.py: an N+ event with no N+ cell)
            const bool inj = TF != 0 && np == 0u;
#else
            constexpr bool inj = false;
#endif
            const bool gA = inj || target >= cA, gB = inj || (BD && target >= cB), gC = inj || (BD && target >= cC);
            const bool prolif = gA && !gB;
            const bool death_nm = gB && !gC;
            const bool nplus_ev = prolif || gC;  // ProliferateNPlus or DeathNPlus: a cell is picked
            // the waiting time, formed here (it needs only w0 and a0): its soft-log table read and its chain of dependent
            // f32 operations then share a basic block with the pick's, whose LDS round trips they fill in a lone wave
            // (formed in the commit, behind the rare branch, it followed them)
            const float tau = softlog_neg(w.x, logtab) * rcp_rn(a0);  // (draw mapping v8)

            CYC_MARK(9);
            WordStream ws;
            ws.w2 = w.z;
            ws.w3 = w.w;
            ws.s0 = sp0;
            ws.s1 = sp1;
            ws.nsp = nsp;
            ws.e = e;
            ws.rid_lo = rid_lo;
            ws.rid_hi = rid_hi;
            ws.k0 = k0;
            ws.k1 = k1;
            ws.pos = 1;
            ws.blk_id = 0;  // (ws.blk is only read after the block it holds was generated)

            // uniform N+ cell: Lemire multiply-shift on w2; exact rejection (rare) from the stream
            uint64_t m = mul_u32_wide(w.z, np);
            uint32_t idx, k;
            bool small;
            // K = 64 / u32 in the max-ILP build (C5: the whole run and its 8-GPU shards): a large pick issues its row
            // reads and its segregation's first Philox block ahead of the bin search, so that the wave waits on the
            // row's memory latency behind that work: the picked cell's copy number, the row's tail (what swap_remove
            // moves when the picked cell leaves the row: nb is unchanged up to there) and, for a proliferation,
            // block 1 of the stream (a copy number above 64 needs more than w3 and the two spares: binomial_half's
            // first block is block 1). The same words and values as the loads and blocks they replace. (C5 whole
            // 29.3 -> 28.8 s; with u16 counters, the C4 shard, whose waves share their SIMD until the drain, lost
            // 5 %: profiles/r04p_large_pick_ahead_ab.txt)
            constexpr bool kAhead = SCH == 1 && NG == 8 && C32;
            // the largest n = 2k whose segregation the event's own words cover: w3 (32 bits) and, when there is one, the
            // first spare (64); 0 once a Lemire rejection has consumed stream words (the general path then reads on
            // from the stream position). One compare against it replaces the position and range tests.
            uint32_t seg_lim = 32u << min(nsp, 1u);
            uint32_t k_ahead = 0, tail_ahead = 0;
            bool ahead = false;
            if (SCH == 1) {
                // the max-ILP build (lone waves): one branch for both rare cases. The bins are searched with the
                // first word's index, and a lane whose Lemire test may reject redoes the pick inside the branch,
                // after its rejection loop (C2 8.1 -> 7.5 ms; the occupancy build keeps two branches: C3 +0.8 %)
                idx = (uint32_t)(m >> 32);
                small = idx < ns;
                const uint32_t idx0 = idx;
                if (kAhead) {
                    ahead = nplus_ev & !small;
                    if (ahead) {
                        k_ahead = gload_u16_l2(row + (idx - ns));
                        tail_ahead = gload_u16_l2(row + (nb - 1u));
                        if (prolif) {
                            ws.blk = philox4x32_10<kB3>(make_uint4(e, 1u, rid_lo, rid_hi), rk);
                            ws.blk_id = 1u;
                        }
                    }
                }
                k = bin_find(idx);  // (any index reads the same in-range counters; k of a large pick is replaced below)
                if (nplus_ev & (((uint32_t)m < np) | !small)) {  // Lemire rejection or the large-k row (rare)
                    if ((uint32_t)m < np) {
                        PATH_STAT(3);
                        const uint32_t thr = (0u - np) % np;
                        while ((uint32_t)m < thr) m = (uint64_t)ws.next() * np;
                        if (ws.pos != 1u) seg_lim = 0u;
                        idx = (uint32_t)(m >> 32);
                        small = idx < ns;
                        if (small) k = bin_find(idx);
                    }
                    if (!small) {
                        PATH_STAT(4);
                        k = (kAhead && ahead && idx == idx0) ? k_ahead : gload_u16_l2(row + (idx - ns));
                    }
                }
            } else {
                if (nplus_ev && (uint32_t)m < np) {
                    PATH_STAT(3);
                    const uint32_t thr = (0u - np) % np;
                    while ((uint32_t)m < thr) m = (uint64_t)ws.next() * np;
                    if (ws.pos != 1u) seg_lim = 0u;
                }
                idx = (uint32_t)(m >> 32);
                small = idx < ns;
                k = bin_find(idx);
                if (nplus_ev && !small) {  // large-k row (rare)
                    PATH_STAT(4);
                    k = gload_u16_l2(row + (idx - ns));
                }
            }

            CYC_MARK(10);
            // Exponential::increase_nplus (src/proliferation.rs:25-111): its draws and error checks
            const uint32_t n = 2u * k;
            uint32_t k1v = k;
            uint32_t un = 0;  // 0 False, 1 True, 2 TrueWithoutNMinusIncrease
            uint32_t ev_err = 0;
            if (SEG != ECDNA_SEG_DETERMINISTIC) {
                // popcount of the stream's next n bits: w3 alone (k <= 16) or w3 and the first spare (k <= 32)
                const bool fast = n <= seg_lim;
                // branch-free: the low n bits of the 64-bit word (spare0 : w3), moved to its top by one shift (the
                // value only counts where fast: 1 <= n <= 64)
                const uint64_t x64 = (((uint64_t)sp0 << 32) | w.w) << ((64u - n) & 63u);
                k1v = __popc((uint32_t)(x64 >> 32)) + __popc((uint32_t)x64);
                if (prolif && fast) ws.pos = (n + 63u) >> 5;  // 2 (w3 used) or 3 (w3 and the first spare)
                if (prolif && !fast) {  // larger copy numbers or a rejected pick: more words
                    if (k <= 32767u) {  // (larger ones stop with ECDNA_REP_ERR_OVERFLOW below)
                        PATH_STAT(5);
                        k1v = ws.binomial_half<kAhead, kB3>(n, rk);
                    }
                }
                if (SEG == ECDNA_SEG_BINOMIAL_NO_UNEVEN && prolif && (k1v == 0u || k1v == n)) {
                    // src/segregation.rs:157-174: redraw while uneven (the first draw above was try 1)
                    if (n <= 32u) {
                        bool fail = false;
                        k1v = ws.redraw_even_small<kB3>(n, 1u, kNoUnevenMaxTries, fail, rk);
                        if (fail) ev_err = ECDNA_REP_ERR_REJECTION;
                    } else {
                        uint32_t tries = 1;
                        while (k1v == 0u || k1v == n) {
                            if (tries == kNoUnevenMaxTries) {
                                ev_err = ECDNA_REP_ERR_REJECTION;
                                break;
                            }
                            k1v = ws.binomial_half<kAhead, kB3>(n, rk);
                            ++tries;
                        }
                    }
                }
                if (SEG != ECDNA_SEG_BINOMIAL_NO_UNEVEN)
                    un = (k1v == 0u || k1v == n) ? (SEG == ECDNA_SEG_BINOMIAL_NO_NMINUS ? 2u : 1u) : 0u;
            }
            CYC_MARK(11);
            // the indexing invariant (ECDNA_REP_ERR_INTERNAL, ABI v11), in the runtime-flags instances (TF = 1; the
            // bench's TF = 0 instances keep their event path): an N+ event needs an N+ cell and a pick below n+
            // (np == 0 gives idx 0). Unreachable under draw mapping v7; a broken channel would otherwise swap_remove
            // from an empty large-k row and wrap nb. Any event, death included; the oracle returns the same code.
            const bool internal = TF != 0 && nplus_ev && idx >= np;
            // the waiting time held here, before the rare branch: left free, the compiler sank it into the commit, so
            // its soft-log table load was still pending on the stop path and the loop top waited for every LDS operation
            // of the wave (lgkmcnt(0): the previous event's six counter adds) before the propensities (C2 6.3-6.4 -> 6.1-6.3 ms,
            // the C4 shard -2.5 %, C3 -0.4 %; profiles/r06ag_tau_pin_ab.txt)
            asm volatile("" ::"v"(tau));
            // daughters (none for a death): [k1, k2] on an even split, [n] on an uneven one
            const uint32_t da = (un == 0u) ? k1v : n;
            const uint32_t db = n - k1v;
            const bool has_a = prolif, has_b = prolif & (un == 0u);
            const bool sa = has_a & (da <= K), sb = has_b & (db <= K);
            // the large-k row takes part (bitwise: no short-circuit control flow on the common path)
            const bool row_ev = nplus_ev & (!small | (has_a & !sa) | (has_b & !sb));
            // The event's rare work in one branch: the error checks, the capacity checks and the large-k row's update;
            // the common path carries that branch and the commit's (apply), where it carried three (the capacity gate,
            // the error if / else, the row update inside the commit). capacity: the N+ row (cell_cap) and the large-k
            // row (big_cap <= cell_cap); after an event the large-k row holds at most np + 1 cells, so neither can
            // overflow while np + 1 <= big_cap (C3: 88.0 ms per launch without any big_cap check, 91.8 with it on every
            // event, 89.3 gated). checked_mul: a copy number above 32767 is a large picked cell, which row_ev covers.
            bool apply = true;
            if (row_ev | (np + 1u > big_cap_v) | (prolif & (ev_err != 0u)) | internal) {
                if (k > 32767u) ev_err = ECDNA_REP_ERR_OVERFLOW;  // checked_mul panic (src/proliferation.rs:63-67)
                if (np + 1u > big_cap_v) {
                    PATH_STAT(7);
                    KArgs* const ra = rare_args();
                    if (prolif && ev_err == 0u && un == 0u && np + 1u > ra->cell_cap) ev_err = ECDNA_REP_ERR_CELL_CAP;
                    const uint32_t nb_new =
                        nb - (small ? 0u : 1u) + ((has_a && !sa) ? 1u : 0u) + ((has_b && !sb) ? 1u : 0u);
                    if (prolif && ev_err == 0u && ((has_a && !sa) || (has_b && !sb)) && nb_new > ra->big_cap)
                        ev_err = ECDNA_REP_ERR_CELL_CAP;
                }
                apply = !((prolif && ev_err) || internal);
                if (!apply) {  // the event is not applied; the replicate stops
                    err = internal ? (uint32_t)ECDNA_REP_ERR_INTERNAL : ev_err;
                    stop = ECDNA_STOP_ERROR;
                    active = false;
                } else if (row_ev) {  // the large-k row (ns is the event's; the bins are updated below)
                    PATH_STAT(6);
                    uint32_t open = small ? 0xffffffffu : idx - ns;  // B slot freed by a large picked cell
                    if (has_a && !sa) {
                        if (open != 0xffffffffu) {
                            row[open] = (uint16_t)da;
                            open = 0xffffffffu;
                        } else {
                            row[nb++] = (uint16_t)da;
                        }
                    }
                    if (has_b && !sb) {
                        if (open != 0xffffffffu) {
                            row[open] = (uint16_t)db;
                            open = 0xffffffffu;
                        } else {
                            row[nb++] = (uint16_t)db;
                        }
                    }
                    if (open != 0xffffffffu) {  // swap_remove(open) from B
                        if (open != nb - 1)
                            row[open] = (uint16_t)((kAhead && ahead) ? tail_ahead : gload_u16_l2(row + nb - 1));
                        nb -= 1;
                    }
                }
            }
            CYC_MARK(12);
            if (apply) {
                CYC_MARK(13);
                // common case: every copy number involved is binned -> LDS only, no branch
                // (bin_add_ev clamps its copy number into range, so lanes adding 0 need no select)
                // (the three deltas, 0 / +1 / -1 as u32 words, also update ns: one select each)
                const uint32_t dk = (nplus_ev && small) ? 0xffffffffu : 0u, dda = sa ? 1u : 0u, ddb = sb ? 1u : 0u;
                bin_add_ev(k, dk);
                bin_add_ev(da, dda);
                bin_add_ev(db, ddb);
                ns = ns + dk + dda + ddb;
                CYC_MARK(14);
                spares_update(nplus_ev ? ws.pos : 0u, w.z, w.w, sp0, sp1, nsp);
                nm = nm + ((!gA || (prolif && un == 1u)) ? 1u : 0u) - (death_nm ? 1u : 0u);
                n_un += (prolif && un != 0u) ? 1u : 0u;
                if (BD) n_dm += death_nm ? 1u : 0u;
                e += 1;
                if (f32t)
                    t32 = t32 + tau;
                else
                    t = t + (double)tau;
                if (hash_on) {
                    const uint64_t ch = (uint64_t)gA + (uint64_t)gB + (uint64_t)gC;
                    const uint64_t x = ch | (prolif ? ((uint64_t)k1v << 2) : 0ull) |
                                       (nplus_ev ? ((uint64_t)idx << 20) : 0ull);
                    h = (h ^ x) * kFnvPrime;
                }
            }
        }
    }
    PATH_STATS_FLUSH();
    CYC_FLUSH();
#ifdef ECDNA_ROT_STATS
    if ((threadIdx.x & 63u) == 0u) {
        ROT_STAT(8, c_tick);
        ROT_STAT(9, c_bound);
        ROT_STAT(10, clock64() - c_start);
    }
#endif
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS accesses have completed
    __builtin_amdgcn_wave_barrier();
}

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__device__ __forceinline__ double wave_max(double x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = fmax(x, __shfl_xor(x, o, 64));
    return x;
}

// Histogram + totals over one chunk. Each workgroup owns a contiguous range of replicates; per
// parameter set it accumulates in LDS (u64 atomics) and flushes non-zero bins with one global
// atomic each. Rows are read 16 B (8 cells) per lane per load.
// STATS: each wave first builds its replicate's own histogram in LDS (u32 per bin), derives the
// replicate's ABC statistics from it (mean, entropy, N+ frequency, KS distance to the target CDF by
// a wave prefix scan over the bins — abc.md:38-55), then adds it to the workgroup histogram.
// BAG (bin store, ECDNA_FLAG_BIN_STORE): 0 = rows only; 1 / 2 = per-replicate u16 / u32 bin counters
// bags[q][bag_k] for copy numbers 1..bag_k, plus the large-k cells at the head of the row.
template <bool STATS, int BAG>
__global__ void __launch_bounds__(kHistBlock) ssa_hist(const HistArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
    unsigned long long* hb = lds;                // [bins]
    unsigned long long* tb = lds + a.bins;       // [16] totals words
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nw = blockDim.x >> 6;
    uint32_t* wh = reinterpret_cast<uint32_t*>(lds + a.bins + 16) + wave * a.bins;  // STATS: [bins] per wave
    const uint32_t r_begin = blockIdx.x * a.reps_per_block;
    if (r_begin >= a.n) return;
    const uint32_t r_end = min(a.n, r_begin + a.reps_per_block);
    const uint32_t last = a.bins - 1;

    uint32_t r = r_begin;
    while (r < r_end) {
        // local replicates r .. seg_end - 1 share a parameter set: ids rid0 + r * stride below set_end_rid
        const uint64_t set = (a.rid0 + (uint64_t)r * a.rid_stride) / a.reps_per_set;
        const uint64_t set_end_rid = (set + 1) * a.reps_per_set;
        const uint64_t in_set = (set_end_rid - a.rid0 + a.rid_stride - 1) / a.rid_stride;
        const uint32_t seg_end = (uint32_t)min((uint64_t)r_end, in_set);
        for (uint32_t b = tid; b < a.bins + 16; b += blockDim.x) lds[b] = 0ull;
        __syncthreads();
        for (uint32_t q = r + wave; q < seg_end; q += nw) {
            const ecdna_rep_summary_t* s = a.summaries + q;
            const uint32_t np = (uint32_t)s->nplus;
            const uint16_t* row = a.rows + (uint64_t)q * a.row_stride;
            if (STATS) {
                for (uint32_t b = lane; b < a.bins; b += 64u) wh[b] = 0u;
                wave_sync_lds();
            }
            uint64_t ksum = 0;
            uint32_t nrow = np;  // cells held in the row
            if (BAG) {
                uint32_t small = 0;
                for (uint32_t b = lane; b < a.bag_k; b += 64u) {
                    const uint64_t o = (uint64_t)q * a.bag_k + b;
                    const uint32_t cnt = BAG == 2 ? reinterpret_cast<const uint32_t*>(a.bags)[o]
                                                  : (uint32_t)reinterpret_cast<const uint16_t*>(a.bags)[o];
                    if (cnt) {
                        const uint32_t kk = b + 1u;
                        if (STATS) {
                            atomicAdd(&wh[kk < last ? kk : last], cnt);
                            ksum += (uint64_t)kk * cnt;
                        } else {
                            atomicAdd(&hb[kk < last ? kk : last], (unsigned long long)cnt);
                        }
                    }
                    small += cnt;
                }
                small = wave_sum(small);
                nrow = np >= small ? np - small : 0u;  // (never trust counters past the row)
            }
            for (uint32_t c = lane * 8u; c < nrow; c += 512u) {
                const uint4 v = *reinterpret_cast<const uint4*>(row + c);
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    if (c + (uint32_t)j < nrow) {
                        const uint32_t kk = (wv[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                        if (STATS) {
                            atomicAdd(&wh[kk < last ? kk : last], 1u);
                            ksum += kk;
                        } else {
                            atomicAdd(&hb[kk < last ? kk : last], 1ull);
                        }
                    }
                }
            }
            if (STATS) {
                if (lane == 0) atomicAdd(&wh[0], (uint32_t)s->nminus);
                wave_sync_lds();
                ksum = wave_sum(ksum);
                const uint64_t cells = s->nminus + (uint64_t)np;
                const double inv = cells ? 1.0 / (double)cells : 0.0;
                double carry = 0.0, ent = 0.0, ks = 0.0;
                for (uint32_t base = 0; base < a.bins; base += 64u) {
                    const uint32_t b = base + lane;
                    const uint32_t cnt = b < a.bins ? wh[b] : 0u;
                    if (cnt) atomicAdd(&hb[b], (unsigned long long)cnt);
                    const double p = (double)cnt * inv;
                    if (cnt) ent -= p * log(p);
                    double scan = p;  // inclusive prefix sum over the wave
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const double y = __shfl_up(scan, o, 64);
                        if ((int)lane >= o) scan += y;
                    }
                    if (a.has_target && b < a.bins) ks = fmax(ks, fabs(carry + scan - a.target_cdf[b]));
                    carry += __shfl(scan, 63, 64);
                }
                ent = wave_sum(ent);
                ks = wave_max(ks);
                if (lane == 0) {
                    ecdna_rep_stats_t st;
                    st.cells = cells;
                    st.mean = cells ? (double)ksum * inv : 0.0;
                    st.entropy = ent;
                    st.frequency = cells ? (double)np * inv : 0.0;
                    st.ks = a.has_target ? (cells ? ks : 1.0) : 0.0;
                    const double dm = fabs(st.mean - a.target_mean), de = fabs(st.entropy - a.target_entropy);
                    st.mean_rel = a.has_target ? (a.target_mean > 0.0 ? dm / a.target_mean : dm) : 0.0;
                    st.entropy_rel = a.has_target ? (a.target_entropy > 0.0 ? de / a.target_entropy : de) : 0.0;
                    st.frequency_diff = a.has_target ? fabs(st.frequency - a.target_freq) : 0.0;
                    a.stats[q] = st;
                }
            }
            if (lane == 0) {
                if (!STATS) atomicAdd(&hb[0], (unsigned long long)s->nminus);
                atomicAdd(&tb[0], 1ull);
                atomicAdd(&tb[1], (unsigned long long)s->iters);
                atomicAdd(&tb[2], (unsigned long long)s->events_by_type[0]);
                atomicAdd(&tb[3], (unsigned long long)s->events_by_type[1]);
                atomicAdd(&tb[4], (unsigned long long)s->events_by_type[2]);
                atomicAdd(&tb[5], (unsigned long long)s->events_by_type[3]);
                atomicAdd(&tb[6], (unsigned long long)s->uneven);
                atomicAdd(&tb[7], (unsigned long long)s->nminus);
                atomicAdd(&tb[8], (unsigned long long)s->nplus);
                atomicAdd(&tb[9 + (s->stop_reason < 6u ? s->stop_reason : 5u)], 1ull);
                if (s->error) atomicAdd(&tb[15], 1ull);
            }
        }
        __syncthreads();
        for (uint32_t b = tid; b < a.bins; b += blockDim.x)
            if (hb[b]) atomicAdd((unsigned long long*)&a.hist[set * a.bins + b], hb[b]);
        if (tid < 16 && tb[tid]) atomicAdd(&a.totals[set * 16 + tid], tb[tid]);
        __syncthreads();
        r = seg_end;
    }
}

// Histogram + totals of the bin store without ABC statistics (the bench's pass). One lane per replicate, 64 at a
// time per wave: a lane reads its replicate's summary and sums its counters (how many of its N+ cells are binned,
// so the rest sit at the head of its large-k row), and keeps the totals words in registers; the counters are
// added to the histogram transposed — lane j holds the running sums of bins j, j + 64, ... over the wave's
// replicates in registers, read 64 contiguous counters of one replicate per load, 16 replicates' loads in flight —
// so no two lanes ever add to the same LDS word for them; each lane walks its own replicate's large-k row (up to 64
// cells; longer ones the whole wave), 8 cells per load. Registers reach the workgroup's LDS histogram once per wave
// and parameter set. Same sums as ssa_hist<false, BAG>, which walked one replicate per wave: C3 0.64 -> 0.16 ms per
// launch, C4 (1,024 sets, both parts of the k0 split) 7.7 -> 4.5 ms (profiles/r05s_hist_ab.txt).
template <int BAG>
__global__ void __launch_bounds__(kHistBlock) ssa_hist_bags(const HistArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned long long lds[];
    unsigned long long* hb = lds;          // [bins]
    unsigned long long* tb = lds + a.bins;  // [16] totals words
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t nw = blockDim.x >> 6;
    const uint32_t r_begin = blockIdx.x * a.reps_per_block;
    if (r_begin >= a.n) return;
    const uint32_t r_end = min(a.n, r_begin + a.reps_per_block);
    const uint32_t last = a.bins - 1;
    const uint32_t bag_k = a.bag_k;  // 32, 64 or 256
    auto counter = [&](uint64_t q, uint32_t b) -> uint32_t {
        const uint64_t o = q * bag_k + b;
        return BAG == 2 ? reinterpret_cast<const uint32_t*>(a.bags)[o]
                        : (uint32_t)reinterpret_cast<const uint16_t*>(a.bags)[o];
    };

    uint32_t r = r_begin;
    while (r < r_end) {
        const uint64_t set = (a.rid0 + (uint64_t)r * a.rid_stride) / a.reps_per_set;
        const uint64_t set_end_rid = (set + 1) * a.reps_per_set;
        const uint64_t in_set = (set_end_rid - a.rid0 + a.rid_stride - 1) / a.rid_stride;
        const uint32_t seg_end = (uint32_t)min((uint64_t)r_end, in_set);
        for (uint32_t b = tid; b < a.bins + 16; b += blockDim.x) lds[b] = 0ull;
        __syncthreads();
        // totals words 0..8 per lane (replicates, iters, events_by_type[4], uneven, n-, n+); the stop reasons and
        // errors by ballot (wave-uniform counts)
        uint64_t t_rep = 0, t_it = 0, t_e0 = 0, t_e1 = 0, t_e2 = 0, t_e3 = 0, t_un = 0, t_nm = 0, t_np = 0;
        uint32_t t_stop[6] = {0, 0, 0, 0, 0, 0}, t_err = 0;
        uint64_t acc[4] = {0, 0, 0, 0};  // bins lane + 1, lane + 65, lane + 129, lane + 193
        for (uint32_t base = r + wave * 64u; base < seg_end; base += nw * 64u) {
            const uint32_t q = base + lane;
            const bool valid = q < seg_end;
            uint32_t nrow = 0, stop = 6u;
            if (valid) {
                const ecdna_rep_summary_t* s = a.summaries + q;
                const uint64_t np = s->nplus;
                t_rep += 1;
                t_it += s->iters;
                t_e0 += s->events_by_type[0];
                t_e1 += s->events_by_type[1];
                t_e2 += s->events_by_type[2];
                t_e3 += s->events_by_type[3];
                t_un += s->uneven;
                t_nm += s->nminus;
                t_np += np;
                stop = s->stop_reason < 6u ? s->stop_reason : 5u;
                if (s->error) ++t_err;  // (counted per lane, summed below)
                // its binned cells: the replicate's counters, 16 B per load (4 u32 or 8 u16 counters)
                const uint4* v = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(a.bags) +
                                                                (uint64_t)q * bag_k * (BAG == 2 ? 4u : 2u));
                uint32_t small = 0;
                for (uint32_t b = 0; b < bag_k / (BAG == 2 ? 4u : 8u); ++b) {
                    const uint4 c = v[b];
                    if (BAG == 2)
                        small += c.x + c.y + c.z + c.w;
                    else
                        small += (c.x & 0xffffu) + (c.x >> 16) + (c.y & 0xffffu) + (c.y >> 16) + (c.z & 0xffffu) +
                                 (c.z >> 16) + (c.w & 0xffffu) + (c.w >> 16);
                }
                nrow = np >= small ? (uint32_t)(np - small) : 0u;  // (never trust counters past the row)
            }
#pragma unroll
            for (uint32_t st = 0; st < 6u; ++st) t_stop[st] += (uint32_t)__builtin_popcountll(__ballot(stop == st));
            const uint32_t nq = min(64u, seg_end - base);
            for (uint32_t i0 = 0; i0 < nq; i0 += 16u) {  // the counters, transposed; 16 loads in flight per lane
#pragma unroll
                for (uint32_t m = 0; m < 4u; ++m) {
                    if (lane + 64u * m >= bag_k) continue;  // (wave-uniform for K = 64, 256)
                    uint32_t c[16];
#pragma unroll
                    for (uint32_t i = 0; i < 16u; ++i) c[i] = i0 + i < nq ? counter(base + i0 + i, lane + 64u * m) : 0u;
                    // (u64: a u32 counter holds up to cell_cap < 2^32 cells of one bin, so 16 replicates' sum can
                    // pass 2^32)
                    uint64_t sum = 0;
#pragma unroll
                    for (uint32_t i = 0; i < 16u; ++i) sum += c[i];
                    acc[m] += sum;
                }
            }
            // the large-k rows: up to 64 cells each lane walks its own replicate's, 8 cells per load; longer rows
            // (C4's k0 = 128 sets at K = 64) the whole wave, one replicate at a time
            auto add_cells = [&](uint4 v, uint32_t n_valid) {
                const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (uint32_t j = 0; j < 8u; ++j) {
                    if (j < n_valid) {
                        const uint32_t kk = (wv[j >> 1] >> ((j & 1) * 16)) & 0xffffu;
                        atomicAdd(&hb[kk < last ? kk : last], 1ull);
                    }
                }
            };
            const bool long_row = nrow > 64u;
            const uint16_t* row = a.rows + (uint64_t)q * a.row_stride;
            for (uint32_t c = 0; c < (long_row ? 0u : nrow); c += 8u)
                add_cells(*reinterpret_cast<const uint4*>(row + c), nrow - c);
            uint64_t big = __ballot(long_row);
            while (big) {
                const uint32_t i = (uint32_t)__builtin_ctzll(big);
                big &= big - 1ull;
                const uint32_t n_i = (uint32_t)__builtin_amdgcn_readlane((int)nrow, (int)i);
                const uint16_t* row_i = a.rows + (uint64_t)(base + i) * a.row_stride;
                for (uint32_t c = lane * 8u; c < n_i; c += 512u) add_cells(*reinterpret_cast<const uint4*>(row_i + c), n_i - c);
            }
        }
#pragma unroll
        for (uint32_t m = 0; m < 4u; ++m) {
            const uint32_t kk = lane + 64u * m + 1u;
            if (lane + 64u * m < bag_k && acc[m]) atomicAdd(&hb[kk < last ? kk : last], (unsigned long long)acc[m]);
        }
        t_rep = wave_sum(t_rep);
        t_it = wave_sum(t_it);
        t_e0 = wave_sum(t_e0);
        t_e1 = wave_sum(t_e1);
        t_e2 = wave_sum(t_e2);
        t_e3 = wave_sum(t_e3);
        t_un = wave_sum(t_un);
        t_nm = wave_sum(t_nm);
        t_np = wave_sum(t_np);
        t_err = wave_sum(t_err);
        if (lane == 0 && t_rep) {
            atomicAdd(&hb[0], (unsigned long long)t_nm);
            atomicAdd(&tb[0], (unsigned long long)t_rep);
            atomicAdd(&tb[1], (unsigned long long)t_it);
            atomicAdd(&tb[2], (unsigned long long)t_e0);
            atomicAdd(&tb[3], (unsigned long long)t_e1);
            atomicAdd(&tb[4], (unsigned long long)t_e2);
            atomicAdd(&tb[5], (unsigned long long)t_e3);
            atomicAdd(&tb[6], (unsigned long long)t_un);
            atomicAdd(&tb[7], (unsigned long long)t_nm);
            atomicAdd(&tb[8], (unsigned long long)t_np);
#pragma unroll
            for (uint32_t st = 0; st < 6u; ++st)
                if (t_stop[st]) atomicAdd(&tb[9 + st], (unsigned long long)t_stop[st]);
            if (t_err) atomicAdd(&tb[15], (unsigned long long)t_err);
        }
        __syncthreads();
        for (uint32_t b = tid; b < a.bins; b += blockDim.x)
            if (hb[b]) atomicAdd((unsigned long long*)&a.hist[set * a.bins + b], hb[b]);
        if (tid < 16 && tb[tid]) atomicAdd(&a.totals[set * 16 + tid], tb[tid]);
        __syncthreads();
        r = seg_end;
    }
}

// ---------------------------------------------------------------- launch

#ifndef ECDNA_ILP_BUILD
#define ECDNA_STEPPER_TABLE(BD, WIN)                                                                        \
    {(const void*)ssa_stepper<BD, 0, WIN>, (const void*)ssa_stepper<BD, 1, WIN>,                             \
     (const void*)ssa_stepper<BD, 2, WIN>, (const void*)ssa_stepper<BD, 3, WIN>}

static const void* const kStepperTable[2][2][4] = {
    {ECDNA_STEPPER_TABLE(false, false), ECDNA_STEPPER_TABLE(true, false)},
    {ECDNA_STEPPER_TABLE(false, true), ECDNA_STEPPER_TABLE(true, true)}};
#endif

// bin-store variants: [birth_death][segregation][K = 32 | 64 | 256][u16 | u32 counters]; the 256-bin
// u32 variant runs 64-lane blocks (its 72 KiB of LDS per 64 lanes); this build's schedule (SCH)
#ifdef ECDNA_ILP_BUILD
#define ECDNA_SCH 1
#else
#define ECDNA_SCH 0
#endif
#define ECDNA_BIN_SEG(BD, SEG, TF)                                                                         \
    {{(const void*)ssa_stepper_bins<BD, SEG, 4, false, kStepperBlock, TF, ECDNA_SCH>,                       \
      (const void*)ssa_stepper_bins<BD, SEG, 4, true, kStepperBlock, TF, ECDNA_SCH>},                       \
     {(const void*)ssa_stepper_bins<BD, SEG, 8, false, kStepperBlock, TF, ECDNA_SCH>,                       \
      (const void*)ssa_stepper_bins<BD, SEG, 8, true, kStepperBlock, TF, ECDNA_SCH>},                       \
     {(const void*)ssa_stepper_bins<BD, SEG, 32, false, kBinWideBlock, TF, ECDNA_SCH>,                      \
      (const void*)ssa_stepper_bins<BD, SEG, 32, true, kBinWideBlock, TF, ECDNA_SCH>}}
#define ECDNA_BIN_TABLE(BD, TF) \
    {ECDNA_BIN_SEG(BD, 0, TF), ECDNA_BIN_SEG(BD, 1, TF), ECDNA_BIN_SEG(BD, 2, TF), ECDNA_BIN_SEG(BD, 3, TF)}

// [TF: 0 = f64 time, no hash | 1 = runtime flags][birth_death][segregation][K 32 | 64 | 256][u16 | u32]
static const void* const kBinStepperTable[2][2][4][3][2] = {{ECDNA_BIN_TABLE(false, 0), ECDNA_BIN_TABLE(true, 0)},
                                                            {ECDNA_BIN_TABLE(false, 1), ECDNA_BIN_TABLE(true, 1)}};

static const void* bin_table_entry(int birth_death, int segregation, uint32_t bin_k, int c32, uint32_t flags) {
    const int tf = (flags & kRuntimeFlagMask) ? 1 : 0;
    return kBinStepperTable[tf][birth_death ? 1 : 0][segregation & 3][bin_k > 64 ? 2 : (bin_k > 32 ? 1 : 0)]
                           [c32 ? 1 : 0];
}

#ifndef ECDNA_ILP_BUILD
// K = 64 / u16 under a 128-VGPR cap (SCH = 2): [TF][birth_death][segregation]
#define ECDNA_BIN_OCC4(BD, TF)                                                                               \
    {(const void*)ssa_stepper_bins<BD, 0, 8, false, kStepperBlock, TF, 2>,                                   \
     (const void*)ssa_stepper_bins<BD, 1, 8, false, kStepperBlock, TF, 2>,                                   \
     (const void*)ssa_stepper_bins<BD, 2, 8, false, kStepperBlock, TF, 2>,                                   \
     (const void*)ssa_stepper_bins<BD, 3, 8, false, kStepperBlock, TF, 2>}
static const void* const kBinOcc4Table[2][2][4] = {{ECDNA_BIN_OCC4(false, 0), ECDNA_BIN_OCC4(true, 0)},
                                                   {ECDNA_BIN_OCC4(false, 1), ECDNA_BIN_OCC4(true, 1)}};
#endif

#ifdef ECDNA_ILP_BUILD
const void* bin_stepper_kernel_ilp(int birth_death, int segregation, uint32_t bin_k, int c32, uint32_t flags) {
    return bin_table_entry(birth_death, segregation, bin_k, c32, flags);
}

// paired lanes (PAIR = true; birth-death only, its N- fast-forward is what pairs): [TF][segregation][K = 32 / u32,
// K = 64 / u16, K = 64 / u32]
#define ECDNA_BIN_PAIR_SEG(SEG, TF)                                                                          \
    {(const void*)ssa_stepper_bins<true, SEG, 4, true, kStepperBlock, TF, ECDNA_SCH, true>,                 \
     (const void*)ssa_stepper_bins<true, SEG, 8, false, kStepperBlock, TF, ECDNA_SCH, true>,                \
     (const void*)ssa_stepper_bins<true, SEG, 8, true, kStepperBlock, TF, ECDNA_SCH, true>}
#define ECDNA_BIN_PAIR_TF(TF) \
    {ECDNA_BIN_PAIR_SEG(0, TF), ECDNA_BIN_PAIR_SEG(1, TF), ECDNA_BIN_PAIR_SEG(2, TF), ECDNA_BIN_PAIR_SEG(3, TF)}
static const void* const kBinPairTable[2][4][3] = {ECDNA_BIN_PAIR_TF(0), ECDNA_BIN_PAIR_TF(1)};

const void* bin_stepper_kernel_pair(int segregation, uint32_t bin_k, int c32, uint32_t flags) {
    const int tf = (flags & kRuntimeFlagMask) ? 1 : 0;
    if (bin_k == 32 && c32) return kBinPairTable[tf][segregation & 3][0];
    if (bin_k == 64) return kBinPairTable[tf][segregation & 3][c32 ? 2 : 1];
    return nullptr;
}
#else
const void* stepper_kernel(int birth_death, int segregation, int window) {
    return kStepperTable[window ? 1 : 0][birth_death ? 1 : 0][segregation & 3];
}

const void* bin_stepper_kernel(int birth_death, int segregation, uint32_t bin_k, int c32, uint32_t flags, int ilp) {
    if (ilp == 3) return birth_death ? bin_stepper_kernel_pair(segregation, bin_k, c32, flags) : nullptr;
    if (ilp == 2 && bin_k == 64 && !c32) {
        const int tf = (flags & kRuntimeFlagMask) ? 1 : 0;
        return kBinOcc4Table[tf][birth_death ? 1 : 0][segregation & 3];
    }
    return ilp == 1 ? bin_stepper_kernel_ilp(birth_death, segregation, bin_k, c32, flags)
                    : bin_table_entry(birth_death, segregation, bin_k, c32, flags);
}

int bin_stepper_block(uint32_t bin_k) { return bin_k > 64 ? kBinWideBlock : kStepperBlock; }

hipError_t launch_stepper(const StepperArgs& a, int birth_death, int segregation, int window, uint32_t blocks,
                          hipStream_t stream) {
    StepperArgs copy = a;
    void* args[] = {&copy};
    return hipLaunchKernel(stepper_kernel(birth_death, segregation, window), dim3(blocks), dim3(kStepperBlock), args,
                           0, stream);
}

hipError_t launch_bin_stepper(const StepperArgs& a, int birth_death, int segregation, uint32_t bin_k, int c32, int ilp,
                              uint32_t blocks, hipStream_t stream) {
    StepperArgs copy = a;
    void* args[] = {&copy};
    return hipLaunchKernel(bin_stepper_kernel(birth_death, segregation, bin_k, c32, a.flags, ilp), dim3(blocks),
                           dim3(bin_stepper_block(bin_k)), args, 0, stream);
}

hipError_t launch_hist(const HistArgs& a, uint32_t blocks, hipStream_t stream) {
    HistArgs copy = a;
    void* args[] = {&copy};
    size_t lds = (size_t)(a.bins + 16) * sizeof(unsigned long long);
    if (a.stats) lds += (size_t)(kHistBlock / 64) * a.bins * sizeof(uint32_t);  // per-wave replicate histograms
    // (the bin store without statistics: one lane per replicate, ssa_hist_bags; ECDNA_HIST_PER_WAVE=1 keeps the
    // one-replicate-per-wave pass for A/B)
    static const void* const table[2][3] = {
        {(const void*)ssa_hist<false, 0>, (const void*)ssa_hist_bags<1>, (const void*)ssa_hist_bags<2>},
        {(const void*)ssa_hist<true, 0>, (const void*)ssa_hist<true, 1>, (const void*)ssa_hist<true, 2>}};
    static const void* const per_wave[3] = {(const void*)ssa_hist<false, 0>, (const void*)ssa_hist<false, 1>,
                                            (const void*)ssa_hist<false, 2>};
    const int bag = a.bags ? (a.bag_c32 ? 2 : 1) : 0;
    static const bool keep_per_wave = [] {
        const char* e = getenv("ECDNA_HIST_PER_WAVE");
        return e && e[0] == '1';
    }();
    if (keep_per_wave && !a.stats)
        return hipLaunchKernel(per_wave[bag], dim3(blocks), dim3(kHistBlock), args, lds, stream);
    return hipLaunchKernel(table[a.stats ? 1 : 0][bag], dim3(blocks), dim3(kHistBlock), args, lds, stream);
}
#endif  // ECDNA_ILP_BUILD

}  // namespace ecdna

#if defined(ECDNA_PATH_STATS) && !defined(ECDNA_ILP_BUILD)
// Development: read (and reset) the rare-block counters of the last launches (tools/path_stats.py)
extern "C" int ecdna_dev_path_stats(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ecdna::g_path_stats), sizeof(ecdna::g_path_stats)) != hipSuccess) return -1;
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(ecdna::g_path_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef ECDNA_CYCLE_STATS
// Development: read (and reset) the loop-section cycle counters of the last launches (tools/cycle_stats.py);
// the max-ILP build's kernels count into their own copy
#ifdef ECDNA_ILP_BUILD
extern "C" int ecdna_dev_cycle_stats_ilp(unsigned long long* out) {
#else
extern "C" int ecdna_dev_cycle_stats(unsigned long long* out) {
#endif
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ecdna::ECDNA_CYC_SYM), sizeof(ecdna::ECDNA_CYC_SYM)) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(ecdna::ECDNA_CYC_SYM), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
#if defined(ECDNA_ROT_STATS) && !defined(ECDNA_ILP_BUILD)
// Development: read (and reset) the rotation counters of the last launches (tools/rot_stats.py)
extern "C" int ecdna_dev_rot_stats(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ecdna::g_rot_stats), sizeof(ecdna::g_rot_stats)) != hipSuccess) return -1;
    unsigned long long z[12] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(ecdna::g_rot_stats), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
