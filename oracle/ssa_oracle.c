/*
 * ssa_oracle.c — TEST INFRASTRUCTURE ONLY (see ssa_oracle.h): plain-C
 * restatement of the reference's per-replicate Gillespie loop, "philox" mode.
 *
 * It follows, function by function:
 *   sosa::simulate loop (external crate sosa 3.0.3, Cargo.lock:944-955; call
 *     sites src/main.rs:92-99, 166-173; Options src/clap_app.rs:202-209)
 *     -> simulate_replicate()
 *   PureBirth/BirthDeath::advance_step event dispatch + time accumulation
 *     (src/process.rs:147-184, 291-336) -> the switch in simulate_replicate()
 *   update_state population vectors (src/process.rs:187-196, 339-344)
 *     -> propensities(): [n-, n+] / [n-, n+, n-, n+]
 *   Exponential::increase_nplus (src/proliferation.rs:25-111) -> prolif_nplus()
 *   Exponential::increase_nminus (src/proliferation.rs:113-117), CellDeath
 *     (src/proliferation.rs:126-140) -> the N- cases / death_nplus()
 *   Segregate impls (src/segregation.rs:110-194) -> segregate()
 *   EcDNADistribution pick_remove_random_nplus / decrease_nplus =
 *     gen_range + swap_remove, increase_nplus = push (ecdna-lib 3.0.2,
 *     reconstructed in SURVEY.md App. A.2) -> swap_remove()/push in place
 *   rayon over replicate ids (src/main.rs:221-224) -> pthread pool with an
 *     atomic work counter (run_pool()).
 *
 * The draws follow the engine's mapping, not ChaCha8: see
 * ssa_compat.c for the reference-semantics samplers.
 *
 * Floating point: compile with -ffp-contract=off. Every f32 / f64 operation
 * below is a correctly rounded IEEE add/sub/mul/div/fma in a fixed order (the
 * propensities and time step in f32, the channel's cumulative sums and target
 * in f64, draw mapping v8: the time step a product with RN32(1 / a0); the
 * clock in f64), so the HIP kernel (which spells the same operations with
 * contraction disabled) reproduces the times and channel picks bit for bit.
 */
#include "ssa_oracle.h"
#include "ssa_logtab.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ------------------------------------------------------------------ Philox */

#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

/* Philox4x32-10 (Salmon et al., SC'11; Random123 philox4x32 with 10 rounds). */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += PHILOX_W0;
            k1 += PHILOX_W1;
        }
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

/* -------------------------------------------------------------- soft log */

/* -ln(u), u = ((w >> 9) + 0.5) * 2^-23: the engine's draw mapping (v6 and v7), in f32. d = (w >> 8) | 1
 * (odd, < 2^24: (float)d is exact) = m 2^ex with m in [0.5, 1) and u = d 2^-24; the top 7 fraction bits j of m
 * select {C, LN} = {RN32(1/mid_j), RN32(ln mid_j)} (ssa_logtab.h, tools/gen_logtab.py); r = fma(m, C, -1)
 * (|r| <= 2^-8); ln(1 + r) by a degree-4 series in explicit fmaf (C99 fmaf is the correctly rounded fused
 * operation, like v_fma_f32); -ln u = -(LN + ln(1 + r) + k ln 2), k = ex - 24, ln 2 = LN2_HI + LN2_LO with k LN2_HI
 * exact. Fixed operation order, float arithmetic only (FLT_EVAL_METHOD 0). */
static const float LOGTAB[2 * ECDNA_LOGTAB_N] = ECDNA_LOGTAB_INIT;

float oracle_softlog_neg(uint32_t w) {
    const float d = (float)((w >> 8) | 1u);
    uint32_t bits;
    memcpy(&bits, &d, sizeof bits);
    const int k = (int)(bits >> 23) - 150;
    const uint32_t mb = (bits & 0x007fffffu) | 0x3f000000u;
    float m;
    memcpy(&m, &mb, sizeof m);
    const uint32_t j = (bits >> 16) & 127u;
    const float c = LOGTAB[2 * j], ln = LOGTAB[2 * j + 1];
    const float r = fmaf(m, c, -1.0f);
    float q = fmaf(r, -0.25f, 0x1.555556p-2f); /* -1/4, RN32(1/3) */
    q = fmaf(r, q, -0.5f);
    const float l = fmaf(r * r, q, r); /* ln(1 + r) */
    const float kf = (float)k;
    return -fmaf(kf, ECDNA_LN2_HI, fmaf(kf, ECDNA_LN2_LO, ln + l));
}

void oracle_softlog_many(const uint32_t* w, uint64_t n, float* out) {
    for (uint64_t i = 0; i < n; ++i) out[i] = oracle_softlog_neg(w[i]);
}

/* The channel's target, draw mapping v7: u = (w + 0.5) 2^-32 from all 32 bits of w1 (exact in f64: one fma) times
 * the f64 total propensity A, RN64. u <= 1 - 2^-33 keeps the target below A (a zero-propensity last channel is never
 * drawn) and u >= 2^-33 keeps it above 0 (nor a zero-propensity first channel). */
static double chan_target(uint32_t w, double A) { return fma((double)w, 0x1p-32, 0x1p-33) * A; }

/* Propensities of update_state's population vector [n-, n+(, n-, n+)] (src/process.rs:187-196, 339-344) in f32, the
 * reference's own (src/main.rs:67, 139); cumulative sums c[0..2] and the total *A in f64; returns a0 = RN32(A), the
 * time step's divisor (draw mapping v7). */
static float propensities(const float rates[4], uint64_t nminus, uint64_t nplus, int bd, double c[3], double* A) {
    const float fnm = (float)nminus, fnp = (float)nplus;
    float a[4];
    a[0] = rates[0] * fnm;
    a[1] = rates[1] * fnp;
    a[2] = bd ? rates[2] * fnm : 0.0f;
    a[3] = bd ? rates[3] * fnp : 0.0f;
    c[0] = (double)a[0];
    c[1] = c[0] + (double)a[1];
    c[2] = c[1] + (double)a[2];
    *A = c[2] + (double)a[3];
    return (float)*A;
}

/* direct method: the channel is the number of cumulative propensities <= target */
static int channel_of(const double c[3], double target) {
    return target < c[0] ? 0 : (target < c[1] ? 1 : (target < c[2] ? 2 : 3));
}

int oracle_channel(const float rates[4], uint64_t nminus, uint64_t nplus, int birth_death, uint32_t w1) {
    double c[3], A;
    const float a0 = propensities(rates, nminus, nplus, birth_death, c, &A);
    if (!(a0 > 0.0f)) return -1;
    return channel_of(c, chan_target(w1, A));
}

/* ------------------------------------------------------------ word stream */

/* Per-event stream words (draw mapping v5): [w2, w3, spare[0], .., spare[nsp-1], blk1.x, blk1.y, blk1.z,
 * blk1.w, blk2.x, ...] where blk j = Philox(ctr = (e, j, rid lo, rid hi)) and the spares are words of
 * earlier events' blocks that no draw consumed, kept as a two-slot stack (newest first; spares_update()).
 * Each word is used at most once and whether it is used depends only on draws already made, so every
 * draw stays an independent uniform. pos = words consumed. */
typedef struct {
    uint32_t key[2];
    uint32_t e, rid_lo, rid_hi;
    uint32_t w2, w3;
    uint32_t sp[2];
    uint32_t nsp;
    uint32_t buf[4];
    uint32_t blk;
    uint32_t pos;
} wstream;

static uint32_t ws_next(wstream* s) {
    uint32_t p = s->pos++;
    if (p == 0) return s->w2;
    if (p == 1) return s->w3;
    if (p - 2 < s->nsp) return s->sp[p - 2];
    uint32_t q = p - 2 - s->nsp;
    uint32_t j = q / 4 + 1;
    if (j != s->blk) {
        uint32_t ctr[4] = {s->e, j, s->rid_lo, s->rid_hi};
        oracle_philox4x32_10(ctr, s->key, s->buf);
        s->blk = j;
    }
    return s->buf[q % 4];
}

/* Uniform index in [0, L), L in [1, 2^32): Lemire multiply-shift with exact rejection
 * (stands in for rand 0.8.5 gen_range(0..len)). */
static uint32_t ws_index(wstream* s, uint32_t L) {
    uint64_t m = (uint64_t)ws_next(s) * L;
    uint32_t lo = (uint32_t)m;
    if (lo < L) {
        uint32_t thr = (uint32_t)(0u - L) % L;
        while (lo < thr) {
            m = (uint64_t)ws_next(s) * L;
            lo = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

/* k1 ~ Binomial(n, 1/2) exactly: popcount of n fair bits taken from the stream. */
static uint32_t ws_binomial_half(wstream* s, uint32_t n) {
    uint32_t c = 0;
    while (n >= 32) {
        c += (uint32_t)__builtin_popcount(ws_next(s));
        n -= 32;
    }
    if (n) c += (uint32_t)__builtin_popcount(ws_next(s) & ((1u << n) - 1u));
    return c;
}

#define UNEVEN_FALSE 0
#define UNEVEN_TRUE 1
#define UNEVEN_TRUE_NO_NMINUS 2
#define NO_UNEVEN_MAX_TRIES 4096

/* Segregate::ecdna_segregation for n = 2k (src/segregation.rs:110-194). */
static int segregate(wstream* s, int seg, uint32_t n, uint32_t* k1, int* uneven) {
    switch (seg) {
        case ECDNA_SEG_DETERMINISTIC: /* k1 = k2 = n/2, IsUneven::False (src/segregation.rs:142-155) */
            *k1 = n / 2;
            *uneven = UNEVEN_FALSE;
            return 0;
        case ECDNA_SEG_BINOMIAL: { /* k1 ~ Bin(n, 1/2); uneven iff k1==0 || k2==0 (:110-140) */
            uint32_t x = ws_binomial_half(s, n);
            *k1 = x;
            *uneven = (x == 0 || x == n) ? UNEVEN_TRUE : UNEVEN_FALSE;
            return 0;
        }
        case ECDNA_SEG_BINOMIAL_NO_UNEVEN: { /* redraw while uneven (:157-174) */
            for (int t = 0; t < NO_UNEVEN_MAX_TRIES; ++t) {
                uint32_t x = ws_binomial_half(s, n);
                if (x != 0 && x != n) {
                    *k1 = x;
                    *uneven = UNEVEN_FALSE;
                    return 0;
                }
            }
            return ECDNA_REP_ERR_REJECTION;
        }
        case ECDNA_SEG_BINOMIAL_NO_NMINUS: { /* uneven relabelled (:176-194) */
            uint32_t x = ws_binomial_half(s, n);
            *k1 = x;
            *uneven = (x == 0 || x == n) ? UNEVEN_TRUE_NO_NMINUS : UNEVEN_FALSE;
            return 0;
        }
    }
    return -1;
}

/* After an event that consumed `used` stream words (mapping v5): the unused base words are pushed on a
 * two-slot stack (newest on top, the oldest falls off): w2 then w3 when used == 0, w3 when used == 1;
 * used == 2 leaves it; used >= 3 consumed used - 2 words after w3, the top spares first. (v3 kept the
 * oldest two in a list, v4 a single spare: the list cost ~15 VALU per event on the GPU, the single spare
 * sent 3.5x more events to a second Philox block.) */
static void spares_update(uint32_t sp[2], uint32_t* nsp, uint32_t used, uint32_t w2, uint32_t w3) {
    if (used == 0) {
        sp[1] = w2;
        sp[0] = w3;
        *nsp = 2;
    } else if (used == 1) {
        sp[1] = sp[0];
        sp[0] = w3;
        *nsp = *nsp + 1 > 2 ? 2 : *nsp + 1;
    } else if (used >= 3) {
        const uint32_t c = used - 2;
        if (*nsp > c) {
            sp[0] = sp[1];
            *nsp -= c;
        } else {
            *nsp = 0;
        }
    }
}

static void ws_init(wstream* s, uint64_t seed, uint64_t rid, uint32_t e, uint32_t w2, uint32_t w3) {
    s->key[0] = (uint32_t)seed;
    s->key[1] = (uint32_t)(seed >> 32);
    s->e = e;
    s->rid_lo = (uint32_t)rid;
    s->rid_hi = (uint32_t)(rid >> 32);
    s->w2 = w2;
    s->w3 = w3;
    s->nsp = 0;
    s->blk = 0;
    s->pos = 0;
}

static void event_block(uint64_t seed, uint64_t rid, uint32_t e, uint32_t w[4]) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t ctr[4] = {e, 0u, (uint32_t)rid, (uint32_t)(rid >> 32)};
    oracle_philox4x32_10(ctr, key, w);
}

/* ---------------------------------------------------------- event kernels */

/* Exponential::increase_nplus (src/proliferation.rs:25-111): pick-remove a uniform N+ cell
 * (swap_remove), double its copies (checked: src/proliferation.rs:63-67), segregate, push
 * [k1, k2] (False) or [k1+k2] (+1 N- for True). Returns 0 or an ecdna_rep_error_t; on error the
 * distribution is unchanged. */
static int prolif_nplus(uint16_t* row, uint64_t* len, uint64_t* nminus, uint64_t cap, wstream* ws,
                        int seg, uint32_t* idx_out, uint32_t* k1_out, uint32_t* k2_out, int* uneven_out) {
    uint64_t L = *len;
    uint32_t i = ws_index(ws, (uint32_t)L);
    uint32_t k = row[i];
    if (k > 32767u) return ECDNA_REP_ERR_OVERFLOW;
    uint32_t n = 2u * k;
    uint32_t k1;
    int uneven;
    int err = segregate(ws, seg, n, &k1, &uneven);
    if (err) return err;
    if (uneven == UNEVEN_FALSE && L + 1 > cap) return ECDNA_REP_ERR_CELL_CAP;
    row[i] = row[L - 1]; /* swap_remove(i) */
    L -= 1;
    if (uneven == UNEVEN_FALSE) {
        row[L++] = (uint16_t)k1;
        row[L++] = (uint16_t)(n - k1);
    } else {
        if (uneven == UNEVEN_TRUE) *nminus += 1;
        row[L++] = (uint16_t)n;
    }
    *len = L;
    *idx_out = i;
    *k1_out = k1;
    *k2_out = n - k1;
    *uneven_out = uneven;
    return 0;
}

/* CellDeath::decrease_nplus (src/proliferation.rs:126-133): gen_range + swap_remove. */
static uint32_t death_nplus(uint16_t* row, uint64_t* len, wstream* ws) {
    uint64_t L = *len;
    uint32_t i = ws_index(ws, (uint32_t)L);
    row[i] = row[L - 1];
    *len = L - 1;
    return i;
}

/* ------------------------------------------------------------ bin store */

/* The engine's BIN store (ECDNA_FLAG_BIN_STORE): the replicate's N+ cells as counts
 * c[k] of cells with k copies for k = 1..K (K = bin_kmax), plus a row B of the cells with k > K.
 * Canonical order of the N+ cells: c[1] cells of k = 1, c[2] of k = 2, ..., c[K] of k = K, then
 * B[0..nb). The uniform pick (gen_range over the cells, src/proliferation.rs:57, 132) indexes that
 * order; any fixed arrangement gives the same law, so this stands in for the Vec<u16> with
 * swap_remove of ecdna-lib 3.0.2 in distribution, not seed for seed. */
#define BIN_KMAX_MAX 256
typedef struct {
    uint32_t K;
    uint64_t c[BIN_KMAX_MAX + 1]; /* c[1..K] */
    uint64_t ns;                  /* sum of c */
    uint16_t* big;                /* B */
    uint64_t nb;
    uint64_t big_cap;             /* capacity of B (params big_cap, 0 = cell_cap) */
} binstore;

static void bins_add(binstore* b, uint32_t k) {
    if (k <= b->K) {
        b->c[k] += 1;
        b->ns += 1;
    } else {
        b->big[b->nb++] = (uint16_t)k;
    }
}

/* copy number of the cell at canonical position idx < ns + nb */
static uint32_t bins_get(const binstore* b, uint64_t idx) {
    if (idx >= b->ns) return b->big[idx - b->ns];
    uint64_t run = 0;
    for (uint32_t k = 1;; ++k) {
        run += b->c[k];
        if (idx < run) return k;
    }
}

/* Remove the picked cell (canonical position idx, copy number k) and add the daughters d[0..nd):
 * daughters with k <= K go to their bins; large ones: if the removed cell was itself in B (at j),
 * the first large daughter takes its slot j and the rest are pushed; otherwise they are all pushed
 * in order. A removed B cell with no large daughter is swap_removed from B. */
static void bins_replace(binstore* b, uint64_t idx, uint32_t k, const uint32_t* d, int nd) {
    int slot_open = 0;
    uint64_t j = 0;
    if (idx < b->ns) {
        b->c[k] -= 1;
        b->ns -= 1;
    } else {
        slot_open = 1;
        j = idx - b->ns;
    }
    for (int q = 0; q < nd; ++q) {
        if (d[q] <= b->K) {
            b->c[d[q]] += 1;
            b->ns += 1;
        } else if (slot_open) {
            b->big[j] = (uint16_t)d[q];
            slot_open = 0;
        } else {
            b->big[b->nb++] = (uint16_t)d[q];
        }
    }
    if (slot_open) { /* swap_remove(j) */
        b->big[j] = b->big[b->nb - 1];
        b->nb -= 1;
    }
}

/* canonical row of the N+ cells */
static void bins_expand(const binstore* b, uint16_t* dst) {
    uint64_t pos = 0;
    for (uint32_t k = 1; k <= b->K; ++k)
        for (uint64_t q = 0; q < b->c[k]; ++q) dst[pos++] = (uint16_t)k;
    memcpy(dst + pos, b->big, b->nb * sizeof(uint16_t));
}

/* Exponential::increase_nplus on the bin store: the same draws and checks as prolif_nplus. */
static int prolif_nplus_bins(binstore* b, uint64_t* nminus, uint64_t cap, wstream* ws, int seg,
                             uint32_t* idx_out, uint32_t* k1_out, int* uneven_out) {
    const uint64_t L = b->ns + b->nb;
    uint32_t i = ws_index(ws, (uint32_t)L);
    uint32_t k = bins_get(b, i);
    if (k > 32767u) return ECDNA_REP_ERR_OVERFLOW;
    uint32_t n = 2u * k;
    uint32_t k1;
    int uneven;
    int err = segregate(ws, seg, n, &k1, &uneven);
    if (err) return err;
    if (uneven == UNEVEN_FALSE && L + 1 > cap) return ECDNA_REP_ERR_CELL_CAP;
    { /* room for the large daughters in B (ecdna_ssa_params_t.big_cap); a removed B cell frees its slot */
        const uint64_t large = uneven == UNEVEN_FALSE ? (uint64_t)(k1 > b->K) + (uint64_t)(n - k1 > b->K)
                                                       : (uint64_t)(n > b->K);
        if (large && b->nb - (i >= b->ns ? 1u : 0u) + large > b->big_cap) return ECDNA_REP_ERR_CELL_CAP;
    }
    if (uneven == UNEVEN_FALSE) {
        uint32_t d[2] = {k1, n - k1};
        bins_replace(b, i, k, d, 2);
    } else {
        if (uneven == UNEVEN_TRUE) *nminus += 1;
        uint32_t d[1] = {n};
        bins_replace(b, i, k, d, 1);
    }
    *idx_out = i;
    *k1_out = k1;
    *uneven_out = uneven;
    return 0;
}

/* CellDeath::decrease_nplus on the bin store. */
static uint32_t death_nplus_bins(binstore* b, wstream* ws) {
    uint32_t i = ws_index(ws, (uint32_t)(b->ns + b->nb));
    bins_replace(b, i, bins_get(b, i), NULL, 0);
    return i;
}

/* -------------------------------------------------------------- one run */

typedef struct {
    const ecdna_ssa_params_t* p;
    ecdna_rep_summary_t* summaries;
    uint16_t* rows;
    uint64_t row_stride;
    atomic_ullong next;
    pthread_mutex_t mu;
    uint64_t* hist;
    ecdna_totals_t* totals;
    int compat;
    ecdna_snapshot_t* snap_meta;
    uint16_t* snap_rows;
    uint64_t* rng_words; /* compat: [n] ChaCha8 words handed out per replicate, or NULL */
} run_ctx;

#define FNV_OFFSET 0xcbf29ce484222325ull
#define FNV_PRIME 0x100000001b3ull

static inline uint64_t fnv_fold(uint64_t h, uint64_t x) { return (h ^ x) * FNV_PRIME; }

static _Thread_local ecdna_snapshot_t* tl_snap_meta = NULL;
static _Thread_local uint16_t* tl_snap_rows = NULL;

void oracle_set_snapshot_outputs(ecdna_snapshot_t* meta, uint16_t* rows) {
    tl_snap_meta = meta;
    tl_snap_rows = rows;
}

static _Thread_local uint64_t* tl_rng_words = NULL;

void oracle_set_rng_words_output(uint64_t* words) { tl_rng_words = words; }

/* The snapshot rule at the top of advance_step (src/process.rs:122-145, 267-290): while the deque is
 * non-empty and ANY remaining snapshot equals n- + n+, pop the FRONT snapshot and save the current
 * distribution (time before this event's waiting time). meta/rows: this replicate's [S] / [S][stride]
 * outputs (either may be NULL). Shared with ssa_compat.c. */
void oracle_snapshot_check(const ecdna_ssa_params_t* p, uint32_t* sj, uint64_t nminus, uint64_t nplus,
                           double time, const uint16_t* row, ecdna_snapshot_t* meta, uint16_t* rows,
                           uint64_t stride) {
    const uint64_t total = nminus + nplus;
    while (*sj < p->n_snapshots) {
        int any = 0;
        for (uint32_t q = *sj; q < p->n_snapshots; ++q) any |= p->snapshot_cells[q] == total;
        if (!any) return;
        if (meta) {
            meta[*sj].time = time;
            meta[*sj].nminus = nminus;
            meta[*sj].nplus = nplus;
            meta[*sj].taken = 1;
            meta[*sj].reserved = 0;
        }
        if (rows) memcpy(rows + (uint64_t)*sj * stride, row, nplus * sizeof(uint16_t));
        *sj += 1;
    }
}

static void init_of_set(const ecdna_ssa_params_t* p, uint64_t set, const uint16_t** copies,
                        uint64_t* nplus, uint64_t* nminus) {
    if (p->init_set_offsets) {
        *copies = p->init_copies + p->init_set_offsets[set];
        *nplus = p->init_set_offsets[set + 1] - p->init_set_offsets[set];
        *nminus = p->init_set_nminus ? p->init_set_nminus[set] : p->init_nminus;
    } else {
        *copies = p->init_copies;
        *nplus = p->init_nplus;
        *nminus = p->init_set_nminus ? p->init_set_nminus[set] : p->init_nminus;
    }
}

/* One replicate: the sosa::simulate loop around advance_step (SURVEY.md App. A.3 / DESIGN.md §3.1). */
static void simulate_replicate(const ecdna_ssa_params_t* p, uint64_t rid, uint16_t* row,
                               ecdna_rep_summary_t* out, ecdna_snapshot_t* snap_meta, uint16_t* snap_rows,
                               uint64_t snap_stride) {
    uint32_t sj = 0;
    uint32_t spare[2] = {0, 0}, nspare = 0; /* spare stream words (draw mapping v5) */
    const uint64_t set = rid / p->reps_per_set;
    const ecdna_rates_t rt = p->rates[set];
    const int bd = p->process == ECDNA_BIRTH_DEATH;
    const int f32t = (p->flags & ECDNA_FLAG_TIME_F32) != 0;
    const int hash_on = (p->flags & ECDNA_FLAG_EVENT_HASH) != 0;
    const uint64_t cells_mul = (bd && (p->flags & ECDNA_FLAG_BD_CAP_COMPAT)) ? 2u : 1u;

    const uint16_t* init;
    uint64_t nplus, nminus;
    init_of_set(p, set, &init, &nplus, &nminus);
    const int binned = (p->flags & ECDNA_FLAG_BIN_STORE) != 0;
    binstore* bs = NULL;
    uint16_t* snap_scratch = NULL;
    if (binned) {
        bs = calloc(1, sizeof(binstore));
        bs->K = p->bin_kmax ? p->bin_kmax : 64;
        bs->big_cap = (p->big_cap && p->big_cap < p->cell_cap) ? p->big_cap : p->cell_cap;
        bs->big = malloc(((size_t)p->cell_cap + 1) * sizeof(uint16_t));
        for (uint64_t j = 0; j < nplus; ++j) bins_add(bs, init[j]);
        if (snap_rows) snap_scratch = malloc(((size_t)p->cell_cap + 1) * sizeof(uint16_t));
    } else {
        memcpy(row, init, nplus * sizeof(uint16_t));
    }

    memset(out, 0, sizeof(*out));
    uint64_t h = FNV_OFFSET;
    double t = 0.0;
    float t32 = 0.0f;
    const float max_t32 = (float)p->max_time;
    uint32_t e = 0;
    uint32_t stop = ECDNA_STOP_NONE, err = ECDNA_REP_OK;
    uint64_t cnt[4] = {0, 0, 0, 0}, uneven_n = 0;

    if (nplus == 0 && nminus == 0) { /* ensure!(!distribution.is_empty()) src/process.rs:88, 232 */
        err = ECDNA_REP_ERR_EMPTY;
        stop = ECDNA_STOP_ERROR;
    }
    while (!stop) {
        if ((uint64_t)e >= p->max_iter) {
            stop = ECDNA_STOP_MAX_ITER;
            break;
        }
        if ((nminus + nplus) * cells_mul >= p->max_cells) {
            stop = ECDNA_STOP_MAX_CELLS;
            break;
        }
        if (f32t ? (t32 >= max_t32) : (t >= p->max_time)) {
            stop = ECDNA_STOP_MAX_TIME;
            break;
        }
        /* propensities rate_i * population_i, population = update_state's vector, in f32 (the reference's own,
         * src/main.rs:67, 139); their cumulative sums in f64 and the time step's total a0 = RN32(A) (draw mapping v7) */
        const float rates4[4] = {rt.b0, rt.b1, rt.d0, rt.d1};
        double c[3], A;
        const float a0 = propensities(rates4, nminus, nplus, bd, c, &A);
        if (!(a0 > 0.0f)) {
            stop = ECDNA_STOP_ABSORBING;
            break;
        }
        if (p->n_snapshots) {
            const uint16_t* cur = row;
            if (binned && snap_scratch) {
                bins_expand(bs, snap_scratch);
                cur = snap_scratch;
            }
            oracle_snapshot_check(p, &sj, nminus, nplus, f32t ? (double)t32 : t, cur, snap_meta, snap_rows,
                                  snap_stride);
        }
        uint32_t w[4];
        event_block(p->seed, rid, e, w);
        /* direct method: channel by w1 against the cumulative propensities */
        const int ch = channel_of(c, chan_target(w[1], A));
        /* an N+ event with no N+ cell: the engine's guard (ECDNA_REP_ERR_INTERNAL, ABI v11). Unreachable under draw
         * mapping v8 (a zero-propensity channel is never drawn); the reference's pick_remove_random_nplus errors on an
         * empty N+ set (src/proliferation.rs:55-57). The event is not applied. */
        if ((ch & 1) && nplus == 0) {
            err = ECDNA_REP_ERR_INTERNAL;
            stop = ECDNA_STOP_ERROR;
            continue;
        }
        /* draw mapping v8: the soft log times the correctly rounded reciprocal RN32(1 / a0) (the f64 quotient rounded
         * to f32: 1 / a0 is never within 2^-53 relative of an f32 rounding boundary, so the double rounding is
         * innocuous); the engine forms RN32(1 / a0) from v_rcp_f32 and one Newton step (ssa_device.hpp rcp_rn) */
        float tau = oracle_softlog_neg(w[0]) * (float)(1.0 / (double)a0);
        wstream ws;
        ws_init(&ws, p->seed, rid, e, w[2], w[3]);
        ws.sp[0] = spare[0];
        ws.sp[1] = spare[1];
        ws.nsp = nspare;
        uint64_t x = (uint64_t)ch;
        switch (ch) {
            case ECDNA_EV_PROLIF_NMINUS: /* increase_nminus (src/proliferation.rs:113-117) */
                nminus += 1;
                break;
            case ECDNA_EV_PROLIF_NPLUS: {
                uint32_t i, k1, k2;
                int un;
                int rc;
                if (binned) {
                    rc = prolif_nplus_bins(bs, &nminus, p->cell_cap, &ws, p->segregation, &i, &k1, &un);
                    nplus = bs->ns + bs->nb;
                } else {
                    rc = prolif_nplus(row, &nplus, &nminus, p->cell_cap, &ws, p->segregation, &i, &k1, &k2, &un);
                }
                if (rc) {
                    err = (uint32_t)rc;
                    stop = ECDNA_STOP_ERROR;
                    continue;
                }
                if (un != UNEVEN_FALSE) uneven_n += 1;
                x |= ((uint64_t)k1 << 2) | ((uint64_t)i << 20);
                break;
            }
            case ECDNA_EV_DEATH_NMINUS: /* decrease_nminus (src/proliferation.rs:135-139) */
                nminus -= 1;
                break;
            default: { /* decrease_nplus (src/proliferation.rs:126-133) */
                uint32_t i;
                if (binned) {
                    i = death_nplus_bins(bs, &ws);
                    nplus = bs->ns + bs->nb;
                } else {
                    i = death_nplus(row, &nplus, &ws);
                }
                x |= (uint64_t)i << 20;
                break;
            }
        }
        spares_update(spare, &nspare, (ch & 1) ? ws.pos : 0u, w[2], w[3]);
        cnt[ch] += 1;
        e += 1;
        if (f32t)
            t32 = t32 + tau;
        else
            t = t + (double)tau; /* self.time += reaction.time (src/process.rs:184, 336); the f64 clock */
        if (hash_on) h = fnv_fold(h, x);
    }
    if (binned) {
        bins_expand(bs, row);
        free(bs->big);
        free(bs);
        free(snap_scratch);
    }
    out->nminus = nminus;
    out->nplus = nplus;
    out->iters = e;
    for (int c = 0; c < 4; ++c) out->events_by_type[c] = cnt[c];
    out->uneven = uneven_n;
    out->time = f32t ? (double)t32 : t;
    out->event_hash = hash_on ? h : 0;
    out->stop_reason = stop;
    out->error = err;
}

/* from ssa_compat.c */
void oracle_compat_simulate_replicate(const ecdna_ssa_params_t* p, uint64_t rid, uint16_t* row,
                                      ecdna_rep_summary_t* out, ecdna_snapshot_t* snap_meta, uint16_t* snap_rows,
                                      uint64_t snap_stride, uint64_t* out_words);

static void accumulate(const ecdna_ssa_params_t* p, uint64_t rid, const uint16_t* row,
                       const ecdna_rep_summary_t* s, uint64_t* hist, ecdna_totals_t* tot) {
    const uint64_t set = rid / p->reps_per_set;
    uint64_t* hb = hist + set * p->hist_bins;
    const uint64_t last = p->hist_bins - 1;
    hb[0] += s->nminus;
    for (uint64_t j = 0; j < s->nplus; ++j) {
        uint64_t k = row[j];
        hb[k < last ? k : last] += 1;
    }
    ecdna_totals_t* t = tot + set;
    t->replicates += 1;
    t->events += s->iters;
    for (int c = 0; c < 4; ++c) t->events_by_type[c] += s->events_by_type[c];
    t->uneven += s->uneven;
    t->nminus += s->nminus;
    t->nplus += s->nplus;
    t->stop_reasons[s->stop_reason] += 1;
    t->errors += s->error != 0;
}

static void* worker(void* arg) {
    run_ctx* c = (run_ctx*)arg;
    const ecdna_ssa_params_t* p = c->p;
    uint64_t nb = (uint64_t)p->n_param_sets * p->hist_bins;
    uint64_t* hist = calloc(nb, sizeof(uint64_t));
    ecdna_totals_t* tot = calloc(p->n_param_sets, sizeof(ecdna_totals_t));
    uint16_t* scratch = c->rows ? NULL : malloc((size_t)(p->cell_cap ? p->cell_cap : 1) * sizeof(uint16_t));
    for (;;) {
        uint64_t i = atomic_fetch_add(&c->next, 1);
        if (i >= p->n_replicates) break;
        uint64_t rid = p->first_replicate + i * (p->replicate_stride ? p->replicate_stride : 1u);
        uint16_t* row = c->rows ? c->rows + i * c->row_stride : scratch;
        ecdna_rep_summary_t s;
        /* snapshot outputs: meta [n][S], rows [n][S][cell_cap] */
        const uint64_t S = p->n_snapshots;
        ecdna_snapshot_t* sm = c->snap_meta ? c->snap_meta + i * S : NULL;
        uint16_t* sr = c->snap_rows ? c->snap_rows + i * S * p->cell_cap : NULL;
        if (c->compat)
            oracle_compat_simulate_replicate(p, rid, row, &s, sm, sr, p->cell_cap,
                                             c->rng_words ? c->rng_words + i : NULL);
        else
            simulate_replicate(p, rid, row, &s, sm, sr, p->cell_cap);
        if (c->summaries) c->summaries[i] = s;
        accumulate(p, rid, row, &s, hist, tot);
    }
    pthread_mutex_lock(&c->mu);
    for (uint64_t b = 0; b < nb; ++b) c->hist[b] += hist[b];
    for (uint32_t s = 0; s < p->n_param_sets; ++s) {
        ecdna_totals_t* d = &c->totals[s];
        const ecdna_totals_t* q = &tot[s];
        d->replicates += q->replicates;
        d->events += q->events;
        for (int k = 0; k < 4; ++k) d->events_by_type[k] += q->events_by_type[k];
        d->uneven += q->uneven;
        d->nminus += q->nminus;
        d->nplus += q->nplus;
        for (int k = 0; k < 6; ++k) d->stop_reasons[k] += q->stop_reasons[k];
        d->errors += q->errors;
    }
    pthread_mutex_unlock(&c->mu);
    free(hist);
    free(tot);
    free(scratch);
    return NULL;
}

/* Parameter checks — the same contract as the product (include/ecdna_ssa.h). */
static int validate(const ecdna_ssa_params_t* p, uint64_t row_stride, int want_rows) {
    if (!p || !p->rates || p->n_param_sets == 0 || p->reps_per_set == 0 || p->hist_bins < 2)
        return ECDNA_E_INVALID;
    for (uint32_t s = 0; s < p->n_param_sets; ++s) { /* finite, non-negative rates */
        const float x[4] = {p->rates[s].b0, p->rates[s].b1, p->rates[s].d0, p->rates[s].d1};
        for (int i = 0; i < 4; ++i)
            if (!(x[i] == 0.f || (x[i] >= 0x1p-60f && x[i] <= 0x1p60f))) return ECDNA_E_INVALID;
    }
    if (p->process != ECDNA_PURE_BIRTH && p->process != ECDNA_BIRTH_DEATH) return ECDNA_E_INVALID;
    if (p->segregation < 0 || p->segregation > 3) return ECDNA_E_INVALID;
    if (p->max_iter > 0xffffffffull) return ECDNA_E_INVALID;
    const uint64_t stride = p->replicate_stride ? p->replicate_stride : 1u;
    if (p->n_replicates > 0xffffffffull) return ECDNA_E_INVALID; /* as ssa_api.cpp validate() */
    if (p->n_replicates && (p->n_replicates - 1) > (~0ull - p->first_replicate) / stride)
        return ECDNA_E_INVALID; /* first + (n - 1) * stride would wrap u64 */
    if (p->n_replicates && (p->first_replicate + (p->n_replicates - 1) * stride) / p->reps_per_set >= p->n_param_sets)
        return ECDNA_E_INVALID;
    if (!p->init_copies && (p->init_nplus || p->init_set_offsets)) return ECDNA_E_INVALID;
    uint64_t maxn = 0;
    for (uint32_t s = 0; s < p->n_param_sets; ++s) {
        const uint16_t* c;
        uint64_t np, nm;
        init_of_set(p, s, &c, &np, &nm);
        if (np > maxn) maxn = np;
        for (uint64_t j = 0; j < np; ++j)
            if (c[j] == 0) return ECDNA_E_INVALID;
        if (!p->init_set_offsets) break;
    }
    if (maxn > p->cell_cap) return ECDNA_E_INVALID;
    if ((p->flags & ECDNA_FLAG_BIN_STORE) && p->big_cap) { /* initial cells above bin_kmax fit in B */
        const uint32_t kmax = p->bin_kmax ? p->bin_kmax : 64u;
        for (uint32_t s = 0; s < p->n_param_sets; ++s) {
            const uint16_t* c;
            uint64_t np, nm, big = 0;
            init_of_set(p, s, &c, &np, &nm);
            for (uint64_t j = 0; j < np; ++j) big += c[j] > kmax;
            if (big > p->big_cap) return ECDNA_E_INVALID;
            if (!p->init_set_offsets) break;
        }
    }
    if ((p->flags & ECDNA_FLAG_BIN_STORE) && p->bin_kmax != 0 && p->bin_kmax != 32 && p->bin_kmax != 64 &&
        p->bin_kmax != 256)
        return ECDNA_E_INVALID;
    if (want_rows && row_stride < p->cell_cap) return ECDNA_E_INVALID;
    if (p->n_snapshots > 64 || (p->n_snapshots && !p->snapshot_cells)) return ECDNA_E_INVALID;
    for (uint32_t q = 1; q < p->n_snapshots; ++q)
        if (p->snapshot_cells[q] < p->snapshot_cells[q - 1]) return ECDNA_E_INVALID;
    return ECDNA_OK;
}

static int run_pool(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                    ecdna_totals_t* out_totals, uint16_t* out_rows, uint64_t row_stride, int n_threads,
                    int compat) {
    int rc = validate(p, row_stride, out_rows != NULL);
    if (rc) return rc;
    run_ctx c;
    memset(&c, 0, sizeof(c));
    c.p = p;
    c.summaries = out_summaries;
    c.rows = out_rows;
    c.row_stride = row_stride;
    atomic_init(&c.next, 0);
    pthread_mutex_init(&c.mu, NULL);
    uint64_t nb = (uint64_t)p->n_param_sets * p->hist_bins;
    c.hist = calloc(nb, sizeof(uint64_t));
    c.totals = calloc(p->n_param_sets, sizeof(ecdna_totals_t));
    c.compat = compat;
    c.snap_meta = tl_snap_meta;
    c.snap_rows = tl_snap_rows;
    c.rng_words = compat ? tl_rng_words : NULL;
    if (c.snap_meta) memset(c.snap_meta, 0, p->n_replicates * p->n_snapshots * sizeof(ecdna_snapshot_t));
    if (n_threads <= 0) n_threads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (n_threads < 1) n_threads = 1;
    if ((uint64_t)n_threads > p->n_replicates) n_threads = p->n_replicates ? (int)p->n_replicates : 1;
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int i = 1; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &c);
    worker(&c);
    for (int i = 1; i < n_threads; ++i) pthread_join(th[i], NULL);
    free(th);
    if (out_hist) memcpy(out_hist, c.hist, nb * sizeof(uint64_t));
    if (out_totals) memcpy(out_totals, c.totals, p->n_param_sets * sizeof(ecdna_totals_t));
    free(c.hist);
    free(c.totals);
    pthread_mutex_destroy(&c.mu);
    return ECDNA_OK;
}

int oracle_run_philox(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                      ecdna_totals_t* out_totals, uint16_t* out_rows, uint64_t row_stride, int n_threads) {
    return run_pool(p, out_summaries, out_hist, out_totals, out_rows, row_stride, n_threads, 0);
}

int oracle_run_compat(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                      ecdna_totals_t* out_totals, uint16_t* out_rows, uint64_t row_stride, int n_threads) {
    return run_pool(p, out_summaries, out_hist, out_totals, out_rows, row_stride, n_threads, 1);
}

/* ------------------------------------------------------ single events */

int oracle_increase_nplus(oracle_distr_t* d, int seg, uint64_t seed, uint64_t rid, uint32_t e, uint32_t* k1,
                          uint32_t* k2, int* is_uneven) {
    if (d->len == 0) return ECDNA_REP_ERR_INTERNAL; /* pick_remove_random_nplus fails on no N+ cells (src/proliferation.rs:55-57) */
    uint32_t w[4];
    event_block(seed, rid, e, w);
    wstream ws;
    ws_init(&ws, seed, rid, e, w[2], w[3]);
    uint32_t i;
    return prolif_nplus(d->cells, &d->len, &d->nminus, d->cap, &ws, seg, &i, k1, k2, is_uneven);
}

int oracle_decrease_nplus(oracle_distr_t* d, uint64_t seed, uint64_t rid, uint32_t e) {
    if (d->len == 0) return ECDNA_REP_ERR_INTERNAL; /* as increase_nplus: the engine's guard's code */
    uint32_t w[4];
    event_block(seed, rid, e, w);
    wstream ws;
    ws_init(&ws, seed, rid, e, w[2], w[3]);
    death_nplus(d->cells, &d->len, &ws);
    return 0;
}

int oracle_increase_nminus(oracle_distr_t* d) {
    d->nminus += 1;
    return 0;
}

int oracle_decrease_nminus(oracle_distr_t* d) {
    if (d->nminus == 0) return -1;
    d->nminus -= 1;
    return 0;
}

int oracle_segregate(int seg, uint32_t n, uint64_t seed, uint64_t rid, uint32_t e, uint32_t* k1, uint32_t* k2,
                     int* is_uneven) {
    if (n < 2 || (n & 1u) || n > 65534u) return -1; /* DNACopySegregating::try_from (src/segregation.rs:28-40) */
    uint32_t w[4];
    event_block(seed, rid, e, w);
    wstream ws;
    ws_init(&ws, seed, rid, e, w[2], w[3]);
    ws.pos = 1; /* segregation draws start at w3, after the cell pick's w2 */
    int rc = segregate(&ws, seg, n, k1, is_uneven);
    if (!rc) *k2 = n - *k1;
    return rc;
}
