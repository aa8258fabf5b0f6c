/*
 * ssa_oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference's
 * hot path (fraterenz/ecdna-evo v0.26.0: sosa::simulate driving
 * PureBirth/BirthDeath::advance_step, Exponential/CellDeath and the Segregate
 * rules), used as the parity checker for the HIP engine and as the timed CPU
 * baseline in bench.py. Never linked into, or called by, the product library
 * (ecdna-evo_amd/): only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it.
 *
 * Two modes:
 *   philox  (ssa_oracle.c) — the engine's own draw mapping:
 *           bit-exact with the GPU (event sequence, rows, time, hash).
 *   compat  (ssa_compat.c) — the reference's own samplers as reconstructed in
 *           ChaCha8 streams seed*10+i, first-reaction method,
 *           gen_range + swap_remove, rand_distr Exp1 ziggurat and Binomial
 *           (BINV/BTPE). The crates (sosa 3.0.3, ecdna-lib 3.0.2,
 *           rand 0.8.5, rand_chacha 0.3.1, rand_distr 0.4.3; Cargo.lock:423-438,
 *           802-839, 944-955) are not vendored and no Rust toolchain exists
 *           here, so compat is matched to the reference in distribution only
 *           ("parity unpinned" seed-for-seed).
 */
#ifndef ECDNA_SSA_ORACLE_H
#define ECDNA_SSA_ORACLE_H

#include <stdint.h>

#include "../include/ecdna_ssa.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- primitives (philox mode) ---- */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* -ln(((w >> 9) + 0.5) * 2^-23) by the engine's fixed-operation-order f32 software log (draw mapping v6). */
float oracle_softlog_neg(uint32_t w);
/* out[i] = oracle_softlog_neg(w[i]) for i < n (the time draw's whole law in one call: tests/test_mapping_v7.py). */
void oracle_softlog_many(const uint32_t* w, uint64_t n, float* out);
/* The channel the direct method draws with word w1 from the state (n-, n+) under rates {b0, b1, d0, d1} (draw mapping
 * v7: f32 propensities, f64 cumulative sums, target (w1 + 0.5) 2^-32 A): 0 ProliferateNMinus, 1 ProliferateNPlus,
 * 2 DeathNMinus, 3 DeathNPlus; -1 when every propensity is 0. Pure birth: birth_death = 0 (d0, d1 ignored). */
int oracle_channel(const float rates[4], uint64_t nminus, uint64_t nplus, int birth_death, uint32_t w1);

/* ---- whole runs ---- */
/* Same contract as ecdna_ssa_run (include/ecdna_ssa.h) with host buffers; out_rows, if given,
 * receives [n_replicates][row_stride] final N+ rows. n_threads <= 0: all hardware threads. */
int oracle_run_philox(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries,
                      uint64_t* out_hist, ecdna_totals_t* out_totals, uint16_t* out_rows,
                      uint64_t row_stride, int n_threads);
/* Snapshot outputs for the next oracle_run_* call on this thread (NULL = discard):
 * meta[n_replicates][n_snapshots], rows[n_replicates][n_snapshots][row_stride]. */
void oracle_set_snapshot_outputs(ecdna_snapshot_t* meta, uint16_t* rows);
/* Compat mode: per replicate, the number of 32-bit words its ChaCha8 stream handed out by the end of the
 * run (the position where the reference's subsampling continues the same rng, src/main.rs:110-123) for the
 * next oracle_run_compat call on this thread (NULL = discard): words[n_replicates]. */
void oracle_set_rng_words_output(uint64_t* words);
/* Reference-semantics CPU path: stream of global replicate r is seed*10 + r (src/main.rs:56-58,
 * 213-215). Time is always accumulated in f32 like process.time (src/process.rs:184, 336);
 * ECDNA_FLAG_EVENT_HASH is honoured, ECDNA_FLAG_TIME_F32 is implied. */
int oracle_run_compat(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries,
                      uint64_t* out_hist, ecdna_totals_t* out_totals, uint16_t* out_rows,
                      uint64_t row_stride, int n_threads);

/* ---- single-event API (mirrors the reference's unit-tested functions) ---- */
/* EcDNADistribution restated: n- plus one u16 per N+ cell. */
typedef struct {
    uint16_t* cells;
    uint64_t len;
    uint64_t cap;
    uint64_t nminus;
} oracle_distr_t;

/* Exponential::increase_nplus (src/proliferation.rs:25-111) with the philox draws of event e of
 * replicate rid. Returns 0, or an ecdna_rep_error_t. *is_uneven: 0 False, 1 True,
 * 2 TrueWithoutNMinusIncrease (src/segregation.rs:50-57). */
int oracle_increase_nplus(oracle_distr_t* d, int seg, uint64_t seed, uint64_t rid, uint32_t e,
                          uint32_t* k1, uint32_t* k2, int* is_uneven);
/* CellDeath::decrease_nplus (src/proliferation.rs:126-133). Returns 0 or an error. */
int oracle_decrease_nplus(oracle_distr_t* d, uint64_t seed, uint64_t rid, uint32_t e);
/* Exponential::increase_nminus (src/proliferation.rs:113-117) and CellDeath::decrease_nminus
 * (src/proliferation.rs:135-139). decrease returns -1 when there is no N- cell. */
int oracle_increase_nminus(oracle_distr_t* d);
int oracle_decrease_nminus(oracle_distr_t* d);
/* Segregate::ecdna_segregation for n = 2k copies (src/segregation.rs:75-84). Returns 0 or
 * ECDNA_REP_ERR_REJECTION; n must be even and >= 2 (DNACopySegregating, src/segregation.rs:28-40),
 * else returns -1. */
int oracle_segregate(int seg, uint32_t n, uint64_t seed, uint64_t rid, uint32_t e, uint32_t* k1,
                     uint32_t* k2, int* is_uneven);

/* ---- compat-mode primitives ---- */
/* ChaCha block function with `rounds` rounds over the 16-word state in[16] (RFC 7539 layout). */
void oracle_chacha_block(const uint32_t in[16], uint32_t out[16], int rounds);
/* rand_core 0.6 seed_from_u64: the 32-byte ChaCha key (8 words) expanded by PCG32. */
void oracle_chacha_seed_from_u64(uint64_t seed, uint32_t key[8]);
/* Opaque ChaCha8Rng (rand_chacha 0.3.1) and its samplers, for distribution tests. */
typedef struct oracle_chacha oracle_chacha;
oracle_chacha* oracle_chacha_new(uint64_t seed, uint64_t stream);
void oracle_chacha_free(oracle_chacha* r);
uint32_t oracle_chacha_next_u32(oracle_chacha* r);
uint64_t oracle_chacha_next_u64(oracle_chacha* r);
uint64_t oracle_compat_gen_range(oracle_chacha* r, uint64_t n);   /* rand 0.8.5 gen_range(0..n) */
double oracle_compat_exp1(oracle_chacha* r);                        /* rand_distr Exp1 (ziggurat) */
uint64_t oracle_compat_binomial(oracle_chacha* r, uint64_t n, double p); /* rand_distr Binomial */
/* ecdna-lib 3.0.2 EcDNADistribution::into_subsampled(nb_cells, rng) as reconstructed (not
 * vendored, parity unpinned): the cells in the order [n- N- cells (copy number 0), then the N+ cells in
 * Vec order], min(nb_cells, cells) of them drawn without replacement (CHANGELOG.md:213-216) by rand 0.8.5
 * SliceRandom::choose_multiple = seq::index::sample (Floyd / in-place / rejection by its size rule), from the
 * ChaCha8 stream `stream` of seed_from_u64(seed) continued at word *word_pos (advanced past the words used).
 * out_cells[min(nb_cells, cells)] receives the chosen cells' copy numbers in index-vector order. Returns
 * the number chosen, or -1 when there are 2^32 or more cells. */
int64_t oracle_compat_subsample(const uint16_t* nplus_cells, uint64_t nplus, uint64_t nminus, uint64_t nb_cells,
                                uint64_t seed, uint64_t stream, uint64_t* word_pos, uint16_t* out_cells);
/* The compat mapping's ln and exp: correctly rounded (double-double), DESIGN.md §4.1. */
double oracle_compat_log(double x);
double oracle_compat_exp(double x);

#ifdef __cplusplus
}
#endif

#endif
