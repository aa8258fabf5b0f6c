/* ecdna_host.h — C ABI of libecdna_host.so: the reference's I/O around the hot path, so a host in
 * any language can name, write, read and subsample distributions exactly as fraterenz/ecdna-evo
 * v0.26.0 does. Plain C++17 behind it, no GPU. The simulation itself is include/ecdna_ssa.h.
 *
 * Reference interfaces replaced (file:line in the reference):
 *   ecdna_host_rate_str       f32 Display with '.' -> "dot" inside file names      src/lib.rs:27-45
 *   ecdna_host_timepoint_dir  "{time:.1}" with '.' -> "dot", plus "years"         src/process.rs:31-55
 *   ecdna_host_filename       PureBirth / BirthDeath file stems                   src/process.rs:267-291,
 *                                                                                 src/lib.rs:27-45
 *   ecdna_host_save           process::save of one distribution                   src/process.rs:31-55
 *   ecdna_host_load           EcDNADistribution::load for --initial               src/clap_app.rs:177-192
 *   ecdna_host_subsample      EcDNADistribution::into_subsampled (no replacement) src/main.rs:110-123
 *   ecdna_host_subsample_reference  the same, continuing the replicate's ChaCha8 rng src/main.rs:110-123,
 *                                                                                 184-197
 *
 * String outputs: written NUL-terminated to out[0..n); the return value is the string length, or -1
 * when the buffer is too small or the call failed. */
#ifndef ECDNA_HOST_H
#define ECDNA_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Rust's f32 Display (shortest round-trip, fixed notation) with '.' replaced by "dot". */
int ecdna_host_rate_str(float r, char* out, size_t n);
/* The timepoint directory of a save at process time t: "{t:.1}" with '.' -> "dot", then "years". */
int ecdna_host_timepoint_dir(float t, char* out, size_t n);
/* File stem of replicate file index idx (seed*10 + i, src/main.rs:214). birth_death: 0 uses b0, b1
 * (PureBirth naming), 1 uses all four rates (BirthDeath naming). */
int ecdna_host_filename(int birth_death, float b0, float b1, float d0, float d1, uint64_t idx, char* out,
                        size_t n);
/* Writes {dir}/{timepoint_dir(time)}/{filename}.json with the histogram body {"0": n-, "k": cells}
 * (dynamics.md:8), creating directories; the created path goes to out_path. */
int ecdna_host_save(const char* dir, const char* filename, float time, const uint16_t* nplus, uint64_t n_plus,
                    uint64_t nminus, char* out_path, size_t n);
/* Reads such a JSON histogram: N+ cells in ascending copy number (the reference's HashMap order is
 * random per process) into out_nplus[0..cap), n- into *out_nminus. Returns the N+ count or -1. */
int64_t ecdna_host_load(const char* path, uint16_t* out_nplus, uint64_t cap, uint64_t* out_nminus);
/* nb_cells of the n- + n+ cells uniformly without replacement (Floyd's algorithm). Randomness comes
 * from replicate rid's Philox key (seed) in a counter region the stepper never uses:
 * (sample_index, 0x80000000 | block, rid). nb_cells >= n- + n+ returns the distribution unchanged.
 * out_nplus needs min(nb_cells, n_plus) entries. Returns 0, or -1 on failure. */
int ecdna_host_subsample(const uint16_t* nplus, uint64_t n_plus, uint64_t nminus, uint64_t nb_cells, uint64_t seed,
                         uint64_t rid, uint32_t sample_index, uint16_t* out_nplus, uint64_t* out_n_plus,
                         uint64_t* out_nminus);
/* into_subsampled under the reference's own draws: the reference subsamples with the rng that ran the
 * replicate (src/main.rs:110-123, 184-197), so this continues ChaCha8Rng::seed_from_u64(seed), stream `stream`
 * (= seed*10 + idx), at word *word_pos (ecdna_ssa_ctx_download_rng_words; advanced past the words used, so
 * consecutive subsamples of one replicate chain as in the reference's loop). Reconstruction of ecdna-lib 3.0.2
 * (not vendored; parity unpinned): cells ordered [n- N- cells, then the N+ cells in order], min(nb_cells,
 * cells) chosen by rand 0.8.5 SliceRandom::choose_multiple (seq::index::sample). out_nplus needs
 * min(nb_cells, n_plus) entries. Returns 0, or -1 on failure. */
int ecdna_host_subsample_reference(const uint16_t* nplus, uint64_t n_plus, uint64_t nminus, uint64_t nb_cells,
                                   uint64_t seed, uint64_t stream, uint64_t* word_pos, uint16_t* out_nplus,
                                   uint64_t* out_n_plus, uint64_t* out_nminus);

#ifdef __cplusplus
}
#endif

#endif /* ECDNA_HOST_H */
