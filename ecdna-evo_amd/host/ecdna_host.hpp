// ecdna_host.hpp — host-side mirror of the reference's I/O around the hot path:
// the EcDNADistribution value type (ecdna-lib 3.0.2; n- plus one u16 per N+ cell), its JSON
// histogram load/save (`EcDNADistribution::load`, process::save, src/process.rs:31-55, format in
// dynamics.md:8), the output file names (src/lib.rs:27-45), the default snapshot schedule
// (src/clap_app.rs:102-134) and end-of-run subsampling without replacement (`into_subsampled`,
// src/main.rs:110-123; CHANGELOG 0.26.0). Plain C++17, no HIP: the simulation itself runs through the
// C ABI (include/ecdna_ssa.h).
#pragma once

#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace ecdna {
namespace host {

struct Distribution {
    uint64_t nminus = 0;
    std::vector<uint16_t> nplus;  // one entry per N+ cell (copy number >= 1)

    uint64_t cells() const { return nminus + nplus.size(); }
    std::map<uint32_t, uint64_t> histogram() const;  // {k: cells}, key 0 = n-
    // EcDNADistribution::new from a histogram; N+ cells pushed in ascending k (the reference iterates a
    // HashMap, whose order is random per process — SURVEY.md App. B.5). More than max_nplus N+ cells
    // throw before anything is reserved or expanded (a corrupt count cannot force a huge allocation).
    static Distribution from_histogram(const std::map<uint32_t, uint64_t>& h, uint64_t max_nplus = 0xffffffffull);
};

struct IoError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// {"0":n-,"k":cells,...} with ascending keys (dynamics.md:8).
std::string to_json(const Distribution& d);
// max_nplus: the caller's capacity for N+ cells (checked before the cells are expanded)
Distribution from_json(const std::string& text, uint64_t max_nplus = 0xffffffffull);
Distribution load_json(const std::string& path, uint64_t max_nplus = 0xffffffffull);  // EcDNADistribution::load

// f32 `Display` of Rust (shortest round-trip, fixed notation) with '.' -> "dot" (src/lib.rs:27-45).
std::string rate_str(float r);
std::string filename_pure_birth(float b0, float b1, uint64_t idx);
std::string filename_birth_death(float b0, float b1, float d0, float d1, uint64_t idx);
// `format!("{:.1}", time).replace('.', "dot") + "years"` (src/process.rs:277-278).
std::string timepoint_dir(float time);
// process::save: writes {dir}/{cells}cells/ecdna/{time}years/{filename}.json; returns the path.
std::string save(const std::string& dir, const std::string& filename, float time, const Distribution& d);

// build_snapshots_from_cells (src/clap_app.rs:121-134), sorted.
std::vector<uint64_t> default_snapshots(uint64_t cells, uint32_t n_snapshots = 11);

// into_subsampled: `nb_cells` cells drawn uniformly without replacement from all n- + n+ cells (Floyd's
// algorithm over cell positions: N- cells first, then the N+ row in its order). Randomness continues
// the replicate's Philox stream in a region the stepper never uses: key (seed lo, seed hi), counter
// (sample index, 0x80000000 | block, rid lo, rid hi). nb_cells >= cells returns the whole distribution.
Distribution subsample(const Distribution& d, uint64_t nb_cells, uint64_t seed, uint64_t rid, uint32_t sample_index);

// into_subsampled under the reference's own draws (--draws reference): the reference subsamples with the SAME
// rng that ran the replicate (`into_subsampled(*nb_cells, &mut rng)`, src/main.rs:110-123, 184-197), so this
// continues ChaCha8Rng::seed_from_u64(seed) on stream `stream` (= seed * 10 + idx) at word `word_pos` (where the
// stepper left it, ecdna_ssa_ctx_download_rng_words) and advances word_pos past the words it uses. ecdna-lib
// 3.0.2's into_subsampled is not vendored; reconstructed (parity unpinned): the cells in the order
// [n- N- cells, then the N+ cells in Vec order], min(nb_cells, cells) of them chosen by rand 0.8.5
// SliceRandom::choose_multiple, i.e. seq::index::sample (Floyd / in-place / rejection by its size rule).
Distribution subsample_reference(const Distribution& d, uint64_t nb_cells, uint64_t seed, uint64_t stream,
                                 uint64_t& word_pos);

// The multi-device --pooled reduction (ecdna-dynamics --gpus N): one host thread per device shard, and the
// histogram all-reduce is an RCCL collective that every rank must join. Every shard thread reaches the
// rendezvous; the collective runs only if all shards succeeded, else no thread calls it (a rank that skips a
// collective its peers entered would hang them).
struct Rendezvous {
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0, failed = 0, total = 0;
    bool all_ok(bool ok) {
        std::unique_lock<std::mutex> lk(mu);
        arrived += 1;
        failed += ok ? 0 : 1;
        if (arrived == total) cv.notify_all();
        cv.wait(lk, [&] { return arrived == total; });
        return failed == 0;
    }
};

constexpr int kPeerFailed = -1000;  // join_reduction: another shard failed, the collective was skipped

// A shard's part of the reduction: rc = its own status so far; reduce() runs the collective (and download) and
// returns its status. Returns reduce()'s status when every shard succeeded, kPeerFailed when this shard
// succeeded but another did not, and rc (unchanged) when this shard itself failed.
template <class Reduce>
int join_reduction(Rendezvous& rv, int rc, Reduce&& reduce) {
    const bool all = rv.all_ok(rc == 0);
    if (rc) return rc;
    return all ? reduce() : kPeerFailed;
}

}  // namespace host
}  // namespace ecdna
