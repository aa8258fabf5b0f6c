// ecdna_host.hpp — host-side mirror of the reference's I/O around the hot path:
// the EcDNADistribution value type (ecdna-lib 3.0.2; n- plus one u16 per N+ cell), its JSON
// histogram load/save (`EcDNADistribution::load`, process::save, src/process.rs:31-55, format in
// dynamics.md:8), the output file names (src/lib.rs:27-45), the default snapshot schedule
// (src/clap_app.rs:102-134) and end-of-run subsampling without replacement (`into_subsampled`,
// src/main.rs:110-123; CHANGELOG 0.26.0). Plain C++17, no HIP: the simulation itself runs through the
// C ABI (include/ecdna_ssa.h).
#pragma once

#include <cstdint>
#include <map>
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

}  // namespace host
}  // namespace ecdna
