// ecdna_host_c.cpp — C entry points of the host I/O library (libecdna_host.so), so the naming,
// JSON and subsampling rules can be exercised from tests and other hosts without the CLI.
#include <cstring>
#include <string>

#include "../../include/ecdna_host.h"
#include "ecdna_host.hpp"

namespace {
int copy_out(const std::string& s, char* out, size_t n) {
    if (!out || n <= s.size()) return -1;
    std::memcpy(out, s.c_str(), s.size() + 1);
    return (int)s.size();
}
}  // namespace

extern "C" {

int ecdna_host_rate_str(float r, char* out, size_t n) { return copy_out(ecdna::host::rate_str(r), out, n); }

int ecdna_host_timepoint_dir(float t, char* out, size_t n) {
    return copy_out(ecdna::host::timepoint_dir(t), out, n);
}

int ecdna_host_filename(int birth_death, float b0, float b1, float d0, float d1, uint64_t idx, char* out, size_t n) {
    return copy_out(birth_death ? ecdna::host::filename_birth_death(b0, b1, d0, d1, idx)
                                : ecdna::host::filename_pure_birth(b0, b1, idx),
                    out, n);
}

// into_subsampled; out_nplus must hold min(nb_cells, n_plus) entries.
int ecdna_host_subsample(const uint16_t* nplus, uint64_t n_plus, uint64_t nminus, uint64_t nb_cells, uint64_t seed,
                         uint64_t rid, uint32_t sample_index, uint16_t* out_nplus, uint64_t* out_n_plus,
                         uint64_t* out_nminus) {
    try {
        ecdna::host::Distribution d;
        d.nminus = nminus;
        if (n_plus) d.nplus.assign(nplus, nplus + n_plus);
        ecdna::host::Distribution s = ecdna::host::subsample(d, nb_cells, seed, rid, sample_index);
        if (!s.nplus.empty()) std::memcpy(out_nplus, s.nplus.data(), s.nplus.size() * sizeof(uint16_t));
        *out_n_plus = s.nplus.size();
        *out_nminus = s.nminus;
        return 0;
    } catch (...) {
        return -1;
    }
}

// into_subsampled under the reference's draws (the replicate's ChaCha8 stream continued at *word_pos).
int ecdna_host_subsample_reference(const uint16_t* nplus, uint64_t n_plus, uint64_t nminus, uint64_t nb_cells,
                                   uint64_t seed, uint64_t stream, uint64_t* word_pos, uint16_t* out_nplus,
                                   uint64_t* out_n_plus, uint64_t* out_nminus) {
    try {
        ecdna::host::Distribution d;
        d.nminus = nminus;
        if (n_plus) d.nplus.assign(nplus, nplus + n_plus);
        ecdna::host::Distribution s = ecdna::host::subsample_reference(d, nb_cells, seed, stream, *word_pos);
        if (!s.nplus.empty()) std::memcpy(out_nplus, s.nplus.data(), s.nplus.size() * sizeof(uint16_t));
        *out_n_plus = s.nplus.size();
        *out_nminus = s.nminus;
        return 0;
    } catch (...) {
        return -1;
    }
}

// save() into dir; writes the created path.
int ecdna_host_save(const char* dir, const char* filename, float time, const uint16_t* nplus, uint64_t n_plus,
                    uint64_t nminus, char* out_path, size_t n) {
    try {
        ecdna::host::Distribution d;
        d.nminus = nminus;
        d.nplus.assign(nplus, nplus + n_plus);
        return copy_out(ecdna::host::save(dir, filename, time, d), out_path, n);
    } catch (...) {
        return -1;
    }
}

// EcDNADistribution::load: returns the number of N+ cells (<= cap) or -1.
int64_t ecdna_host_load(const char* path, uint16_t* out_nplus, uint64_t cap, uint64_t* out_nminus) {
    try {
        ecdna::host::Distribution d = ecdna::host::load_json(path, cap);  // rejects > cap before expanding
        if (!d.nplus.empty()) std::memcpy(out_nplus, d.nplus.data(), d.nplus.size() * sizeof(uint16_t));
        *out_nminus = d.nminus;
        return (int64_t)d.nplus.size();
    } catch (...) {
        return -1;
    }
}

}  // extern "C"
