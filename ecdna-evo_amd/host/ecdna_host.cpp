// ecdna_host.cpp — see ecdna_host.hpp.
#include "ecdna_host.hpp"

#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <charconv>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <set>
#include <sstream>
#include <unordered_set>

namespace ecdna {
namespace host {

std::map<uint32_t, uint64_t> Distribution::histogram() const {
    std::map<uint32_t, uint64_t> h;
    h[0] = nminus;
    for (uint16_t k : nplus) h[k] += 1;
    return h;
}

Distribution Distribution::from_histogram(const std::map<uint32_t, uint64_t>& h, uint64_t max_nplus) {
    // the engine counts cells in u32 (include/ecdna_ssa.h: initial N- and N+ below 2^32); checked before
    // anything is expanded, so a corrupt count fails here instead of in a terabyte allocation
    uint64_t cells = 0;
    for (const auto& kv : h) {
        if (kv.second > 0xffffffffull) throw IoError("cell count " + std::to_string(kv.second) + " does not fit u32");
        if (kv.first != 0) cells += kv.second;
    }
    if (cells > 0xffffffffull) throw IoError("more than 2^32 - 1 N+ cells");
    if (cells > max_nplus)
        throw IoError(std::to_string(cells) + " N+ cells exceed the capacity " + std::to_string(max_nplus));
    Distribution d;
    d.nplus.reserve(cells);
    for (const auto& kv : h) {
        if (kv.first == 0) {
            d.nminus = kv.second;
            continue;
        }
        if (kv.first > 65535) throw IoError("copy number " + std::to_string(kv.first) + " does not fit u16");
        d.nplus.insert(d.nplus.end(), kv.second, (uint16_t)kv.first);
    }
    return d;
}

std::string to_json(const Distribution& d) {
    std::string s = "{";
    bool first = true;
    for (const auto& kv : d.histogram()) {
        if (!first) s += ",";
        first = false;
        s += "\"" + std::to_string(kv.first) + "\":" + std::to_string(kv.second);
    }
    return s + "}";
}

namespace {

void skip_ws(const std::string& t, size_t& i) {
    while (i < t.size() && (t[i] == ' ' || t[i] == '\n' || t[i] == '\r' || t[i] == '\t')) ++i;
}

uint64_t parse_uint(const std::string& t, size_t& i) {
    size_t j = i;
    while (j < t.size() && t[j] >= '0' && t[j] <= '9') ++j;
    if (j == i) throw IoError("expected an unsigned integer at offset " + std::to_string(i));
    uint64_t v = 0;
    auto r = std::from_chars(t.data() + i, t.data() + j, v);
    if (r.ec != std::errc()) throw IoError("integer out of range at offset " + std::to_string(i));
    i = j;
    return v;
}

}  // namespace

Distribution from_json(const std::string& t, uint64_t max_nplus) {
    std::map<uint32_t, uint64_t> h;
    size_t i = 0;
    skip_ws(t, i);
    if (i >= t.size() || t[i] != '{') throw IoError("expected '{'");
    ++i;
    skip_ws(t, i);
    if (i < t.size() && t[i] == '}') return Distribution::from_histogram(h, max_nplus);
    for (;;) {
        skip_ws(t, i);
        if (i >= t.size() || t[i] != '"') throw IoError("expected a quoted copy number");
        ++i;
        uint64_t k = parse_uint(t, i);
        if (i >= t.size() || t[i] != '"') throw IoError("expected '\"'");
        ++i;
        skip_ws(t, i);
        if (i >= t.size() || t[i] != ':') throw IoError("expected ':'");
        ++i;
        skip_ws(t, i);
        uint64_t v = parse_uint(t, i);
        if (k > 65535) throw IoError("copy number " + std::to_string(k) + " does not fit u16");
        if (v > ~0ull - h[(uint32_t)k]) throw IoError("cell count overflows u64 at offset " + std::to_string(i));
        h[(uint32_t)k] += v;
        skip_ws(t, i);
        if (i < t.size() && t[i] == ',') {
            ++i;
            continue;
        }
        if (i < t.size() && t[i] == '}') break;
        throw IoError("expected ',' or '}'");
    }
    return Distribution::from_histogram(h, max_nplus);
}

Distribution load_json(const std::string& path, uint64_t max_nplus) {
    std::ifstream f(path);
    if (!f) throw IoError("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    try {
        return from_json(ss.str(), max_nplus);
    } catch (const IoError& e) {
        throw IoError("cannot load the ecDNA distribution from " + path + ": " + e.what());
    }
}

std::string rate_str(float r) {
    char buf[64];
    auto res = std::to_chars(buf, buf + sizeof(buf), r, std::chars_format::fixed);
    std::string s(buf, res.ptr);
    std::string out;
    for (char c : s) {
        if (c == '.')
            out += "dot";
        else
            out += c;
    }
    return out;
}

std::string filename_pure_birth(float b0, float b1, uint64_t idx) {
    return rate_str(b0) + "b0_" + rate_str(b1) + "b1_0d0_0d1_" + std::to_string(idx) + "idx";
}

std::string filename_birth_death(float b0, float b1, float d0, float d1, uint64_t idx) {
    return rate_str(b0) + "b0_" + rate_str(b1) + "b1_" + rate_str(d0) + "d0_" + rate_str(d1) + "d1_" +
           std::to_string(idx) + "idx";
}

std::string timepoint_dir(float time) {
    char buf[64];
    std::snprintf(buf, sizeof(buf), "%.1f", (double)time);
    std::string out;
    for (const char* p = buf; *p; ++p) {
        if (*p == '.')
            out += "dot";
        else
            out += *p;
    }
    return out + "years";
}

namespace {

void mkdirs(const std::string& path) {
    std::string cur;
    for (size_t i = 0; i < path.size(); ++i) {
        cur += path[i];
        if ((path[i] == '/' && i > 0) || i + 1 == path.size()) {
            if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) throw IoError("cannot create dir " + cur);
        }
    }
}

}  // namespace

std::string save(const std::string& dir, const std::string& filename, float time, const Distribution& d) {
    std::string base = dir;
    if (!base.empty() && base.back() != '/') base += '/';
    const std::string folder = base + std::to_string(d.cells()) + "cells/ecdna/" + timepoint_dir(time);
    mkdirs(folder);
    const std::string path = folder + "/" + filename + ".json";
    std::ofstream f(path);
    if (!f) throw IoError("cannot write " + path);
    f << to_json(d);
    if (!f) throw IoError("cannot write " + path);
    return path;
}

std::vector<uint64_t> default_snapshots(uint64_t cells, uint32_t n) {
    const uint64_t dx = cells / (n - 1);
    std::vector<uint64_t> x(n, 1);
    for (uint32_t i = 1; i + 1 < n; ++i) x[i] = x[i - 1] + dx;
    x[n - 1] = cells;
    std::sort(x.begin(), x.end());
    return x;
}

namespace {

// Philox4x32-10 (Salmon et al. 2011) — the engine's generator, for host-side draws.
void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
    }
}

struct Words {
    uint32_t k0, k1, sample, rid_lo, rid_hi, block = 0, pos = 4;
    uint32_t buf[4];
    uint32_t next() {
        if (pos == 4) {
            buf[0] = sample;
            buf[1] = 0x80000000u | block++;
            buf[2] = rid_lo;
            buf[3] = rid_hi;
            philox(buf, k0, k1);
            pos = 0;
        }
        return buf[pos++];
    }
    // uniform in [0, n), n in [1, 2^32): Lemire with exact rejection
    uint32_t below(uint64_t n) {
        uint64_t m = (uint64_t)next() * n;
        uint32_t lo = (uint32_t)m;
        if (lo < n) {
            const uint32_t thr = (uint32_t)((0x100000000ull - n) % n);
            while (lo < thr) {
                m = (uint64_t)next() * n;
                lo = (uint32_t)m;
            }
        }
        return (uint32_t)(m >> 32);
    }
};

}  // namespace

Distribution subsample(const Distribution& d, uint64_t nb_cells, uint64_t seed, uint64_t rid, uint32_t sample_index) {
    const uint64_t N = d.cells();
    if (nb_cells >= N) return d;
    if (N > 0xffffffffull) throw IoError("subsampling needs fewer than 2^32 cells");
    Words w;
    w.k0 = (uint32_t)seed;
    w.k1 = (uint32_t)(seed >> 32);
    w.sample = sample_index;
    w.rid_lo = (uint32_t)rid;
    w.rid_hi = (uint32_t)(rid >> 32);
    std::set<uint64_t> pick;  // Floyd: for j in N-m .. N-1: t = U[0, j]; take t, or j if t was taken
    for (uint64_t j = N - nb_cells; j < N; ++j) {
        const uint64_t t = w.below(j + 1);
        if (!pick.insert(t).second) pick.insert(j);
    }
    Distribution out;
    for (uint64_t idx : pick) {
        if (idx < d.nminus)
            out.nminus += 1;
        else
            out.nplus.push_back(d.nplus[idx - d.nminus]);
    }
    return out;
}

namespace {

// rand_chacha 0.3.1 ChaCha8Rng: ChaCha with 8 rounds, 64-bit block counter in words 12-13, stream in words
// 14-15, handed out one 32-bit word at a time in block order (rand_core BlockRng over a 4-block buffer; the
// buffer only batches blocks, so the word sequence is the blocks' words in counter order). Key:
// seed_from_u64 = rand_core 0.6.4's PCG32 expansion of the u64 seed into 8 little-endian words.
struct ChaCha8Stream {
    uint32_t in[16];
    uint32_t blk[16];
    uint64_t pos;       // words handed out
    uint64_t blk_id = ~0ull;

    ChaCha8Stream(uint64_t seed, uint64_t stream, uint64_t word_pos) : pos(word_pos) {
        in[0] = 0x61707865u;
        in[1] = 0x3320646eu;
        in[2] = 0x79622d32u;
        in[3] = 0x6b206574u;
        uint64_t st = seed;
        for (int i = 0; i < 8; ++i) {
            st = st * 6364136223846793005ull + 11634580027462260723ull;
            const uint32_t xs = (uint32_t)(((st >> 18) ^ st) >> 27), rot = (uint32_t)(st >> 59);
            in[4 + i] = (xs >> rot) | (xs << ((32u - rot) & 31u));
        }
        in[14] = (uint32_t)stream;
        in[15] = (uint32_t)(stream >> 32);
    }
    static uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
    void block(uint64_t b) {
        in[12] = (uint32_t)b;
        in[13] = (uint32_t)(b >> 32);
        uint32_t x[16];
        std::memcpy(x, in, sizeof(x));
        auto qr = [&](int a, int bb, int c, int d) {
            x[a] += x[bb]; x[d] ^= x[a]; x[d] = rotl(x[d], 16);
            x[c] += x[d]; x[bb] ^= x[c]; x[bb] = rotl(x[bb], 12);
            x[a] += x[bb]; x[d] ^= x[a]; x[d] = rotl(x[d], 8);
            x[c] += x[d]; x[bb] ^= x[c]; x[bb] = rotl(x[bb], 7);
        };
        for (int r = 0; r < 8; r += 2) {
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
        }
        for (int i = 0; i < 16; ++i) blk[i] = x[i] + in[i];
        blk_id = b;
    }
    uint32_t next_u32() {
        const uint64_t b = pos >> 4;
        if (b != blk_id) block(b);
        return blk[pos++ & 15u];
    }
    // rand 0.8.5 UniformInt<u32>::sample_single_inclusive(low, high): next_u32 widened by range, conservative
    // zone (range << lz(range)) - 1
    uint32_t range_incl(uint32_t low, uint32_t high) {
        const uint32_t range = high - low + 1u;
        if (range == 0) return next_u32();
        const uint32_t zone = (range << __builtin_clz(range)) - 1u;
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * range;
            if ((uint32_t)m <= zone) return low + (uint32_t)(m >> 32);
        }
    }
    // rand 0.8.5 Uniform::new(0, n) over u32, sampled: the exact zone u32::MAX - (2^32 - n) % n
    uint32_t uniform(uint32_t n) {
        const uint32_t zone = 0xffffffffu - (uint32_t)((0x100000000ull - n) % n);
        for (;;) {
            const uint64_t m = (uint64_t)next_u32() * n;
            if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
        }
    }
};

// rand 0.8.5 seq::index::sample(rng, length, amount), length < 2^32: its algorithm choice (f32 arithmetic) and
// each algorithm's draws; the chosen indices (their order does not matter to a histogram, the draws do).
std::vector<uint32_t> index_sample(ChaCha8Stream& rng, uint32_t length, uint32_t amount) {
    const int j = length < 500000u ? 0 : 1;
    int alg;  // 0 Floyd, 1 in place, 2 rejection
    if (amount < 163u) {
        const float c0[2] = {1.6f, 8.0f / 45.0f}, c1[2] = {10.0f, 70.0f / 9.0f};
        const float a = (float)amount;
        alg = (amount > 11u && (float)length < (c1[j] + c0[j] * a) * a) ? 1 : 0;
    } else {
        const float c[2] = {270.0f, 330.0f / 9.0f};
        alg = ((float)length < c[j] * (float)amount) ? 1 : 2;
    }
    std::vector<uint32_t> idx;
    idx.reserve(amount);
    if (alg == 0) {
        const bool shuffle_after = amount >= 50u;  // below 50: Floyd's fully shuffled variant (inserts, no draws)
        std::unordered_set<uint32_t> taken;
        for (uint32_t jj = length - amount; jj < length; ++jj) {
            const uint32_t t = rng.range_incl(0u, jj);
            idx.push_back(taken.insert(t).second ? t : jj);
            if (idx.back() == jj) taken.insert(jj);
        }
        if (shuffle_after)
            for (uint32_t i = amount - 1; i >= 1; --i) std::swap(idx[i], idx[rng.range_incl(0u, i)]);
    } else if (alg == 1) {
        std::vector<uint32_t> all(length);
        for (uint32_t i = 0; i < length; ++i) all[i] = i;
        for (uint32_t i = 0; i < amount; ++i) std::swap(all[i], all[rng.range_incl(i, length - 1u)]);
        idx.assign(all.begin(), all.begin() + amount);
    } else {
        std::unordered_set<uint32_t> cache;
        for (uint32_t q = 0; q < amount; ++q) {
            uint32_t pos = rng.uniform(length);
            while (!cache.insert(pos).second) pos = rng.uniform(length);
            idx.push_back(pos);
        }
    }
    return idx;
}

}  // namespace

Distribution subsample_reference(const Distribution& d, uint64_t nb_cells, uint64_t seed, uint64_t stream,
                                 uint64_t& word_pos) {
    const uint64_t N = d.cells();
    if (N > 0xffffffffull) throw IoError("subsampling needs fewer than 2^32 cells");
    const uint32_t amount = (uint32_t)std::min<uint64_t>(nb_cells, N);  // choose_multiple clamps the amount
    ChaCha8Stream rng(seed, stream, word_pos);
    Distribution out;
    for (uint32_t i : index_sample(rng, (uint32_t)N, amount)) {
        if (i < d.nminus)
            out.nminus += 1;
        else
            out.nplus.push_back(d.nplus[i - d.nminus]);
    }
    word_pos = rng.pos;
    return out;
}

}  // namespace host
}  // namespace ecdna
