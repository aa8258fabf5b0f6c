// ssa_api.cpp — the C ABI of include/ecdna_ssa.h: parameter validation,
// device-resident run contexts, chunking by HBM capacity, and launches of the
// stepper and histogram kernels (ssa_kernels.hip).
//
// This file replaces, for one GPU, the per-replicate driver loop of the
// reference: run_simulations(idx) mapped by rayon over seed*10 .. seed*10+runs
// (src/main.rs:55-225). Everything here is host code; there is no CPU
// fallback — without a gfx950 device every entry point returns
// ECDNA_E_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ecdna_ssa.h"
#include "ssa_launch.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess)                                                                        \
            return fail(_e == hipErrorOutOfMemory ? ECDNA_E_NOMEM : ECDNA_E_HIP,                     \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                          \
    } while (0)

uint64_t round_up(uint64_t x, uint64_t m) { return (x + m - 1) / m * m; }

struct InitOfSet {
    const uint16_t* copies;
    uint64_t nplus;
    uint64_t nminus;
};

InitOfSet init_of_set(const ecdna_ssa_params_t* p, uint64_t s) {
    InitOfSet r;
    if (p->init_set_offsets) {
        r.copies = p->init_copies + p->init_set_offsets[s];
        r.nplus = p->init_set_offsets[s + 1] - p->init_set_offsets[s];
    } else {
        r.copies = p->init_copies;
        r.nplus = p->init_nplus;
    }
    r.nminus = p->init_set_nminus ? p->init_set_nminus[s] : p->init_nminus;
    return r;
}

int validate(const ecdna_ssa_params_t* p) {
    if (!p) return fail(ECDNA_E_INVALID, "params is NULL");
    if (!p->rates || p->n_param_sets == 0) return fail(ECDNA_E_INVALID, "rates/n_param_sets");
    for (uint32_t s = 0; s < p->n_param_sets; ++s) {  // (the steppers' f32 time-step division relies on it)
        const ecdna_rates_t& r = p->rates[s];
        for (const float x : {r.b0, r.b1, r.d0, r.d1})
            if (!(x == 0.f || (x >= 0x1p-60f && x <= 0x1p60f)))
                return fail(ECDNA_E_INVALID, "rates must be 0 or in [2^-60, 2^60]");
    }
    if (p->reps_per_set == 0) return fail(ECDNA_E_INVALID, "reps_per_set must be >= 1");
    if (p->reserved0) return fail(ECDNA_E_INVALID, "reserved0 must be 0");
    // (bit 31 is the library's internal snapshot bit, kFlagSnapshotsRt: a caller setting it, or any other unknown bit,
    // would silently select another kernel instance)
    if (p->flags & ~(uint32_t)ECDNA_FLAG_ALL) return fail(ECDNA_E_INVALID, "unknown bits in flags");
    if (p->hist_bins < 2 || p->hist_bins > ecdna::kMaxHistBins)
        return fail(ECDNA_E_INVALID, "hist_bins must be in [2, 4096]");
    if ((p->flags & ECDNA_FLAG_REP_STATS) && p->hist_bins > 2048)
        return fail(ECDNA_E_INVALID, "ECDNA_FLAG_REP_STATS needs hist_bins <= 2048");
    if (p->process != ECDNA_PURE_BIRTH && p->process != ECDNA_BIRTH_DEATH)
        return fail(ECDNA_E_INVALID, "unknown process");
    if (p->segregation < 0 || p->segregation > 3) return fail(ECDNA_E_INVALID, "unknown segregation");
    if (p->max_iter > 0xffffffffull) return fail(ECDNA_E_INVALID, "max_iter must be < 2^32");
    if (p->n_replicates > 0xffffffffull) return fail(ECDNA_E_INVALID, "n_replicates must be < 2^32 per call");
    const uint64_t stride = p->replicate_stride ? p->replicate_stride : 1u;
    if (p->n_replicates && (p->n_replicates - 1) > (~0ull - p->first_replicate) / stride)
        return fail(ECDNA_E_INVALID, "replicate ids overflow u64");
    if (p->n_replicates && (p->first_replicate + (p->n_replicates - 1) * stride) / p->reps_per_set >= p->n_param_sets)
        return fail(ECDNA_E_INVALID, "replicate ids map past the last parameter set");
    if (p->cell_cap == 0) return fail(ECDNA_E_INVALID, "cell_cap must be >= 1");
    if ((p->flags & ECDNA_FLAG_REFERENCE_DRAWS) && (p->flags & ECDNA_FLAG_BIN_STORE))
        return fail(ECDNA_E_INVALID, "ECDNA_FLAG_REFERENCE_DRAWS runs the row store only (no ECDNA_FLAG_BIN_STORE)");
    if ((p->flags & ECDNA_FLAG_BIN_STORE) && p->bin_kmax != 0 && p->bin_kmax != 32 && p->bin_kmax != 64 &&
        p->bin_kmax != 256)
        return fail(ECDNA_E_INVALID, "bin_kmax must be 0 (= 64), 32, 64 or 256");
    if (p->n_snapshots > ecdna::kMaxSnapshots) return fail(ECDNA_E_INVALID, "at most 64 snapshots");
    if (p->n_snapshots && !p->snapshot_cells) return fail(ECDNA_E_INVALID, "snapshot_cells is NULL");
    for (uint32_t q = 1; q < p->n_snapshots; ++q)
        if (p->snapshot_cells[q] < p->snapshot_cells[q - 1])
            return fail(ECDNA_E_INVALID, "snapshot_cells must be sorted ascending");
    if (!p->init_copies && (p->init_nplus || p->init_set_offsets))
        return fail(ECDNA_E_INVALID, "init_copies is NULL");
    for (uint32_t s = 0; s < p->n_param_sets; ++s) {
        InitOfSet in = init_of_set(p, s);
        if (in.nplus > p->cell_cap) return fail(ECDNA_E_INVALID, "initial N+ cells exceed cell_cap");
        if ((p->flags & ECDNA_FLAG_BIN_STORE) && p->big_cap) {
            const uint32_t kmax = p->bin_kmax ? p->bin_kmax : 64u;
            uint64_t big = 0;
            for (uint64_t j = 0; j < in.nplus; ++j) big += in.copies[j] > kmax;
            if (big > p->big_cap) return fail(ECDNA_E_INVALID, "initial cells above bin_kmax exceed big_cap");
        }
        if (in.nminus > 0xffffffffull) return fail(ECDNA_E_INVALID, "initial N- cells must be < 2^32");
        for (uint64_t j = 0; j < in.nplus; ++j)
            if (in.copies[j] == 0) return fail(ECDNA_E_INVALID, "initial copy numbers must be >= 1");
        if (!p->init_set_offsets && !p->init_set_nminus) break;
    }
    return ECDNA_OK;
}

// Reference draws (ECDNA_FLAG_REFERENCE_DRAWS): rand_core 0.6.4 seed_from_u64 — the 32-byte ChaCha key filled
// by a PCG32 sequence from the seed (little-endian words).
void chacha_key_from_u64(uint64_t state, uint32_t key[8]) {
    const uint64_t mul = 6364136223846793005ull, inc = 11634580027462260723ull;
    for (int i = 0; i < 8; ++i) {
        state = state * mul + inc;
        const uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        const uint32_t rot = (uint32_t)(state >> 59);
        key[i] = (xorshifted >> rot) | (xorshifted << ((32u - rot) & 31u));
    }
}

// rand_distr 0.4.3 BTPE setup of Binomial(n, 1/2) (the step-0 constants; oracle/ssa_compat.c computes the same
// per call), one row of refdraws::kBtpeRow doubles per copy number k = n / 2: npq, m, p1, x_m, x_l, x_r, c,
// p2, lambda_l, lambda_r, p3, p4, then 1 / lambda_l, 1 / lambda_r for the GPU's filtered step. Only n >= 20 (n p >= 10) takes BTPE.
void btpe_setup(uint64_t n_u, double* row) {
    const double p = 0.5, q = 1.0 - p;
    const double n = (double)n_u;
    const double np = n * p;
    const double npq = np * q;
    const double f_m = np + p;
    const int64_t m = (int64_t)f_m;
    const double p1 = std::floor(2.195 * std::sqrt(npq) - 4.6 * q) + 0.5;
    const double x_m = (double)m + 0.5;
    const double x_l = x_m - p1;
    const double x_r = x_m + p1;
    const double c = 0.134 + 20.5 / (15.3 + (double)m);
    const double p2 = p1 * (1. + 2. * c);
    const double al = (f_m - x_l) / (f_m - x_l * p);
    const double lambda_l = al * (1. + 0.5 * al);
    const double ar = (x_r - f_m) / (x_r * q);
    const double lambda_r = ar * (1. + 0.5 * ar);
    const double p3 = p2 + c / lambda_l;
    const double p4 = p3 + c / lambda_r;
    // (+ 1 / lambda_l, 1 / lambda_r: not the reference's arithmetic; only the GPU's filtered region-3/4 step uses them,
    // refdraws::trunc_log_ratio, where a quotient within ~2^-37 decides)
    const double v[14] = {npq, (double)m, p1, x_m, x_l, x_r, c, p2, lambda_l, lambda_r, p3, p4, 1.0 / lambda_l, 1.0 / lambda_r};
    for (int i = 0; i < 14; ++i) row[i] = v[i];
}
constexpr int kBtpeRow = 16;  // refdraws::kBtpeRow

struct Chunk {
    uint64_t first;  // local index of the first replicate
    uint32_t n;
    hipEvent_t ev[3];
    // replicate rotation (bin store; 0 = off): partition size and the counters it starts from
    uint32_t rot_n_pad = 0;
    std::vector<ecdna::RotPart> rot_init;
    // persistent grid of the chunk and its drain control (admit_slot 0xffffffff: off)
    uint32_t blocks = 1;
    uint32_t admit_slot = 0xffffffffu;
    uint32_t admit_remaining = 0;
};

}  // namespace

struct ecdna_ssa_ctx {
    ecdna_ssa_params_t p{};
    int device = 0;
    int cus = 0;
    uint64_t row_stride = 0;  // device rows (the bin store: its large-k rows, big_cap cells)
    uint64_t out_stride = 0;  // downloaded and snapshot rows (cell_cap cells)
    uint32_t big_cap = 0;     // bin store: large-k row capacity
    uint64_t chunk_reps = 0;
    uint32_t stepper_blocks_cap = 0;
    int window = 1;  // LDS tail window stepper (ECDNA_SSA_WINDOW=0 selects the HBM-only variant)
    // bin store (ECDNA_FLAG_BIN_STORE): binned copy numbers (0 = row store), u32 counters, the
    // per-replicate final counters [chunk_reps][bin_k]
    uint32_t bin_k = 0;
    int bin_c32 = 0;
    int bin_ilp = 0;  // the bin stepper's schedule: 0 default, 1 max-ILP (lone waves), 2 128-VGPR K = 64, 3 max-ILP paired lanes (ssa_launch.h)
    void* d_bags = nullptr;
    uint32_t stepper_block = ecdna::kStepperBlock;
    // reference draws (ECDNA_FLAG_REFERENCE_DRAWS): the ChaCha8 key and the BTPE constants per copy number
    bool refdraws = false;
    uint32_t* d_ref_key = nullptr;
    double* d_ref_btpe = nullptr;
    uint64_t* d_rng_words = nullptr;  // [n] ChaCha8 stream position of each replicate at its end
    // owned copies of the host inputs
    std::vector<ecdna_rates_t> rates;
    std::vector<uint16_t> init_copies;
    std::vector<uint32_t> init_offsets;
    std::vector<uint64_t> init_nminus_set;
    std::vector<uint64_t> snap_cells;
    // ABC statistics target
    bool has_target = false;
    double target_mean = 0.0, target_entropy = 0.0, target_freq = 0.0;
    double* d_target_cdf = nullptr;
    ecdna_rep_stats_t* d_stats = nullptr;
    // device buffers
    float4* d_rates = nullptr;
    uint16_t* d_init = nullptr;
    uint32_t* d_init_off = nullptr;
    uint64_t* d_init_nm = nullptr;
    uint64_t* d_snap_cells = nullptr;
    ecdna_snapshot_t* d_snap_meta = nullptr;
    uint16_t* d_snap_rows = nullptr;
    uint16_t* d_rows = nullptr;
    ecdna_rep_summary_t* d_summ = nullptr;
    uint32_t* d_heads = nullptr;  // one work counter per chunk
    uint32_t* d_order = nullptr;  // [n] chunk-local start order (set_cost_hint) or nullptr
    // replicate rotation (bin store): per-partition counters, state bytes, parked scalars (one chunk's worth)
    ecdna::RotPart* d_rot_parts = nullptr;
    uint32_t* d_rot_flags = nullptr;
    uint4* d_rot_park = nullptr;
    uint32_t rot_tick_log2 = 11;
    int32_t rot_park_min = 0;
    uint64_t* d_hist_own = nullptr;
    ecdna_totals_t* d_tot_own = nullptr;
    uint64_t* d_hist = nullptr;
    ecdna_totals_t* d_tot = nullptr;
    hipStream_t last_stream = nullptr;
    std::vector<Chunk> chunks;
    bool launched = false;
};

namespace {

// the flags the kernels see: the caller's, plus the internal snapshot bit that selects the runtime-flags instances
uint32_t kernel_flags(const ecdna_ssa_params_t& p) { return p.flags | (p.n_snapshots ? ecdna::kFlagSnapshotsRt : 0u); }

int pick_device(int dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(ECDNA_E_NODEVICE, "no HIP device");
    if (dev < 0 || dev >= n) return fail(ECDNA_E_NODEVICE, "device ordinal out of range");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(ECDNA_E_NODEVICE, "device query failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(ECDNA_E_NODEVICE, std::string("not a gfx950 device: ") + prop.gcnArchName);
    if (hipSetDevice(dev) != hipSuccess) return fail(ECDNA_E_NODEVICE, "hipSetDevice failed");
    return ECDNA_OK;
}

uint64_t env_u64(const char* name, uint64_t dflt) {
    const char* v = std::getenv(name);
    if (!v || !*v) return dflt;
    return std::strtoull(v, nullptr, 10);
}

// The bin stepper's instruction-schedule rule, a pure function of the run's shape and the kernels'
// occupancies so that the CPU tests can walk any shape through it (ecdna_dev_bin_schedule, tests/test_host.py).
// Returns ecdna_ssa_instance_t.schedule: 0 occupancy-first, 1 max-ILP, 2 the 128-VGPR build (K = 64 / u16), 3 max-ILP
// paired lanes. pair_ok: birth-death without snapshots and a paired instance exists; pair_mode ECDNA_SSA_PAIR (0 off,
// 1 pairs whenever possible, 2 auto); sched ECDNA_SSA_SCHED (0, 1, 2 auto, 3);
// max_chunk the largest chunk's replicates; occ_def / occ_ilp workgroups per CU of the two builds.
int bin_schedule_rule(bool pair_ok, uint64_t pair_mode, uint64_t sched, uint64_t max_chunk, uint32_t cus, bool k64u16,
                      bool tf0, int occ_def, int occ_ilp, uint32_t stepper_block) {
    if (pair_ok && (pair_mode == 1 ||
                    (pair_mode == 2 && sched == 2 && max_chunk <= (uint64_t)cus * (ecdna::kStepperBlock / 2))))
        return 3;
    if (sched == 1 || (sched == 2 && max_chunk <= (uint64_t)cus * 256u)) return 1;
    if (k64u16 && (sched == 3 || (sched == 2 && tf0 && max_chunk >= 4ull * cus * 4u * ecdna::kStepperBlock))) return 2;
    if (sched == 2 && (occ_ilp >= occ_def || max_chunk < 4ull * (uint64_t)occ_def * cus * stepper_block)) return 1;
    return 0;
}

void free_ctx(ecdna_ssa_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    for (auto& ch : c->chunks)
        for (auto& e : ch.ev)
            if (e) (void)hipEventDestroy(e);
    (void)hipFree(c->d_rates);
    (void)hipFree(c->d_init);
    (void)hipFree(c->d_init_off);
    (void)hipFree(c->d_init_nm);
    (void)hipFree(c->d_snap_cells);
    (void)hipFree(c->d_snap_meta);
    (void)hipFree(c->d_snap_rows);
    (void)hipFree(c->d_target_cdf);
    (void)hipFree(c->d_stats);
    (void)hipFree(c->d_rows);
    (void)hipFree(c->d_bags);
    (void)hipFree(c->d_summ);
    (void)hipFree(c->d_heads);
    (void)hipFree(c->d_order);
    (void)hipFree(c->d_rot_parts);
    (void)hipFree(c->d_rot_flags);
    (void)hipFree(c->d_rot_park);
    (void)hipFree(c->d_ref_key);
    (void)hipFree(c->d_ref_btpe);
    (void)hipFree(c->d_rng_words);
    (void)hipFree(c->d_hist_own);
    (void)hipFree(c->d_tot_own);
    delete c;
}

}  // namespace

// library-internal entry points for ssa_comm.cpp (the RCCL reduction)
__attribute__((visibility("hidden"))) int ecdna_ssa_internal_fail(int code, const std::string& msg) {
    return fail(code, msg);
}

__attribute__((visibility("hidden"))) int ecdna_ssa_internal_ctx_outputs(ecdna_ssa_ctx* c, uint64_t** d_hist,
                                                                         ecdna_totals_t** d_tot, uint32_t* n_sets,
                                                                         uint32_t* bins, int* device, void** stream) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "reduce before launch");
    *d_hist = c->d_hist;
    *d_tot = c->d_tot;
    *n_sets = c->p.n_param_sets;
    *bins = c->p.hist_bins;
    *device = c->device;
    *stream = c->last_stream;
    return ECDNA_OK;
}

extern "C" {

int ecdna_ssa_abi_version(void) { return ECDNA_SSA_ABI_VERSION; }

// (development / test entry point, not part of include/ecdna_ssa.h: bin_schedule_rule for the CPU tests)
int ecdna_dev_bin_schedule(int pair_ok, uint64_t pair_mode, uint64_t sched, uint64_t max_chunk, uint32_t cus,
                           int k64u16, int tf0, int occ_def, int occ_ilp, uint32_t stepper_block) {
    return bin_schedule_rule(pair_ok != 0, pair_mode, sched, max_chunk, cus, k64u16 != 0, tf0 != 0, occ_def, occ_ilp,
                             stepper_block);
}

const char* ecdna_ssa_strerror(int code) {
    switch (code) {
        case ECDNA_OK: return "ok";
        case ECDNA_E_INVALID: return "invalid argument";
        case ECDNA_E_HIP: return "HIP runtime error";
        case ECDNA_E_NOMEM: return "device out of memory";
        case ECDNA_E_NODEVICE: return "no usable gfx950 device";
        case ECDNA_E_STATE: return "invalid call order";
        case ECDNA_E_COMM: return "RCCL communication error (or librccl.so.1 missing)";
        default: return "unknown error";
    }
}

const char* ecdna_ssa_last_error_message(void) { return g_last_error.c_str(); }

int ecdna_ssa_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
            ++good;
    }
    return good;
}

int ecdna_ssa_ctx_create(const ecdna_ssa_params_t* p, ecdna_ssa_ctx** out) {
    if (!out) return fail(ECDNA_E_INVALID, "out is NULL");
    *out = nullptr;
    int rc = validate(p);
    if (rc) return rc;
    rc = pick_device(p->device);
    if (rc) return rc;

    ecdna_ssa_ctx* c = new ecdna_ssa_ctx();
    c->p = *p;
    c->device = p->device;
    // own copies of host inputs
    c->rates.assign(p->rates, p->rates + p->n_param_sets);
    uint64_t n_init = p->init_set_offsets ? p->init_set_offsets[p->n_param_sets] : p->init_nplus;
    c->init_copies.assign(p->init_copies ? p->init_copies : nullptr,
                          p->init_copies ? p->init_copies + n_init : nullptr);
    if (c->init_copies.empty()) c->init_copies.push_back(1);
    if (p->init_set_offsets) c->init_offsets.assign(p->init_set_offsets, p->init_set_offsets + p->n_param_sets + 1);
    if (p->init_set_nminus) c->init_nminus_set.assign(p->init_set_nminus, p->init_set_nminus + p->n_param_sets);
    if (p->n_snapshots) c->snap_cells.assign(p->snapshot_cells, p->snapshot_cells + p->n_snapshots);
    c->p.snapshot_cells = nullptr;
    c->p.rates = nullptr;
    c->p.init_copies = nullptr;
    c->p.init_set_offsets = nullptr;
    c->p.init_set_nminus = nullptr;

    auto bail = [&](int code) {
        free_ctx(c);
        return code;
    };
#define CTX_TRY(expr)                                                                                \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess)                                                                        \
            return bail(fail(_e == hipErrorOutOfMemory ? ECDNA_E_NOMEM : ECDNA_E_HIP,                \
                             std::string(#expr) + ": " + hipGetErrorString(_e)));                     \
    } while (0)

    hipDeviceProp_t prop;
    CTX_TRY(hipGetDeviceProperties(&prop, c->device));
    c->cus = prop.multiProcessorCount;

    // inputs
    std::vector<float4> r4(p->n_param_sets);
    for (uint32_t s = 0; s < p->n_param_sets; ++s)
        r4[s] = make_float4(p->rates[s].b0, p->rates[s].b1, p->rates[s].d0, p->rates[s].d1);
    CTX_TRY(hipMalloc(&c->d_rates, r4.size() * sizeof(float4)));
    CTX_TRY(hipMemcpy(c->d_rates, r4.data(), r4.size() * sizeof(float4), hipMemcpyHostToDevice));
    CTX_TRY(hipMalloc(&c->d_init, c->init_copies.size() * sizeof(uint16_t)));
    CTX_TRY(hipMemcpy(c->d_init, c->init_copies.data(), c->init_copies.size() * sizeof(uint16_t),
                      hipMemcpyHostToDevice));
    if (!c->init_offsets.empty()) {
        CTX_TRY(hipMalloc(&c->d_init_off, c->init_offsets.size() * sizeof(uint32_t)));
        CTX_TRY(hipMemcpy(c->d_init_off, c->init_offsets.data(), c->init_offsets.size() * sizeof(uint32_t),
                          hipMemcpyHostToDevice));
    }
    if (!c->init_nminus_set.empty()) {
        CTX_TRY(hipMalloc(&c->d_init_nm, c->init_nminus_set.size() * sizeof(uint64_t)));
        CTX_TRY(hipMemcpy(c->d_init_nm, c->init_nminus_set.data(), c->init_nminus_set.size() * sizeof(uint64_t),
                          hipMemcpyHostToDevice));
    }

    if (!c->snap_cells.empty()) {
        CTX_TRY(hipMalloc(&c->d_snap_cells, c->snap_cells.size() * sizeof(uint64_t)));
        CTX_TRY(hipMemcpy(c->d_snap_cells, c->snap_cells.data(), c->snap_cells.size() * sizeof(uint64_t),
                          hipMemcpyHostToDevice));
    }

    // ABC statistics: the target's CDF over the bins and its mean / entropy / N+ frequency (the overflow bin
    // counts at k = bins - 1), computed once on the host
    if ((p->flags & ECDNA_FLAG_REP_STATS) && p->n_replicates) {
        CTX_TRY(hipMalloc(&c->d_stats, p->n_replicates * sizeof(ecdna_rep_stats_t)));
        if (p->stats_target_hist) {
            const uint32_t bins = p->hist_bins;
            double tot = 0.0;
            for (uint32_t b = 0; b < bins; ++b) tot += (double)p->stats_target_hist[b];
            if (!(tot > 0.0)) return bail(fail(ECDNA_E_INVALID, "stats_target_hist is empty"));
            std::vector<double> cdf(bins);
            double acc = 0.0, ksum = 0.0, ent = 0.0;
            for (uint32_t b = 0; b < bins; ++b) {
                const double pb = (double)p->stats_target_hist[b] / tot;
                acc += pb;
                cdf[b] = acc;
                ksum += (double)b * (double)p->stats_target_hist[b];
                if (pb > 0.0) ent -= pb * std::log(pb);
            }
            c->has_target = true;
            c->target_mean = ksum / tot;
            c->target_entropy = ent;
            c->target_freq = 1.0 - (double)p->stats_target_hist[0] / tot;
            CTX_TRY(hipMalloc(&c->d_target_cdf, bins * sizeof(double)));
            CTX_TRY(hipMemcpy(c->d_target_cdf, cdf.data(), bins * sizeof(double), hipMemcpyHostToDevice));
        }
    }
    c->p.stats_target_hist = nullptr;

    // outputs
    const uint64_t n = p->n_replicates;
    const uint64_t nb = (uint64_t)p->n_param_sets * p->hist_bins;
    CTX_TRY(hipMalloc(&c->d_hist_own, nb * sizeof(uint64_t)));
    CTX_TRY(hipMalloc(&c->d_tot_own, p->n_param_sets * sizeof(ecdna_totals_t)));
    CTX_TRY(hipMemset(c->d_hist_own, 0, nb * sizeof(uint64_t)));
    CTX_TRY(hipMemset(c->d_tot_own, 0, p->n_param_sets * sizeof(ecdna_totals_t)));
    c->d_hist = c->d_hist_own;
    c->d_tot = c->d_tot_own;
    CTX_TRY(hipMalloc(&c->d_summ, std::max<uint64_t>(n, 1) * sizeof(ecdna_rep_summary_t)));

    c->row_stride = round_up(p->cell_cap, 64);
    c->out_stride = c->row_stride;
    if (p->flags & ECDNA_FLAG_BIN_STORE) {
        c->big_cap = (p->big_cap && p->big_cap < p->cell_cap) ? p->big_cap : p->cell_cap;
        c->row_stride = round_up(c->big_cap, 64);
        c->bin_k = p->bin_kmax ? p->bin_kmax : 64;
        // u16 counters hold at most 65535 cells per bin/group; K = 32 always uses u32 counters: the same LDS
        // footprint as K = 64/u16 (144 B per lane), no 16-bit packing in the updates and the scan (C3:
        // 119 ms against 126 ms with u16)
        // (ECDNA_SSA_C32 = 1 forces u32 counters at any K: a development knob, results are the same)
        c->bin_c32 = (p->cell_cap > 65535u || c->bin_k <= 32 || env_u64("ECDNA_SSA_C32", 0)) ? 1 : 0;
        c->stepper_block = (uint32_t)ecdna::bin_stepper_block(c->bin_k);
    }
    const uint64_t bag_bytes = (uint64_t)c->bin_k * (c->bin_c32 ? 4u : 2u);
    if (p->n_snapshots && n) {  // snapshot outputs cover the whole run (not chunked)
        CTX_TRY(hipMalloc(&c->d_snap_meta, n * p->n_snapshots * sizeof(ecdna_snapshot_t)));
        if (p->flags & ECDNA_FLAG_SNAPSHOT_ROWS)
            CTX_TRY(hipMalloc(&c->d_snap_rows, n * p->n_snapshots * c->out_stride * sizeof(uint16_t)));
    }

    // rows: one u16 row per replicate of the chunk; chunk bounded by free HBM
    const uint64_t rot_bytes = c->bin_k ? ecdna::kParkVecs * 16u + 4u : 0u;  // parked scalars + state word
    const uint64_t row_bytes = c->row_stride * sizeof(uint16_t) + bag_bytes + rot_bytes;
    size_t free_b = 0, total_b = 0;
    CTX_TRY(hipMemGetInfo(&free_b, &total_b));
    uint64_t budget = (uint64_t)((double)free_b * 0.85);
    uint64_t cap_budget = env_u64("ECDNA_SSA_MAX_ROW_BYTES", 0);
    if (cap_budget) budget = std::min<uint64_t>(budget, cap_budget);
    uint64_t fit = budget / row_bytes;
    uint64_t max_chunk = env_u64("ECDNA_SSA_MAX_CHUNK", 0);
    if (max_chunk) fit = std::min<uint64_t>(fit, max_chunk);
    if (fit == 0) return bail(fail(ECDNA_E_NOMEM, "one replicate row does not fit in device memory"));
    c->chunk_reps = std::min<uint64_t>(std::max<uint64_t>(n, 1), fit);
    CTX_TRY(hipMalloc(&c->d_rows, c->chunk_reps * c->row_stride * sizeof(uint16_t)));
    if (c->bin_k) CTX_TRY(hipMalloc(&c->d_bags, c->chunk_reps * bag_bytes));

    const uint64_t n_chunks = n ? (n + c->chunk_reps - 1) / c->chunk_reps : 0;
    CTX_TRY(hipMalloc(&c->d_heads, std::max<uint64_t>(n_chunks, 1) * sizeof(uint32_t)));
    for (uint64_t k = 0; k < n_chunks; ++k) {
        Chunk ch{};
        ch.first = k * c->chunk_reps;
        ch.n = (uint32_t)std::min<uint64_t>(c->chunk_reps, n - ch.first);
        c->chunks.push_back(ch);
        for (auto& e : c->chunks.back().ev) CTX_TRY(hipEventCreate(&e));
    }

    // start order (set_cost_hint): within each chunk, replicates of costlier sets first, then by id
    if (p->set_cost_hint && n) {
        const uint64_t stride = p->replicate_stride ? p->replicate_stride : 1u;
        std::vector<uint32_t> order(n);
        for (const Chunk& ch : c->chunks) {
            uint32_t* o = order.data() + ch.first;
            for (uint32_t i = 0; i < ch.n; ++i) o[i] = i;
            auto cost = [&](uint32_t i) {
                const float v = p->set_cost_hint[(p->first_replicate + (ch.first + i) * stride) / p->reps_per_set];
                return v == v ? v : 0.0f;  // (NaN: no preference)
            };
            std::stable_sort(o, o + ch.n, [&](uint32_t x, uint32_t y) { return cost(x) > cost(y); });
        }
        CTX_TRY(hipMalloc(&c->d_order, n * sizeof(uint32_t)));
        CTX_TRY(hipMemcpy(c->d_order, order.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
    }

    // persistent stepper grid: as many resident lanes as the occupancy allows
    c->window = env_u64("ECDNA_SSA_WINDOW", 1) ? 1 : 0;
    int per_cu = 0;
    c->refdraws = (p->flags & ECDNA_FLAG_REFERENCE_DRAWS) != 0;
    if (c->refdraws) {
        uint32_t key[8];
        chacha_key_from_u64(p->seed, key);
        CTX_TRY(hipMalloc(&c->d_ref_key, sizeof(key)));
        CTX_TRY(hipMemcpy(c->d_ref_key, key, sizeof(key), hipMemcpyHostToDevice));
        std::vector<double> bt((uint64_t)32768 * kBtpeRow, 0.0);
        for (uint64_t k = 10; k < 32768; ++k) btpe_setup(2 * k, bt.data() + k * kBtpeRow);
        CTX_TRY(hipMalloc(&c->d_ref_btpe, bt.size() * sizeof(double)));
        CTX_TRY(hipMemcpy(c->d_ref_btpe, bt.data(), bt.size() * sizeof(double), hipMemcpyHostToDevice));
        CTX_TRY(hipMalloc(&c->d_rng_words, std::max<uint64_t>(n, 1) * sizeof(uint64_t)));
        c->stepper_block = (uint32_t)ecdna::refdraws_block();
        CTX_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, ecdna::refdraws_kernel(p->process, p->segregation), (int)c->stepper_block, 0));
    } else if (c->bin_k) {
        // Instruction schedule: with at most one wave of replicates per SIMD (every chunk within 256 lanes
        // per CU) each wave runs alone and waits on its own dependencies, and the max-ILP schedule is faster
        // (C2 8.6 -> 8.1 ms, C5 8-GPU shard 22.0 -> 21.1 s); with more, issue binds and the default schedule
        // keeps 4 waves per SIMD (max-ILP: 3, C3 +8 %). The K = 64 / u16 kernel needs 130 VGPRs (3
        // workgroups per CU); its 128-VGPR build fits 4 and pays once lanes run many replicates each (the
        // whole C4 sweep on one GPU, 16 per lane: 834 -> 771 ms) but not with few (C4 8-GPU shard, 2 per
        // lane: a longer drain, 127 -> 134 ms), so auto takes it from 4 replicates per lane of its grid on.
        // ECDNA_SSA_SCHED = 0 default, 1 max-ILP, 2 auto, 3 the 128-VGPR build (K = 64 / u16; else 0).
        uint64_t max_chunk = 0;
        for (const auto& ch : c->chunks) max_chunk = std::max<uint64_t>(max_chunk, ch.n);
        const uint32_t kflags = kernel_flags(*p);
        const uint64_t sched = env_u64("ECDNA_SSA_SCHED", 2);
        // (auto only without f32 time and the event hash: that variant spills 12 B at 128 VGPRs)
        const bool k64u16 = c->bin_k == 64 && !c->bin_c32;
        const bool tf0 = (kflags & ecdna::kRuntimeFlagMask) == 0;
        // Where the max-ILP build keeps the default's occupancy (LDS bounds both: K = 32 / u32 and K = 64 / u32
        // since the f32 draw mapping v6, K = 256) it is taken too: its schedule then costs no lanes (C3 78.3 ->
        // 77.3 ms, C5 whole 31.9 -> 30.4 s, same box). With fewer than four replicates per lane of the default
        // grid it is taken even at one workgroup per CU less (K = 64 / u16, 118 against 134 VGPRs since v6: the
        // C4 8-GPU shard, two replicates per lane, 127 -> 119 ms), as the drain of the last replicates is
        // latency-bound (profiles/r04d_v6_suite_and_sched_sweep.txt).
        int occ_def = 0, occ_ilp = 0;
        CTX_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ_def, ecdna::bin_stepper_kernel(p->process, p->segregation, c->bin_k, c->bin_c32, kflags, 0),
            (int)c->stepper_block, 0));
        CTX_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &occ_ilp, ecdna::bin_stepper_kernel(p->process, p->segregation, c->bin_k, c->bin_c32, kflags, 1),
            (int)c->stepper_block, 0));
        // Paired lanes: with at most half a wave of replicates per SIMD (the C5 8-GPU shard) the
        // idle half of each wave computes the next event's Philox block and soft log in the N- fast-forward.
        // Birth-death without snapshots (the fast-forward's domain). ECDNA_SSA_PAIR = 0 off, 1 whenever
        // possible, 2 auto.
        const uint64_t pair_mode = env_u64("ECDNA_SSA_PAIR", 2);
        const bool pair_ok = p->process == ECDNA_BIRTH_DEATH && p->n_snapshots == 0 &&
                             ecdna::bin_stepper_kernel_pair(p->segregation, c->bin_k, c->bin_c32, kflags) != nullptr;
        c->bin_ilp = bin_schedule_rule(pair_ok, pair_mode, sched, max_chunk, c->cus, k64u16, tf0, occ_def, occ_ilp,
                                       c->stepper_block);
        // bin store: LDS-resident events, bounded by issue and LDS latency: every resident block helps
        CTX_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu,
            ecdna::bin_stepper_kernel(p->process, p->segregation, c->bin_k, c->bin_c32, kflags, c->bin_ilp),
            (int)c->stepper_block, 0));
    } else {
        CTX_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per_cu, ecdna::stepper_kernel(p->process, p->segregation, c->window), ecdna::kStepperBlock, 0));
        // Memory-level parallelism of the random row accesses saturates HBM at about 3 resident 256-lane
        // blocks per CU (C3 sweep, DESIGN.md §8: 1/2/3/4/7 blocks -> 617/372/329/336/349 ms); fewer
        // lanes also mean more replicates per lane and a shorter drain once the work queue is empty.
        per_cu = std::min(per_cu, 3);
    }
    uint64_t bpc = env_u64("ECDNA_SSA_BLOCKS_PER_CU", 0);
    if (bpc) per_cu = (int)bpc;
    if (per_cu < 1) per_cu = 1;
    c->stepper_blocks_cap = (uint32_t)(per_cu * c->cus);
    if (p->max_workgroups) c->stepper_blocks_cap = std::min(c->stepper_blocks_cap, p->max_workgroups);
    uint64_t max_blocks = env_u64("ECDNA_SSA_MAX_BLOCKS", 0);  // testing: force lane refill
    if (max_blocks) c->stepper_blocks_cap = (uint32_t)std::min<uint64_t>(c->stepper_blocks_cap, max_blocks);

    // Replicate rotation (bin store, 256-lane blocks): on when lanes have at least three
    // replicates each (ECDNA_SSA_ROTATE = 0 off, 1 on whenever possible, 2 auto); with two (C4 8-GPU shard)
    // the drain control is faster (74 ms against 84). Auto also leaves it off when the caller gave a cost
    // hint: the costliest-first start order then already balances the lanes, and parking only mixes the
    // order up again (C4 whole sweep, same box: 710-718 ms without rotation against 738-750 with it under
    // the 128-VGPR build, 747-749 against 792-805 under the default one). Results do not depend on it.
    // Byte offsets into bags/park are u32 in the kernel: chunks stay below 2 GiB of either.
    uint64_t rot_mode = env_u64("ECDNA_SSA_ROTATE", 2);
    const bool hinted = c->d_order != nullptr;
    // Rotation hands a parked replicate only to lanes of the same partition, partition = XCC id mod
    // kRotParts, and relies on those lanes sharing one L2 (the parked state is read with L1-bypassing
    // loads). That holds when the agent has at most kRotParts XCCs (gfx950 SPX: 8, CPX: 1); otherwise
    // two L2s would share a partition, so rotation stays off.
    {
        int xccs = 0;
        if (hipDeviceGetAttribute(&xccs, hipDeviceAttributeNumberOfXccs, c->device) != hipSuccess || xccs < 1 ||
            xccs > (int)ecdna::kRotParts)
            rot_mode = 0;
    }
    c->rot_tick_log2 = (uint32_t)std::min<uint64_t>(env_u64("ECDNA_SSA_ROT_TICK", 10), 30);
    bool any_rot = false;
    for (auto& ch : c->chunks) {
        const uint64_t need = (ch.n + c->stepper_block - 1) / c->stepper_block;
        const uint64_t lanes = std::max<uint64_t>(1, std::min<uint64_t>(need, c->stepper_blocks_cap)) * c->stepper_block;
        const bool ok = c->bin_k && c->stepper_block == ecdna::kStepperBlock &&
                        (uint64_t)ch.n * std::max<uint64_t>(bag_bytes, ecdna::kParkVecs * 16u) < (1ull << 31);
        if (!ok || rot_mode == 0 || (rot_mode == 2 && (ch.n < 3 * lanes || hinted))) continue;
        const uint32_t per = (ch.n + ecdna::kRotParts - 1) / ecdna::kRotParts;
        ch.rot_n_pad = (per + ecdna::kRotBlock - 1) / ecdna::kRotBlock * ecdna::kRotBlock;
        ch.rot_init.assign(ecdna::kRotParts, ecdna::RotPart{});
        for (uint32_t x = 0; x < ecdna::kRotParts; ++x) {
            const int cnt = x < ch.n ? (int)((ch.n - x + ecdna::kRotParts - 1) / ecdna::kRotParts) : 0;  // r = x mod 8
            ch.rot_init[x].waiting = cnt;
            ch.rot_init[x].fresh = cnt;
        }
        any_rot = true;
    }
    if (any_rot) {
        const uint64_t n_pad_max = (c->chunk_reps + ecdna::kRotParts - 1) / ecdna::kRotParts + ecdna::kRotBlock;
        CTX_TRY(hipMalloc(&c->d_rot_parts, ecdna::kRotParts * sizeof(ecdna::RotPart)));
        CTX_TRY(hipMalloc(&c->d_rot_flags, ecdna::kRotParts * n_pad_max * sizeof(uint32_t)));
        CTX_TRY(hipMalloc(&c->d_rot_park, c->chunk_reps * ecdna::kParkVecs * sizeof(uint4)));
        // park only while at least 1.5 partition grids' worth of replicates wait; below that the lanes run
        // their replicates to the end (C3 sweep, DESIGN.md §5: 0.5 / 1 / 2 / 3 grids -> 88.2 / 87.2 / 87.1 / 97.5 ms)
        const uint64_t lanes_all = (uint64_t)c->stepper_blocks_cap * c->stepper_block;
        c->rot_park_min = (int32_t)env_u64("ECDNA_SSA_ROT_PARK_MIN",
                                           std::max<uint64_t>(1, lanes_all * 3 / 2 / ecdna::kRotParts));
    }
    // grid and drain control per chunk. Drain control (bin store, 256-lane blocks, one wave per SIMD per block):
    // when lanes run more than two replicates each, the youngest wave slot of every SIMD stops taking fresh
    // replicates once fewer than 1.5 grids' worth are left (C3: 105 -> 101 ms). ECDNA_SSA_ADMIT=0:
    // off. Rotation replaces it.
    for (auto& ch : c->chunks) {
        // (paired lanes: owners only)
        const uint32_t per_block = c->bin_ilp == 3 ? c->stepper_block / 2 : c->stepper_block;
        const uint32_t need = (ch.n + per_block - 1) / per_block;
        ch.blocks = std::max<uint32_t>(1, std::min<uint32_t>(need, c->stepper_blocks_cap));
        const uint64_t lanes = (uint64_t)ch.blocks * c->stepper_block;
        const uint32_t per_cu = c->cus ? (uint32_t)((ch.blocks + c->cus - 1) / c->cus) : 0u;
        if (!ch.rot_n_pad && c->bin_k && c->stepper_block == 256 && per_cu >= 2 && ch.n > 2 * lanes &&
            env_u64("ECDNA_SSA_ADMIT", 1)) {
            const uint32_t slots = (uint32_t)std::min<uint64_t>(env_u64("ECDNA_SSA_ADMIT_SLOTS", 1), per_cu - 1);
            ch.admit_slot = per_cu - std::max<uint32_t>(slots, 1u);
            const uint64_t x8 = env_u64("ECDNA_SSA_ADMIT_X8", 12);  // eighths of a grid (tuning)
            ch.admit_remaining = (uint32_t)std::min<uint64_t>(lanes * x8 / 8, ch.n);
        }
    }
    *out = c;
    return ECDNA_OK;
#undef CTX_TRY
}

int ecdna_ssa_ctx_set_outputs(ecdna_ssa_ctx* c, uint64_t* d_hist, ecdna_totals_t* d_totals) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    c->d_hist = d_hist ? d_hist : c->d_hist_own;
    c->d_tot = d_totals ? d_totals : c->d_tot_own;
    return ECDNA_OK;
}

int ecdna_ssa_ctx_launch(ecdna_ssa_ctx* c, void* stream) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;  // NULL = the default (null) stream
    const ecdna_ssa_params_t& p = c->p;
    const uint64_t nb = (uint64_t)p.n_param_sets * p.hist_bins;
    HIP_TRY(hipMemsetAsync(c->d_hist, 0, nb * sizeof(uint64_t), st));
    HIP_TRY(hipMemsetAsync(c->d_tot, 0, p.n_param_sets * sizeof(ecdna_totals_t), st));
    if (!c->chunks.empty())
        HIP_TRY(hipMemsetAsync(c->d_heads, 0, c->chunks.size() * sizeof(uint32_t), st));
    if (c->d_snap_meta)
        HIP_TRY(hipMemsetAsync(c->d_snap_meta, 0, p.n_replicates * p.n_snapshots * sizeof(ecdna_snapshot_t), st));

    for (size_t k = 0; k < c->chunks.size(); ++k) {
        Chunk& ch = c->chunks[k];
        ecdna::StepperArgs a{};
        a.rows = c->d_rows;
        a.summaries = c->d_summ + ch.first;
        a.head = c->d_heads + k;
        a.order = c->d_order ? c->d_order + ch.first : nullptr;
        a.rates = c->d_rates;
        a.init_copies = c->d_init;
        a.init_offsets = c->d_init_off;
        a.init_nminus_set = c->d_init_nm;
        a.row_stride = c->row_stride;
        a.seed = p.seed;
        const uint64_t stride = p.replicate_stride ? p.replicate_stride : 1u;
        a.rid0 = p.first_replicate + ch.first * stride;
        a.rid_stride = stride;
        a.reps_per_set = p.reps_per_set;
        a.max_cells = p.max_cells;
        a.init_nminus = p.init_nminus;
        a.max_time = p.max_time;
        a.max_time32 = (float)p.max_time;
        a.n = ch.n;
        a.init_nplus = p.init_nplus;
        a.max_iter = (uint32_t)p.max_iter;
        a.cell_cap = p.cell_cap;
        a.flags = kernel_flags(p);  // (with the internal snapshot bit: it selects the kernel instance)
        // (n- + n+) * 2 >= max_cells  <=>  n- + n+ >= ceil(max_cells / 2)
        a.stop_cells = (p.process == ECDNA_BIRTH_DEATH && (p.flags & ECDNA_FLAG_BD_CAP_COMPAT))
                           ? p.max_cells / 2 + (p.max_cells & 1)
                           : p.max_cells;
        a.n_snap = p.n_snapshots;
        a.snap_cells = c->d_snap_cells;
        a.snap_meta = c->d_snap_meta ? c->d_snap_meta + ch.first * p.n_snapshots : nullptr;
        a.snap_rows = c->d_snap_rows ? c->d_snap_rows + ch.first * p.n_snapshots * c->out_stride : nullptr;
        a.snap_stride = c->out_stride;
        a.big_cap = c->big_cap;
        a.bags = c->d_bags;
        const uint32_t blocks = ch.blocks;
        a.admit_slot = ch.admit_slot;  // (drain control, decided at create)
        a.admit_remaining = ch.admit_remaining;
        if (ch.rot_n_pad) {  // rotation replaces the drain control
            a.rot_parts = c->d_rot_parts;
            a.rot_flags = c->d_rot_flags;
            a.rot_park = c->d_rot_park;
            a.rot_n_pad = ch.rot_n_pad;
            a.rot_tick_log2 = c->rot_tick_log2;
            a.rot_park_min = c->rot_park_min;
            const uint64_t n_flags = (uint64_t)ecdna::kRotParts * ch.rot_n_pad;
            HIP_TRY(hipMemsetD32Async(c->d_rot_flags, ecdna::ROT_FRESH, ch.n, st));
            if (n_flags > ch.n)
                HIP_TRY(hipMemsetD32Async(c->d_rot_flags + ch.n, ecdna::ROT_DONE, n_flags - ch.n, st));
            HIP_TRY(hipMemcpyAsync(c->d_rot_parts, ch.rot_init.data(), ecdna::kRotParts * sizeof(ecdna::RotPart),
                                   hipMemcpyHostToDevice, st));
        }

        a.ref_key = c->d_ref_key;
        a.ref_btpe = c->d_ref_btpe;
        a.rng_words = c->d_rng_words ? c->d_rng_words + ch.first : nullptr;
        HIP_TRY(hipEventRecord(ch.ev[0], st));
        if (c->refdraws)
            HIP_TRY(ecdna::launch_refdraws(a, p.process, p.segregation, blocks, st));
        else if (c->bin_k)
            HIP_TRY(ecdna::launch_bin_stepper(a, p.process, p.segregation, c->bin_k, c->bin_c32, c->bin_ilp, blocks, st));
        else
            HIP_TRY(ecdna::launch_stepper(a, p.process, p.segregation, c->window, blocks, st));
        HIP_TRY(hipEventRecord(ch.ev[1], st));

        ecdna::HistArgs hsa{};
        hsa.rows = c->d_rows;
        hsa.summaries = c->d_summ + ch.first;
        hsa.hist = c->d_hist;
        hsa.totals = reinterpret_cast<unsigned long long*>(c->d_tot);
        hsa.row_stride = c->row_stride;
        hsa.rid0 = p.first_replicate + ch.first * stride;
        hsa.rid_stride = stride;
        hsa.reps_per_set = p.reps_per_set;
        hsa.n = ch.n;
        hsa.bins = p.hist_bins;
        // (eight workgroups per CU for either histogram pass: one per CU made the bin store's lane-per-replicate
        // pass no faster at C3, 0.29 -> 0.30 ms, and C4's 1,024 sets 5 -> 28 ms, each workgroup walking more sets)
        const uint32_t hist_blocks_max = (uint32_t)c->cus * 8u;
        uint32_t rpb = (ch.n + hist_blocks_max - 1) / hist_blocks_max;
        // at least one replicate per lane of a workgroup, or the chunk's replicates of one parameter set if fewer: small
        // runs otherwise spread over 2,048 workgroups of mostly idle waves, each adding its own nonzero bins to the
        // same global words (C2: 0.061 -> 0.023 ms per launch at 256, 0.038 at 64, 0.052 at 1,024;
        // profiles/r06ak_hist_rpb.txt); sweeps of small sets keep about one set per workgroup
        const uint64_t set_local = std::max<uint64_t>(1, p.reps_per_set / stride);
        const uint32_t rpb_min = (uint32_t)std::max<uint64_t>(4, std::min<uint64_t>(ecdna::kHistBlock, set_local));
        if (rpb < rpb_min) rpb = rpb_min;
        hsa.reps_per_block = rpb;
        hsa.stats = c->d_stats ? c->d_stats + ch.first : nullptr;
        hsa.target_cdf = c->d_target_cdf;
        hsa.target_mean = c->target_mean;
        hsa.target_entropy = c->target_entropy;
        hsa.target_freq = c->target_freq;
        hsa.has_target = c->has_target ? 1u : 0u;
        hsa.bags = c->d_bags;
        hsa.bag_k = c->bin_k;
        hsa.bag_c32 = (uint32_t)c->bin_c32;
        const uint32_t hblocks = (ch.n + rpb - 1) / rpb;
        HIP_TRY(ecdna::launch_hist(hsa, hblocks, st));
        HIP_TRY(hipEventRecord(ch.ev[2], st));
    }
    c->last_stream = st;
    c->launched = true;
    return ECDNA_OK;
}

int ecdna_ssa_ctx_sync(ecdna_ssa_ctx* c, float* ssa_ms, float* hist_ms) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "sync before launch");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    float s = 0.f, h = 0.f;
    for (auto& ch : c->chunks) {
        float a = 0.f, b = 0.f;
        HIP_TRY(hipEventElapsedTime(&a, ch.ev[0], ch.ev[1]));
        HIP_TRY(hipEventElapsedTime(&b, ch.ev[1], ch.ev[2]));
        s += a;
        h += b;
    }
    if (ssa_ms) *ssa_ms = s;
    if (hist_ms) *hist_ms = h;
    return ECDNA_OK;
}

int ecdna_ssa_ctx_device_outputs(ecdna_ssa_ctx* c, uint64_t** d_hist, ecdna_totals_t** d_totals) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (d_hist) *d_hist = c->d_hist;
    if (d_totals) *d_totals = c->d_tot;
    return ECDNA_OK;
}

int64_t ecdna_ssa_ctx_row_stride(const ecdna_ssa_ctx* c) {
    if (!c) return 0;
    return c->chunks.size() <= 1 ? (int64_t)c->out_stride : 0;
}

int ecdna_ssa_ctx_geometry(const ecdna_ssa_ctx* c, uint64_t* chunk_replicates, uint64_t* grid_lanes) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (chunk_replicates) *chunk_replicates = c->chunk_reps;
    if (grid_lanes) *grid_lanes = (uint64_t)c->stepper_blocks_cap * c->stepper_block;
    return ECDNA_OK;
}

int ecdna_ssa_ctx_instance(const ecdna_ssa_ctx* c, ecdna_ssa_instance_t* out) {
    if (!c || !out) return fail(ECDNA_E_INVALID, "ctx / out is NULL");
    const ecdna_ssa_params_t& p = c->p;
    ecdna_ssa_instance_t r{};
    const void* fn;
    if (c->refdraws) {
        r.kernel = ECDNA_KERNEL_REFDRAWS;
        r.schedule = -1;
        fn = ecdna::refdraws_kernel(p.process, p.segregation);
    } else if (c->bin_k) {
        r.kernel = ECDNA_KERNEL_BINS;
        r.schedule = c->bin_ilp;
        r.paired = c->bin_ilp == 3 ? 1 : 0;
        r.bin_kmax = c->bin_k;
        r.bin_c32 = (uint32_t)c->bin_c32;
        r.runtime_flags = (kernel_flags(p) & ecdna::kRuntimeFlagMask) ? 1 : 0;
        fn = ecdna::bin_stepper_kernel(p.process, p.segregation, c->bin_k, c->bin_c32, kernel_flags(p), c->bin_ilp);
    } else {
        r.kernel = ECDNA_KERNEL_ROWS;
        r.schedule = -1;
        r.window = (uint32_t)c->window;
        r.runtime_flags = 1;
        fn = ecdna::stepper_kernel(p.process, p.segregation, c->window);
    }
    for (const auto& ch : c->chunks) {
        r.rotation += ch.rot_n_pad ? 1 : 0;
        r.drain_control += ch.admit_slot != 0xffffffffu ? 1 : 0;
    }
    r.rot_tick_log2 = (int32_t)c->rot_tick_log2;
    r.cost_order = c->d_order ? 1 : 0;
    r.block_lanes = c->stepper_block;
    r.cus = (uint32_t)c->cus;
    // the grid actually launched (the largest chunk's; a small or paired run launches fewer blocks than the
    // occupancy cap), and its workgroups per CU rounded up
    uint32_t launched = 0;
    for (const auto& ch : c->chunks) launched = std::max<uint32_t>(launched, ch.blocks);
    r.blocks_per_cu = c->cus ? (launched + (uint32_t)c->cus - 1u) / (uint32_t)c->cus : 0u;
    r.n_chunks = (uint32_t)c->chunks.size();
    r.chunk_replicates = c->chunk_reps;
    r.grid_lanes = (uint64_t)launched * c->stepper_block;
    hipFuncAttributes fa{};
    if (fn && hipFuncGetAttributes(&fa, fn) == hipSuccess) {
        r.vgprs = (uint32_t)fa.numRegs;
        r.lds_bytes = (uint32_t)fa.sharedSizeBytes;
        r.scratch_bytes = (uint32_t)fa.localSizeBytes;
    }
    *out = r;
    return ECDNA_OK;
}

int ecdna_ssa_ctx_download(ecdna_ssa_ctx* c, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                           ecdna_totals_t* out_totals, uint16_t* out_rows) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "download before launch");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    const ecdna_ssa_params_t& p = c->p;
    if (out_summaries && p.n_replicates)
        HIP_TRY(hipMemcpy(out_summaries, c->d_summ, p.n_replicates * sizeof(ecdna_rep_summary_t),
                          hipMemcpyDeviceToHost));
    if (out_hist)
        HIP_TRY(hipMemcpy(out_hist, c->d_hist, (uint64_t)p.n_param_sets * p.hist_bins * sizeof(uint64_t),
                          hipMemcpyDeviceToHost));
    if (out_totals)
        HIP_TRY(hipMemcpy(out_totals, c->d_tot, p.n_param_sets * sizeof(ecdna_totals_t), hipMemcpyDeviceToHost));
    if (out_rows) {
        if (c->chunks.size() > 1) return fail(ECDNA_E_STATE, "rows are not downloadable from a chunked run");
        if (p.n_replicates && !c->bin_k)
            HIP_TRY(hipMemcpy(out_rows, c->d_rows, p.n_replicates * c->row_stride * sizeof(uint16_t),
                              hipMemcpyDeviceToHost));
        if (c->bin_k && p.n_replicates) {
            std::vector<uint16_t> dev_rows(p.n_replicates * c->row_stride);  // the large-k rows
            HIP_TRY(hipMemcpy(dev_rows.data(), c->d_rows, dev_rows.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
            // bin store: canonical rows = the counters expanded (k ascending), then the large-k row
            std::vector<ecdna_rep_summary_t> summ(p.n_replicates);
            HIP_TRY(hipMemcpy(summ.data(), c->d_summ, p.n_replicates * sizeof(ecdna_rep_summary_t),
                              hipMemcpyDeviceToHost));
            const uint64_t kb = c->bin_k;
            std::vector<uint32_t> bags(p.n_replicates * kb);
            if (c->bin_c32) {
                HIP_TRY(hipMemcpy(bags.data(), c->d_bags, bags.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
            } else {
                std::vector<uint16_t> b16(bags.size());
                HIP_TRY(hipMemcpy(b16.data(), c->d_bags, b16.size() * sizeof(uint16_t), hipMemcpyDeviceToHost));
                std::copy(b16.begin(), b16.end(), bags.begin());
            }
            std::vector<uint16_t> big;
            for (uint64_t i = 0; i < p.n_replicates; ++i) {
                uint16_t* r = out_rows + i * c->out_stride;
                const uint16_t* dr = dev_rows.data() + i * c->row_stride;
                uint64_t small = 0;
                for (uint64_t b = 0; b < kb; ++b) small += bags[i * kb + b];
                const uint64_t nbig = std::min<uint64_t>(summ[i].nplus >= small ? summ[i].nplus - small : 0,
                                                         c->row_stride);
                big.assign(dr, dr + nbig);
                uint64_t pos = 0;
                for (uint64_t b = 0; b < kb; ++b)
                    for (uint32_t q = 0; q < bags[i * kb + b] && pos < c->out_stride; ++q) r[pos++] = (uint16_t)(b + 1);
                const uint64_t tail = std::min<uint64_t>(big.size(), c->out_stride - pos);
                std::copy(big.begin(), big.begin() + tail, r + pos);
            }
        }
    }
    return ECDNA_OK;
}

int ecdna_ssa_ctx_download_snapshots(ecdna_ssa_ctx* c, ecdna_snapshot_t* meta, uint16_t* rows) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "download before launch");
    const ecdna_ssa_params_t& p = c->p;
    if (!p.n_snapshots || !p.n_replicates) return ECDNA_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    const uint64_t ns = p.n_replicates * p.n_snapshots;
    if (meta) HIP_TRY(hipMemcpy(meta, c->d_snap_meta, ns * sizeof(ecdna_snapshot_t), hipMemcpyDeviceToHost));
    if (rows) {
        if (!c->d_snap_rows) return fail(ECDNA_E_STATE, "snapshot rows need ECDNA_FLAG_SNAPSHOT_ROWS");
        HIP_TRY(hipMemcpy(rows, c->d_snap_rows, ns * c->out_stride * sizeof(uint16_t), hipMemcpyDeviceToHost));
    }
    return ECDNA_OK;
}

int ecdna_ssa_ctx_download_stats(ecdna_ssa_ctx* c, ecdna_rep_stats_t* out) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "download before launch");
    if (!c->d_stats) return fail(ECDNA_E_STATE, "statistics need ECDNA_FLAG_REP_STATS");
    if (!out || !c->p.n_replicates) return ECDNA_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipMemcpy(out, c->d_stats, c->p.n_replicates * sizeof(ecdna_rep_stats_t), hipMemcpyDeviceToHost));
    return ECDNA_OK;
}

int ecdna_ssa_ctx_download_rng_words(ecdna_ssa_ctx* c, uint64_t* out) {
    if (!c) return fail(ECDNA_E_INVALID, "ctx is NULL");
    if (!c->launched) return fail(ECDNA_E_STATE, "download before launch");
    if (!c->d_rng_words) return fail(ECDNA_E_STATE, "stream positions need ECDNA_FLAG_REFERENCE_DRAWS");
    if (!out || !c->p.n_replicates) return ECDNA_OK;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->last_stream));
    HIP_TRY(hipMemcpy(out, c->d_rng_words, c->p.n_replicates * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return ECDNA_OK;
}

int ecdna_ssa_ctx_destroy(ecdna_ssa_ctx* c) {
    free_ctx(c);
    return ECDNA_OK;
}

int ecdna_ssa_run(const ecdna_ssa_params_t* p, ecdna_rep_summary_t* out_summaries, uint64_t* out_hist,
                  ecdna_totals_t* out_totals, void* stream) {
    ecdna_ssa_ctx* c = nullptr;
    int rc = ecdna_ssa_ctx_create(p, &c);
    if (rc) return rc;
    rc = ecdna_ssa_ctx_launch(c, stream);
    if (!rc) rc = ecdna_ssa_ctx_download(c, out_summaries, out_hist, out_totals, nullptr);
    ecdna_ssa_ctx_destroy(c);
    return rc;
}

}  // extern "C"
