// ssa_comm.cpp — the multi-GPU reduction of the C ABI (include/ecdna_ssa.h, ABI v6): communicators and the
// all-reduce of a run's copy-number histogram and totals over RCCL (xGMI between the GPUs of a node).
//
// The reference's only parallelism is independent replicates (rayon over replicate ids, src/main.rs:221-224);
// here replicates shard over GPUs by global id and the shards' outputs are plain integer sums, so the whole
// run's histogram and totals are one ncclAllReduce(ncclUint64, ncclSum) of [n_param_sets * hist_bins] +
// [n_param_sets * 16] words (~8 KiB per set, 8 MiB for the 1024-set ABC sweep) — exact and
// independent of the reduction order.
//
// RCCL is loaded on first use (dlopen of librccl.so.1): the engine itself runs without it, and in a process
// that already loaded torch's RCCL the soname resolves to that copy, so a caller-made communicator and these
// calls use one library.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "../../include/ecdna_ssa.h"

// from ssa_api.cpp (library-internal)
__attribute__((visibility("hidden"))) int ecdna_ssa_internal_fail(int code, const std::string& msg);
__attribute__((visibility("hidden"))) int ecdna_ssa_internal_ctx_outputs(ecdna_ssa_ctx* c, uint64_t** d_hist, ecdna_totals_t** d_tot, uint32_t* n_sets,
                                   uint32_t* bins, int* device, void** stream);

namespace {

struct Rccl {
    bool ok = false;
    std::string why;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
        bool all = true;
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
            all &= fn != nullptr;
        };
        sym(r.get_unique_id, "ncclGetUniqueId");
        sym(r.init_rank, "ncclCommInitRank");
        sym(r.init_all, "ncclCommInitAll");
        sym(r.destroy, "ncclCommDestroy");
        sym(r.all_reduce, "ncclAllReduce");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
        r.ok = all;
        if (!all) r.why = "librccl.so.1 lacks an expected symbol";
    });
    return r;
}

int need_rccl() {
    Rccl& r = rccl();
    return r.ok ? ECDNA_OK : ecdna_ssa_internal_fail(ECDNA_E_COMM, r.why);
}

int nccl_fail(ncclResult_t e, const char* what) {
    return ecdna_ssa_internal_fail(ECDNA_E_COMM, std::string(what) + ": " + rccl().error_string(e));
}

}  // namespace

extern "C" {

int ecdna_ssa_comm_unique_id(uint8_t out_id[ECDNA_COMM_ID_BYTES]) {
    if (!out_id) return ecdna_ssa_internal_fail(ECDNA_E_INVALID, "out_id is NULL");
    if (int rc = need_rccl()) return rc;
    static_assert(sizeof(ncclUniqueId) == ECDNA_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId id;
    if (ncclResult_t e = rccl().get_unique_id(&id)) return nccl_fail(e, "ncclGetUniqueId");
    std::memcpy(out_id, &id, sizeof(id));
    return ECDNA_OK;
}

int ecdna_ssa_comm_init_rank(const uint8_t id[ECDNA_COMM_ID_BYTES], int n_ranks, int rank, int device,
                             void** out_comm) {
    if (!id || !out_comm || n_ranks < 1 || rank < 0 || rank >= n_ranks)
        return ecdna_ssa_internal_fail(ECDNA_E_INVALID, "comm_init_rank: bad arguments");
    *out_comm = nullptr;
    if (int rc = need_rccl()) return rc;
    if (hipSetDevice(device) != hipSuccess) return ecdna_ssa_internal_fail(ECDNA_E_NODEVICE, "hipSetDevice failed");
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    if (ncclResult_t e = rccl().init_rank(&comm, n_ranks, uid, rank)) return nccl_fail(e, "ncclCommInitRank");
    *out_comm = comm;
    return ECDNA_OK;
}

int ecdna_ssa_comm_init_all(int n_devices, const int* devices, void** out_comms) {
    if (n_devices < 1 || !devices || !out_comms)
        return ecdna_ssa_internal_fail(ECDNA_E_INVALID, "comm_init_all: bad arguments");
    if (int rc = need_rccl()) return rc;
    ncclComm_t* comms = reinterpret_cast<ncclComm_t*>(out_comms);
    if (ncclResult_t e = rccl().init_all(comms, n_devices, devices)) return nccl_fail(e, "ncclCommInitAll");
    return ECDNA_OK;
}

int ecdna_ssa_comm_destroy(void* comm) {
    if (!comm) return ECDNA_OK;
    if (int rc = need_rccl()) return rc;
    if (ncclResult_t e = rccl().destroy(reinterpret_cast<ncclComm_t>(comm))) return nccl_fail(e, "ncclCommDestroy");
    return ECDNA_OK;
}

int ecdna_ssa_reduce_hist(void* comm, uint64_t* d_hist, ecdna_totals_t* d_totals, uint32_t n_param_sets,
                          uint32_t hist_bins, void* stream) {
    if (!comm || !d_hist || !d_totals || n_param_sets == 0 || hist_bins == 0)
        return ecdna_ssa_internal_fail(ECDNA_E_INVALID, "reduce_hist: bad arguments");
    if (int rc = need_rccl()) return rc;
    Rccl& r = rccl();
    ncclComm_t cm = reinterpret_cast<ncclComm_t>(comm);
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const size_t nh = (size_t)n_param_sets * hist_bins, nt = (size_t)n_param_sets * (sizeof(ecdna_totals_t) / 8);
    if (ncclResult_t e = r.group_start()) return nccl_fail(e, "ncclGroupStart");
    ncclResult_t e1 = r.all_reduce(d_hist, d_hist, nh, ncclUint64, ncclSum, cm, st);
    ncclResult_t e2 = r.all_reduce(d_totals, d_totals, nt, ncclUint64, ncclSum, cm, st);
    ncclResult_t e3 = r.group_end();
    if (e1) return nccl_fail(e1, "ncclAllReduce(histogram)");
    if (e2) return nccl_fail(e2, "ncclAllReduce(totals)");
    if (e3) return nccl_fail(e3, "ncclGroupEnd");
    return ECDNA_OK;
}

int ecdna_ssa_ctx_reduce(ecdna_ssa_ctx* c, void* comm) {
    uint64_t* h = nullptr;
    ecdna_totals_t* t = nullptr;
    uint32_t sets = 0, bins = 0;
    int device = 0;
    void* stream = nullptr;
    if (int rc = ecdna_ssa_internal_ctx_outputs(c, &h, &t, &sets, &bins, &device, &stream)) return rc;
    if (hipSetDevice(device) != hipSuccess) return ecdna_ssa_internal_fail(ECDNA_E_HIP, "hipSetDevice failed");
    return ecdna_ssa_reduce_hist(comm, h, t, sets, bins, stream);
}

}  // extern "C"
