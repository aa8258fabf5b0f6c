// chain_probe.hip — per-lane dependent chains of the stepper's memory shape at a latency-bound lane
// count (C5 shard: 32,768 lanes, 2 MB regions), to see what the in-order vmcnt costs:
//   0 load        : v = row[j_i]                                   (load latency only)
//   1 rmw         : v = row[j_i]; row[j_i] = v + 1                 (the next load waits for this store)
//   2 rmw_pf      : row[j_{i+1}] loaded before the store of step i, compiler waits (vmcnt(0))
//   3 rmw_pf_cnt  : the same, the load in inline asm and a counted s_waitcnt vmcnt(1): the store of
//                   step i may still be in flight when step i+1 uses its value
// Indices j_i depend on i and on the previous value (so the chain is real); in 2 and 3 j_{i+1} is
// known one step early (as the stepper's next cell is, from the counter-based RNG).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e = (x);                                                                     \
        if (e != hipSuccess) {                                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

template <int MODE>
__global__ void __launch_bounds__(256) chain(uint16_t* buf, uint64_t cells, int iters, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint16_t* row = buf + tid * cells;
    uint32_t acc = 0;
    auto idx = [&](int i) -> uint64_t { return (mix(tid * 0x9e3779b97f4a7c15ull + (uint64_t)i) >> 11) % cells; };
    if (MODE == 0) {
        for (int i = 0; i < iters; ++i) acc += row[(idx(i) + (acc & 1)) % cells];
    } else if (MODE == 1) {
        for (int i = 0; i < iters; ++i) {
            const uint64_t j = (idx(i) + (acc & 1)) % cells;
            const uint32_t v = row[j];
            row[j] = (uint16_t)(v + 1);
            acc += v;
        }
    } else if (MODE == 2) {
        uint64_t j = idx(0);
        uint32_t v = row[j];
        for (int i = 0; i < iters; ++i) {
            const uint64_t jn = idx(i + 1);
            const uint32_t vn = *(const __attribute__((address_space(1))) uint16_t*)(row + jn);
            if (jn != j) row[j] = (uint16_t)(v + 1);
            acc += v;
            j = jn;
            v = vn;
        }
    } else {
        uint64_t j = idx(0);
        uint32_t v;
        const uint16_t* p0 = row + j;
        asm volatile("global_load_ushort %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p0) : "memory");
        for (int i = 0; i < iters; ++i) {
            const uint64_t jn = idx(i + 1);
            uint32_t vn;
            const uint16_t* pn = row + jn;
            asm volatile("global_load_ushort %0, %1, off" : "=v"(vn) : "v"(pn) : "memory");
            uint16_t* pj = row + j;
            const uint32_t nv = (jn != j) ? (v + 1u) : v;  // same cell: the store must not race the load
            asm volatile("global_store_short %0, %1, off" ::"v"(pj), "v"(nv) : "memory");
            acc += v;
            asm volatile("s_waitcnt vmcnt(1)" : "+v"(vn)::"memory");
            j = jn;
            v = vn;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    out[tid] = acc;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t region = 2000000, cells = region / 2;
    const int lane_blocks[] = {128, 256, 768};
    const uint64_t max_lanes = 768ull * 256;
    const uint64_t bytes = 32768ull * region;  // 65.5 GB; larger lane counts use smaller regions
    uint16_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    CK(hipMalloc(&out, max_lanes * sizeof(uint32_t)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"load", "rmw", "rmw_pf", "rmw_pf_cnt"};
    for (int lb : lane_blocks) {
        const uint64_t lanes = (uint64_t)lb * 256;
        const uint64_t c = bytes / 2 / lanes < cells ? bytes / 2 / lanes : cells;
        for (int m = 0; m < 4; ++m) {
            auto k = m == 0 ? chain<0> : m == 1 ? chain<1> : m == 2 ? chain<2> : chain<3>;
            const int iters = 512;
            hipLaunchKernelGGL(k, dim3(lb), dim3(256), 0, 0, buf, c, 8, out);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k, dim3(lb), dim3(256), 0, 0, buf, c, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("{\"mode\": \"%s\", \"lanes\": %llu, \"region_bytes\": %llu, \"ms\": %.3f, \"ops_per_s\": %.4g, "
                        "\"ns_per_op_per_lane\": %.1f}\n",
                        names[m], (unsigned long long)lanes, (unsigned long long)(c * 2), ms,
                        lanes * (double)iters / (ms * 1e-3), ms * 1e6 / iters);
        }
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
