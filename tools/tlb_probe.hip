// tlb_probe.hip — random 2-B loads and stores where each lane stays inside its own region of R bytes
// (its "row"), at the stepper's lane counts. Regions are laid out back to back, so the footprint is
// lanes x R. This separates the HBM transaction limit from address-translation (UTCL1/UTCL2) reach:
// C3's rows are ~20 KB (4 GB active), C5's ~2 MB (64 GB active for a 32,768-replicate shard).
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
__global__ void __launch_bounds__(256) region(uint16_t* buf, uint64_t cells, int iters, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint16_t* row = buf + tid * cells;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const uint64_t j = (mix(tid * 0x9e3779b97f4a7c15ull + (uint64_t)i * 7919u + acc) >> 11) % cells;
        if (MODE == 0) {
            acc += row[j];
        } else {
            const uint32_t v = row[j];
            row[j] = (uint16_t)(v + 1);
            acc += v;
        }
    }
    out[tid] = acc;
}

int main() {
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t max_bytes = 72ull << 30;
    uint16_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, max_bytes));
    CK(hipMemset(buf, 1, max_bytes));
    CK(hipMalloc(&out, (uint64_t)cus * 4 * 256 * sizeof(uint32_t)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const uint64_t regions[] = {2048, 20480, 204800, 2000000};
    const int lane_blocks[] = {128, 768};  // 32,768 and 196,608 lanes
    for (int mode = 0; mode < 2; ++mode)
        for (int lb : lane_blocks)
            for (uint64_t r : regions) {
                const uint64_t lanes = (uint64_t)lb * 256;
                if (lanes * r > max_bytes) continue;
                const uint64_t cells = r / 2;
                const int iters = 256;
                auto k = mode == 0 ? region<0> : region<1>;
                hipLaunchKernelGGL(k, dim3(lb), dim3(256), 0, 0, buf, cells, 8, out);
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(k, dim3(lb), dim3(256), 0, 0, buf, cells, iters, out);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                std::printf("{\"op\": \"%s\", \"lanes\": %llu, \"region_bytes\": %llu, \"footprint_gb\": %.2f, "
                            "\"ms\": %.3f, \"ops_per_s\": %.4g, \"ns_per_op_per_lane\": %.1f}\n",
                            mode == 0 ? "load_u16" : "rmw_u16", (unsigned long long)lanes, (unsigned long long)r,
                            lanes * r / 1e9, ms, lanes * (double)iters / (ms * 1e-3), ms * 1e6 / iters);
            }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
