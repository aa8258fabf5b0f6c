// pmc_calib.hip — calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the SSA stepper's
// access shapes (MI355X_MICROARCH.md §HBM: "calibrate on a known byte count in your own access
// pattern before trusting an absolute"). Each kernel makes a KNOWN number of accesses to a 4 GiB
// buffer (far beyond the 256 MiB Infinity Cache):
//   rand_load_u16   : one random 2-B load per lane-iteration (+ one 4-B store per lane at the end)
//   rand_store_u16  : one random 2-B store per lane-iteration
//   rand_rmw_u16    : random 2-B load, then a 2-B store to the same address (the swap_remove slot)
//   stream_load_x4  : 16 B per lane, coalesced, whole buffer once (the guide's reference shape)
// Output: one line per kernel with the access count; divide rocprofv3's per-dispatch FETCH_SIZE /
// WRITE_SIZE (KiB) by it to get bytes per access.
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

__global__ void rand_load_u16(const uint16_t* buf, uint64_t mask, int iters, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) acc += buf[mix(tid * 1315423911ull + i) & mask];
    out[tid] = acc;
}

__global__ void rand_store_u16(uint16_t* buf, uint64_t mask, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; ++i) buf[mix(tid * 2654435761ull + i) & mask] = (uint16_t)i;
}

__global__ void rand_rmw_u16(uint16_t* buf, uint64_t mask, int iters) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    for (int i = 0; i < iters; ++i) {
        const uint64_t j = mix(tid * 40503ull + i) & mask;
        buf[j] = (uint16_t)(buf[j] + 1);
    }
}

__global__ void stream_load_x4(const uint4* buf, uint64_t n, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = tid; i < n; i += stride) {
        const uint4 v = buf[i];
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    out[tid] = acc;
}

int main() {
    const uint64_t bytes = 4ull << 30;
    const uint64_t n16 = bytes / 2, mask = n16 - 1;
    uint16_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    const int blocks = 256 * 16, threads = 256, iters = 64;
    const uint64_t lanes = (uint64_t)blocks * threads;
    CK(hipMalloc(&out, lanes * sizeof(uint32_t)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;

    CK(hipEventRecord(a));
    rand_load_u16<<<blocks, threads>>>(buf, mask, iters, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("rand_load_u16 accesses=%llu out_store_bytes=%llu ms=%.3f\n", (unsigned long long)(lanes * iters),
                (unsigned long long)(lanes * 4), ms);

    CK(hipEventRecord(a));
    rand_store_u16<<<blocks, threads>>>(buf, mask, iters);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("rand_store_u16 accesses=%llu ms=%.3f\n", (unsigned long long)(lanes * iters), ms);

    CK(hipEventRecord(a));
    rand_rmw_u16<<<blocks, threads>>>(buf, mask, iters);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("rand_rmw_u16 accesses=%llu ms=%.3f\n", (unsigned long long)(lanes * iters), ms);

    CK(hipEventRecord(a));
    stream_load_x4<<<blocks, threads>>>((const uint4*)buf, bytes / 16, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("stream_load_x4 bytes=%llu ms=%.3f GB/s=%.1f\n", (unsigned long long)bytes, ms, bytes / ms / 1e6);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
