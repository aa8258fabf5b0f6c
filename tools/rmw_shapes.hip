// rmw_shapes.hip — access-shape microbenchmark for the stepper's random row traffic (timing only).
// The stepper's ProliferateNPlus is a random 2-B read-modify-write of one row cell; DeathNPlus is a
// random 2-B store. This measures, on a 4 GiB buffer (far beyond the 256 MiB Infinity Cache) and at
// several resident-lane counts, how many such operations per second the chip sustains for:
//   load_u16      random 2-B load
//   store_u16     random 2-B store
//   rmw_u16       random 2-B load + 2-B store to the same address (the stepper today)
//   rmw_nt_u16    the same with a nontemporal store
//   rmw_x4        16-B aligned load + 16-B store of the block holding the cell (full 16-B write)
//   rmw_32        32-B sector: two 16-B loads + two 16-B stores (full-sector write)
//   rmw_64        64-B: four 16-B loads + four 16-B stores
//   store_32      32-B sector store, no load
// Every lane runs `iters` dependent iterations (the next index depends on the loaded value, like
// the stepper's next event on the previous one), so the rate is latency x parallelism limited
// exactly as the stepper is.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

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
__global__ void __launch_bounds__(256) shape(uint16_t* buf, uint64_t mask16, int iters, uint32_t* out) {
    const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int i = 0; i < iters; ++i) {
        const uint64_t j = mix(tid * 0x9e3779b97f4a7c15ull + (uint64_t)i * 7919u + acc) & mask16;
        if (MODE == 0) {
            acc += buf[j];
        } else if (MODE == 1) {
            buf[j] = (uint16_t)(i + tid);
            acc += 1;
        } else if (MODE == 2) {
            const uint32_t v = buf[j];
            buf[j] = (uint16_t)(v + 1);
            acc += v;
        } else if (MODE == 3) {
            const uint32_t v = buf[j];
            __builtin_nontemporal_store((uint16_t)(v + 1), buf + j);
            acc += v;
        } else if (MODE == 4) {
            uint4* p = reinterpret_cast<uint4*>(buf + (j & ~7ull));
            uint4 v = *p;
            v.x += 1;
            *p = v;
            acc += v.y;
        } else if (MODE == 5) {
            uint4* p = reinterpret_cast<uint4*>(buf + (j & ~15ull));
            uint4 v0 = p[0], v1 = p[1];
            v0.x += 1;
            p[0] = v0;
            p[1] = v1;
            acc += v1.y;
        } else if (MODE == 6) {
            uint4* p = reinterpret_cast<uint4*>(buf + (j & ~31ull));
            uint4 v0 = p[0], v1 = p[1], v2 = p[2], v3 = p[3];
            v0.x += 1;
            p[0] = v0;
            p[1] = v1;
            p[2] = v2;
            p[3] = v3;
            acc += v3.y;
        } else if (MODE == 7) {
            uint4* p = reinterpret_cast<uint4*>(buf + (j & ~15ull));
            const uint4 v = make_uint4(i, tid, 0, 0);
            p[0] = v;
            p[1] = v;
            acc += 1;
        }
    }
    out[tid] = acc;
}

typedef void (*kfn)(uint16_t*, uint64_t, int, uint32_t*);

int main(int argc, char** argv) {
    const uint64_t bytes = 4ull << 30;
    const uint64_t mask16 = bytes / 2 - 1;
    uint16_t* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int max_bpc = 8;
    CK(hipMalloc(&out, (uint64_t)cus * max_bpc * 256 * sizeof(uint32_t)));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char* names[] = {"load_u16", "store_u16", "rmw_u16", "rmw_nt_u16", "rmw_x4", "rmw_32", "rmw_64", "store_32"};
    kfn fns[] = {shape<0>, shape<1>, shape<2>, shape<3>, shape<4>, shape<5>, shape<6>, shape<7>};
    const int bpcs[] = {1, 2, 3, 4, 8};
    const int iters = argc > 1 ? std::atoi(argv[1]) : 256;
    for (int m = 0; m < 8; ++m) {
        for (int bpc : bpcs) {
            const int blocks = cus * bpc;
            const uint64_t lanes = (uint64_t)blocks * 256;
            hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, buf, mask16, 8, out);  // warm
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(fns[m], dim3(blocks), dim3(256), 0, 0, buf, mask16, iters, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double ops = (double)lanes * iters;
            std::printf("{\"shape\": \"%s\", \"blocks_per_cu\": %d, \"lanes\": %llu, \"ms\": %.3f, \"ops_per_s\": %.4g, "
                        "\"ns_per_op_per_lane\": %.1f}\n",
                        names[m], bpc, (unsigned long long)lanes, ms, ops / (ms * 1e-3), ms * 1e6 / iters);
        }
    }
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
