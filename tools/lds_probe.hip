// Co-residency vs static LDS size: a latency-bound LDS pointer chase per block; the kernel time with
// R blocks per CU over the time with 1 block per CU tells how many blocks really run at once.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int BYTES>
__global__ void __launch_bounds__(256) k_lds(uint32_t* out, int spin) {
    __shared__ uint32_t buf[BYTES / 4];
    const int t = threadIdx.x;
    constexpr int N = BYTES / 4;
    for (int i = t; i < N; i += 256) buf[i] = (i * 97u + 1u) % N;
    __syncthreads();
    uint32_t idx = t;
    for (int i = 0; i < spin; ++i) idx = buf[idx];
    if (idx == 0xffffffffu) out[0] = idx;
}

template <int BYTES>
void run(int cus) {
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k_lds<BYTES>, 256, 0);
    uint32_t* d;
    hipMalloc(&d, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float ms[9] = {0};
    for (int r : {1, 2, 3, 4, 6, 8}) {
        hipLaunchKernelGGL(k_lds<BYTES>, dim3(cus * r), dim3(256), 0, 0, d, 20000);  // warm
        hipEventRecord(a);
        hipLaunchKernelGGL(k_lds<BYTES>, dim3(cus * r), dim3(256), 0, 0, d, 20000);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms[r], a, b);
    }
    printf("LDS %6d B/block (runtime occupancy %d): time ratio vs 1 block/CU at 2,3,4,6,8 blocks/CU: %.2f %.2f %.2f %.2f %.2f  (1/CU %.3f ms)\n",
           BYTES, occ, ms[2] / ms[1], ms[3] / ms[1], ms[4] / ms[1], ms[6] / ms[1], ms[8] / ms[1], ms[1]);
    hipFree(d);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    printf("%s maxSharedMemoryPerMultiProcessor=%zu CUs=%d\n", p.gcnArchName, p.maxSharedMemoryPerMultiProcessor,
           p.multiProcessorCount);
    run<8192>(p.multiProcessorCount);
    run<16384>(p.multiProcessorCount);
    run<32768>(p.multiProcessorCount);
    run<36864>(p.multiProcessorCount);
    run<53248>(p.multiProcessorCount);
    run<65536>(p.multiProcessorCount);
    return 0;
}
