// Exhaustive check of the time step's reciprocal on the GPU: for every f32 b in [2^-60, 2^95) (every total propensity
// the stepper can divide by: rates 0 or in [2^-60, 2^60], u32 populations), the device sequence
// rcp_rn (ecdna-evo_amd/csrc/ssa_device.hpp: y1 = fma(fma(-b, r, 1), r, r), r = v_rcp_f32(b)) against RN32(1 / b) (the f64 quotient rounded to f32: 1 / b is never
// within 2^-53 relative of an f32 rounding boundary, so the double rounding is innocuous). Prints the mismatch count,
// the first mismatches and the hardware rcp's distribution (exact RN or not). Verification tool (tests/test_gpu_rcp.py).
// Build: ecdna-evo_amd/Makefile (bin/rcp_check; __graft_entry__.build() runs it)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "ssa_device.hpp"

__global__ void check(uint32_t e_lo, unsigned long long* bad, unsigned long long* rcp_not_rn, uint32_t* first) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // binade offset << 23 | mantissa
    const uint32_t u = ((e_lo + (uint32_t)(g >> 23)) << 23) | (uint32_t)(g & 0x7fffffu);
    const float b = __uint_as_float(u);
    const float r = __builtin_amdgcn_rcpf(b);
    const float y1 = ecdna::rcp_rn(b);
    const float yt = (float)(1.0 / (double)b);
    if (r != yt) atomicAdd(rcp_not_rn, 1ull);
    if (y1 != yt) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 8) {
            first[3 * k] = u;
            first[3 * k + 1] = __float_as_uint(r);
            first[3 * k + 2] = __float_as_uint(y1);
        }
    }
}

int main() {
    const uint32_t e_lo = 127 - 60, e_hi = 127 + 95;  // biased exponents [2^-60, 2^95)
    unsigned long long *bad, *nrn;
    uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&nrn, 8) != hipSuccess || hipMalloc(&first, 24 * 4) != hipSuccess ||
        hipMemset(bad, 0, 8) != hipSuccess || hipMemset(nrn, 0, 8) != hipSuccess || hipMemset(first, 0, 96) != hipSuccess)
        return 3;
    const uint64_t n = (uint64_t)(e_hi - e_lo) << 23;
    hipLaunchKernelGGL(check, dim3((unsigned)(n / 256)), dim3(256), 0, 0, e_lo, bad, nrn, first);
    unsigned long long hb = 0, hn = 0;
    uint32_t hf[24];
    if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&hn, nrn, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(hf, first, 96, hipMemcpyDeviceToHost) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return 3;
    printf("{\"values\": %llu, \"newton_not_rn\": %llu, \"rcp_not_rn\": %llu, \"first\": [", (unsigned long long)n, hb, hn);
    for (unsigned k = 0; k < (hb < 8 ? hb : 8); ++k)
        printf("%s[\"0x%08x\", \"0x%08x\", \"0x%08x\"]", k ? ", " : "", hf[3 * k], hf[3 * k + 1], hf[3 * k + 2]);
    printf("]}\n");
    return hb == 0 ? 0 : 1;
}
