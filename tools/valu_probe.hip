// Throughput of the instruction classes the SSA stepper is made of, on this chip: each kernel runs
// 8 independent dependency chains per lane of one instruction (inline asm, so the compiler cannot
// fold them) at full occupancy; reported as wave-instructions per cycle per SIMD (clock from
// hipDeviceProp), i.e. 0.5 = one wave64 instruction every 2 cycles.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 16384;

#define CHAINS8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ void __launch_bounds__(256) k_add_u32(uint32_t* out, uint32_t s) {
    uint32_t v[8];
#define I(j) v[j] = threadIdx.x + j;
    CHAINS8(I)
#undef I
    for (int i = 0; i < ITERS; ++i) {
#define I(j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[j]) : "s"(s));
        CHAINS8(I)
#undef I
    }
    uint32_t r = 0;
#define I(j) r ^= v[j];
    CHAINS8(I)
#undef I
    if (r == 0x12345) out[0] = r;
}

__global__ void __launch_bounds__(256) k_mad_u64(uint32_t* out, uint32_t s) {
    uint64_t v[8];
#define I(j) v[j] = threadIdx.x + j;
    CHAINS8(I)
#undef I
    for (int i = 0; i < ITERS; ++i) {
#define I(j) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(v[j]) : "v"((uint32_t)v[j]), "s"(s) : "vcc");
        CHAINS8(I)
#undef I
    }
    uint64_t r = 0;
#define I(j) r ^= v[j];
    CHAINS8(I)
#undef I
    if (r == 0x12345) out[0] = (uint32_t)r;
}

__global__ void __launch_bounds__(256) k_fma_f64(uint32_t* out, double s) {
    double v[8];
#define I(j) v[j] = threadIdx.x + j;
    CHAINS8(I)
#undef I
    for (int i = 0; i < ITERS; ++i) {
#define I(j) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v[j]) : "v"(s));
        CHAINS8(I)
#undef I
    }
    double r = 0;
#define I(j) r += v[j];
    CHAINS8(I)
#undef I
    if (r == 1.2345) out[0] = 1;
}

__global__ void __launch_bounds__(256) k_add_f64(uint32_t* out, double s) {
    double v[8];
#define I(j) v[j] = threadIdx.x + j;
    CHAINS8(I)
#undef I
    for (int i = 0; i < ITERS; ++i) {
#define I(j) asm volatile("v_add_f64 %0, %0, %1" : "+v"(v[j]) : "v"(s));
        CHAINS8(I)
#undef I
    }
    double r = 0;
#define I(j) r += v[j];
    CHAINS8(I)
#undef I
    if (r == 1.2345) out[0] = 1;
}

__global__ void __launch_bounds__(256) k_cndmask(uint32_t* out, uint32_t s) {
    uint32_t v[8];
#define I(j) v[j] = threadIdx.x + j;
    CHAINS8(I)
#undef I
    for (int i = 0; i < ITERS; ++i) {
#define I(j) asm volatile("v_cmp_gt_u32 vcc, %0, %1\n s_nop 1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[j]) : "v"(s) : "vcc");
        CHAINS8(I)
#undef I
    }
    uint32_t r = 0;
#define I(j) r ^= v[j];
    CHAINS8(I)
#undef I
    if (r == 0x12345) out[0] = r;
}

__global__ void __launch_bounds__(256) k_ds_add(uint32_t* out, uint32_t s) {
    __shared__ uint32_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = 0;
    __syncthreads();
    const uint32_t base = threadIdx.x * 4;
    for (int i = 0; i < ITERS; ++i) {
#define I(j) atomicAdd(&lds[(base + j * 1024 + i) & 4095], s);
        CHAINS8(I)
#undef I
    }
    __syncthreads();
    if (lds[threadIdx.x] == 0x12345) out[0] = 1;
}


#define OPKERNEL(NAME, T, INIT, ASM, CONSTR, ARG)                                                     \
    __global__ void __launch_bounds__(256) NAME(uint32_t* out, ARG s) {                               \
        T v[8];                                                                                       \
        for (int j = 0; j < 8; ++j) v[j] = (T)(threadIdx.x + j + INIT);                               \
        for (int i = 0; i < ITERS; ++i) {                                                             \
            _Pragma("unroll") for (int j = 0; j < 8; ++j) asm volatile(ASM : "+v"(v[j]) : CONSTR(s)); \
        }                                                                                             \
        T r = 0;                                                                                      \
        for (int j = 0; j < 8; ++j) r += v[j];                                                        \
        if (r == (T)12345) out[0] = 1;                                                                \
    }
OPKERNEL(k_fma_f32, float, 0.5f, "v_fma_f32 %0, %0, %1, %1", "v", float)
OPKERNEL(k_add_f32, float, 0.5f, "v_add_f32 %0, %0, %1", "v", float)
OPKERNEL(k_pk_fma_f32, double, 0.5, "v_pk_fma_f32 %0, %0, %1, %1", "v", double)
OPKERNEL(k_and_b32, uint32_t, 1, "v_and_b32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_lshl_add, uint32_t, 1, "v_lshl_add_u32 %0, %0, 1, %1", "v", uint32_t)
OPKERNEL(k_bcnt, uint32_t, 1, "v_bcnt_u32_b32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_mul_u24, uint32_t, 1, "v_mul_u32_u24 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_mul_lo_u32, uint32_t, 1, "v_mul_lo_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_pk_add_u16, uint32_t, 1, "v_pk_add_u16 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_cvt_f64_u32, double, 1, "v_cvt_f64_u32 %0, %1", "v", uint32_t)
OPKERNEL(k_mov_b32, uint32_t, 1, "v_mov_b32 %0, %1", "v", uint32_t)

OPKERNEL(k_add_u32_v, uint32_t, 1, "v_add_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_sub_u32_v, uint32_t, 1, "v_sub_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_xor_v, uint32_t, 1, "v_xor_b32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_xor_s, uint32_t, 1, "v_xor_b32 %0, %1, %0", "s", uint32_t)
OPKERNEL(k_or_v, uint32_t, 1, "v_or_b32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_lshl_v, uint32_t, 1, "v_lshlrev_b32 %0, %1, %0", "v", uint32_t)
OPKERNEL(k_lshr_v, uint32_t, 1, "v_lshrrev_b32 %0, %1, %0", "v", uint32_t)
OPKERNEL(k_max_u32, uint32_t, 1, "v_max_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_min_u32, uint32_t, 1, "v_min_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_mul_f32, float, 0.5f, "v_mul_f32 %0, %0, %1", "v", float)
OPKERNEL(k_bfe, uint32_t, 1, "v_bfe_u32 %0, %0, 3, 7", "v", uint32_t)
OPKERNEL(k_cndmask_vcc, uint32_t, 1, "v_cndmask_b32 %0, %0, %1, vcc", "v", uint32_t)
OPKERNEL(k_add3, uint32_t, 1, "v_add3_u32 %0, %0, %1, %1", "v", uint32_t)
OPKERNEL(k_and_or, uint32_t, 1, "v_and_or_b32 %0, %0, %1, %1", "v", uint32_t)
OPKERNEL(k_mad_u24, uint32_t, 1, "v_mad_u32_u24 %0, %0, %1, %1", "v", uint32_t)
OPKERNEL(k_mul_hi_u32, uint32_t, 1, "v_mul_hi_u32 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_lshl_add_u64, uint64_t, 1, "v_lshl_add_u64 %0, %0, 1, %1", "v", uint64_t)
OPKERNEL(k_mul_f64, double, 0.5, "v_mul_f64 %0, %0, %1", "v", double)
OPKERNEL(k_cvt_f32_u32, float, 1, "v_cvt_f32_u32 %0, %1", "v", uint32_t)
OPKERNEL(k_rcp_f64, double, 1, "v_rcp_f64 %0, %1", "v", double)
// round 2: encodings and operand kinds of the stepper's instruction mix
OPKERNEL(k_ashr_v, uint32_t, 1, "v_ashrrev_i32 %0, %1, %0", "v", uint32_t)
OPKERNEL(k_bitop3, uint32_t, 1, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96", "v", uint32_t)
OPKERNEL(k_lshl_or, uint32_t, 1, "v_lshl_or_b32 %0, %0, 3, %1", "v", uint32_t)
OPKERNEL(k_perm, uint32_t, 1, "v_perm_b32 %0, %0, %1, %1", "v", uint32_t)
OPKERNEL(k_add_e64, uint32_t, 1, "v_add_u32_e64 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_xor_e64, uint32_t, 1, "v_xor_b32_e64 %0, %0, %1", "v", uint32_t)
OPKERNEL(k_lshr_e64, uint32_t, 1, "v_lshrrev_b32_e64 %0, %1, %0", "v", uint32_t)
OPKERNEL(k_lshl_imm, uint32_t, 1, "v_lshlrev_b32 %0, 3, %0", "v", uint32_t)
OPKERNEL(k_mul_f64_s, double, 0.5, "v_mul_f64 %0, %0, %1", "s", double)
OPKERNEL(k_add_f64_v, double, 0.5, "v_add_f64 %0, %0, %1", "v", double)
OPKERNEL(k_cvt_f64_i32, double, 1, "v_cvt_f64_i32 %0, %1", "v", uint32_t)
OPKERNEL(k_min3, uint32_t, 1, "v_min3_u32 %0, %0, %1, %1", "v", uint32_t)
OPKERNEL(k_sub_co, uint32_t, 1, "v_sub_co_u32 %0, vcc, %0, %1", "v", uint32_t)
OPKERNEL(k_add_lit, uint32_t, 1, "v_add_u32 %0, 0x12345, %0", "v", uint32_t)

__global__ void __launch_bounds__(256) k_mad_u64_v(uint32_t* out, uint32_t s) {
    uint64_t v[8];
    const uint32_t c = s + threadIdx.x * 0u;  // the constant in a VGPR
    uint32_t cv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(cv) : "s"(c));
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j)
            asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(v[j]) : "v"((uint32_t)v[j]), "v"(cv) : "vcc");
    }
    uint64_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= v[j];
    if (r == 0x12345) out[0] = (uint32_t)r;
}

// v_cndmask_b32_e64 with an SGPR-pair condition (the compiler's usual select form)
__global__ void __launch_bounds__(256) k_cndmask_s(uint32_t* out, uint32_t s) {
    uint32_t v[8];
    uint64_t m = (s & 1u) ? 0x5555aaaa5555ull : 0x5555ull;
    asm volatile("" : "+s"(m));
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j)
            asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(v[j]) : "v"(s), "s"(m));
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= v[j];
    if (r == 0x12345) out[0] = r;
}

// v_cmp_gt_u32_e64 into an SGPR pair (8 independent compares per lane per iteration)
__global__ void __launch_bounds__(256) k_cmp_s(uint32_t* out, uint32_t s) {
    uint32_t v[8];
    uint64_t m[8];
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        _Pragma("unroll") for (int j = 0; j < 8; ++j)
            asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m[j]) : "v"(v[j]), "v"(s));
    }
    uint64_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= m[j];
    if (r == 0x12345) out[0] = 1;
}


// v_cndmask_b32_e32 reading VCC (set once per 8), and v_cmp_*_e32 writing VCC
__global__ void __launch_bounds__(256) k_cndmask_e32(uint32_t* out, uint32_t s) {
    uint32_t v[8];
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_gt_u32_e32 vcc, %0, %8\n"
            "v_cndmask_b32_e32 %0, %0, %8, vcc\n v_cndmask_b32_e32 %1, %1, %8, vcc\n"
            "v_cndmask_b32_e32 %2, %2, %8, vcc\n v_cndmask_b32_e32 %3, %3, %8, vcc\n"
            "v_cndmask_b32_e32 %4, %4, %8, vcc\n v_cndmask_b32_e32 %5, %5, %8, vcc\n"
            "v_cndmask_b32_e32 %6, %6, %8, vcc\n v_cndmask_b32_e32 %7, %7, %8, vcc"
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
            : "v"(s) : "vcc");
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= v[j];
    if (r == 0x12345) out[0] = r;
}

__global__ void __launch_bounds__(256) k_cmp_e32(uint32_t* out, uint32_t s) {
    uint32_t v[8];
    uint64_t acc = 0;
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        uint64_t m;
        asm volatile(
            "v_cmp_gt_u32_e32 vcc, %1, %9\n v_cmp_gt_u32_e32 vcc, %2, %9\n"
            "v_cmp_gt_u32_e32 vcc, %3, %9\n v_cmp_gt_u32_e32 vcc, %4, %9\n"
            "v_cmp_gt_u32_e32 vcc, %5, %9\n v_cmp_gt_u32_e32 vcc, %6, %9\n"
            "v_cmp_gt_u32_e32 vcc, %7, %9\n v_cmp_gt_u32_e32 vcc, %8, %9\n s_mov_b64 %0, vcc"
            : "=s"(m) : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(s)
            : "vcc");
        acc ^= m;
    }
    if (acc == 0x12345) out[0] = 1;
}

// v_addc_co_u32_e32: add with the carry in and out through VCC (the borrow/carry counting idiom)
__global__ void __launch_bounds__(256) k_addc_e32(uint32_t* out, uint32_t s) {
    uint32_t v[8];
    for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j;
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_addc_co_u32_e32 %0, vcc, %0, %8, vcc\n v_addc_co_u32_e32 %1, vcc, %1, %8, vcc\n"
            "v_addc_co_u32_e32 %2, vcc, %2, %8, vcc\n v_addc_co_u32_e32 %3, vcc, %3, %8, vcc\n"
            "v_addc_co_u32_e32 %4, vcc, %4, %8, vcc\n v_addc_co_u32_e32 %5, vcc, %5, %8, vcc\n"
            "v_addc_co_u32_e32 %6, vcc, %6, %8, vcc\n v_addc_co_u32_e32 %7, vcc, %7, %8, vcc"
            : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7])
            : "v"(s) : "vcc");
    }
    uint32_t r = 0;
    for (int j = 0; j < 8; ++j) r ^= v[j];
    if (r == 0x12345) out[0] = r;
}

template <typename F>
void time_it(const char* name, F launch, double insts_per_lane_iter, int cus, double clk_hz) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double blocks = cus * 8.0, waves = blocks * 4.0;
    const double wave_insts = waves * ITERS * insts_per_lane_iter;
    const double per_simd_cycle = wave_insts / (cus * 4.0) / (ms * 1e-3 * clk_hz);
    printf("%-12s %8.3f ms  %.3f wave-instr / cycle / SIMD (at %.0f MHz) = %.3e wave-instr/s chip\n", name, ms,
           per_simd_cycle, clk_hz / 1e6, wave_insts / (ms * 1e-3));
}

// round 2 (r02e): what makes the VOP2 select slow — the encoding, the VCC read, or the VALU write of VCC
#define SEL8(fmt)                                                                                        \
    asm volatile(fmt(0) fmt(1) fmt(2) fmt(3) fmt(4) fmt(5) fmt(6) fmt(7)                                \
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),     \
                   "+v"(v[7])                                                                           \
                 : "v"(s), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), \
                   "v"(x[7])                                                                            \
                 : "vcc")
#define E64_VCC(j) "v_cndmask_b32_e64 %" #j ", %" #j ", %8, vcc\n"
#define E32_VCC(j) "v_cndmask_b32_e32 %" #j ", %" #j ", %8, vcc\n"
#define E32_MIX(j) "v_cndmask_b32_e32 %" #j ", %" #j ", %8, vcc\n v_xor_b32 %" #j ", %" #j ", %8\n"
#define XOR_ONLY(j) "v_xor_b32 %" #j ", %" #j ", %8\n v_xor_b32 %" #j ", %" #j ", %8\n"
#define SELKERNEL(name, FMT, SETVCC)                                                                     \
    __global__ void __launch_bounds__(256) name(uint32_t* out, uint32_t s) {                             \
        uint32_t v[8], x[8];                                                                             \
        for (int j = 0; j < 8; ++j) v[j] = threadIdx.x + j, x[j] = threadIdx.x * 3u + j;                \
        asm volatile(SETVCC ::: "vcc");                                                                  \
        for (int i = 0; i < ITERS; ++i) SEL8(FMT);                                                       \
        uint32_t r = 0;                                                                                  \
        for (int j = 0; j < 8; ++j) r ^= v[j];                                                           \
        if (r == 0x12345) out[0] = r;                                                                    \
    }
SELKERNEL(k_sel_e64_vcc, E64_VCC, "s_mov_b64 vcc, 0x5555aaaa")
SELKERNEL(k_sel_e32_svcc, E32_VCC, "s_mov_b64 vcc, 0x5555aaaa")
SELKERNEL(k_sel_e32_mix, E32_MIX, "s_mov_b64 vcc, 0x5555aaaa")
SELKERNEL(k_sel_xor_only, XOR_ONLY, "s_mov_b64 vcc, 0x5555aaaa")

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const double clk = p.clockRate * 1e3;
    uint32_t* d;
    hipMalloc(&d, 64);
    dim3 g(cus * 8), blk(256);
    time_it("add_u32", [&] { hipLaunchKernelGGL(k_add_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mad_u64_u32", [&] { hipLaunchKernelGGL(k_mad_u64, g, blk, 0, 0, d, 0xD2511F53u); }, 8, cus, clk);
    time_it("fma_f64", [&] { hipLaunchKernelGGL(k_fma_f64, g, blk, 0, 0, d, 0.999); }, 8, cus, clk);
    time_it("add_f64", [&] { hipLaunchKernelGGL(k_add_f64, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("cmp+cndmask", [&] { hipLaunchKernelGGL(k_cndmask, g, blk, 0, 0, d, 7u); }, 16, cus, clk);
    time_it("fma_f32", [&] { hipLaunchKernelGGL(k_fma_f32, g, blk, 0, 0, d, 0.999f); }, 8, cus, clk);
    time_it("add_f32", [&] { hipLaunchKernelGGL(k_add_f32, g, blk, 0, 0, d, 0.5f); }, 8, cus, clk);
    time_it("pk_fma_f32", [&] { hipLaunchKernelGGL(k_pk_fma_f32, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("and_b32", [&] { hipLaunchKernelGGL(k_and_b32, g, blk, 0, 0, d, 0xffffu); }, 8, cus, clk);
    time_it("lshl_add_u32", [&] { hipLaunchKernelGGL(k_lshl_add, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("bcnt_u32", [&] { hipLaunchKernelGGL(k_bcnt, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mul_u32_u24", [&] { hipLaunchKernelGGL(k_mul_u24, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mul_lo_u32", [&] { hipLaunchKernelGGL(k_mul_lo_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("pk_add_u16", [&] { hipLaunchKernelGGL(k_pk_add_u16, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("cvt_f64_u32", [&] { hipLaunchKernelGGL(k_cvt_f64_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mov_b32", [&] { hipLaunchKernelGGL(k_mov_b32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("add_u32_v", [&] { hipLaunchKernelGGL(k_add_u32_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("sub_u32_v", [&] { hipLaunchKernelGGL(k_sub_u32_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("xor_v", [&] { hipLaunchKernelGGL(k_xor_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("xor_s", [&] { hipLaunchKernelGGL(k_xor_s, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("or_v", [&] { hipLaunchKernelGGL(k_or_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshlrev_v", [&] { hipLaunchKernelGGL(k_lshl_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshrrev_v", [&] { hipLaunchKernelGGL(k_lshr_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("max_u32", [&] { hipLaunchKernelGGL(k_max_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("min_u32", [&] { hipLaunchKernelGGL(k_min_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mul_f32", [&] { hipLaunchKernelGGL(k_mul_f32, g, blk, 0, 0, d, 0.5f); }, 8, cus, clk);
    time_it("bfe_u32", [&] { hipLaunchKernelGGL(k_bfe, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("cndmask_vcc", [&] { hipLaunchKernelGGL(k_cndmask_vcc, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("add3_u32", [&] { hipLaunchKernelGGL(k_add3, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("and_or_b32", [&] { hipLaunchKernelGGL(k_and_or, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mad_u32_u24", [&] { hipLaunchKernelGGL(k_mad_u24, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mul_hi_u32", [&] { hipLaunchKernelGGL(k_mul_hi_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshl_add_u64", [&] { hipLaunchKernelGGL(k_lshl_add_u64, g, blk, 0, 0, d, (uint64_t)3); }, 8, cus, clk);
    time_it("mul_f64", [&] { hipLaunchKernelGGL(k_mul_f64, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("cvt_f32_u32", [&] { hipLaunchKernelGGL(k_cvt_f32_u32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("rcp_f64", [&] { hipLaunchKernelGGL(k_rcp_f64, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("ds_add_u32", [&] { hipLaunchKernelGGL(k_ds_add, g, blk, 0, 0, d, 1u); }, 8, cus, clk);
    time_it("ashrrev_v", [&] { hipLaunchKernelGGL(k_ashr_v, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("bitop3_v", [&] { hipLaunchKernelGGL(k_bitop3, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshl_or_v", [&] { hipLaunchKernelGGL(k_lshl_or, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("perm_v", [&] { hipLaunchKernelGGL(k_perm, g, blk, 0, 0, d, 0x05040100u); }, 8, cus, clk);
    time_it("add_u32_e64_v", [&] { hipLaunchKernelGGL(k_add_e64, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("xor_e64_v", [&] { hipLaunchKernelGGL(k_xor_e64, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshrrev_e64_v", [&] { hipLaunchKernelGGL(k_lshr_e64, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("lshlrev_imm", [&] { hipLaunchKernelGGL(k_lshl_imm, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mul_f64_s", [&] { hipLaunchKernelGGL(k_mul_f64_s, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("add_f64_v", [&] { hipLaunchKernelGGL(k_add_f64_v, g, blk, 0, 0, d, 0.5); }, 8, cus, clk);
    time_it("cvt_f64_i32", [&] { hipLaunchKernelGGL(k_cvt_f64_i32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("min3_u32", [&] { hipLaunchKernelGGL(k_min3, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("sub_co_vcc", [&] { hipLaunchKernelGGL(k_sub_co, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("add_lit", [&] { hipLaunchKernelGGL(k_add_lit, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("mad_u64_v", [&] { hipLaunchKernelGGL(k_mad_u64_v, g, blk, 0, 0, d, 0xD2511F53u); }, 8, cus, clk);
    time_it("cndmask_e64_s", [&] { hipLaunchKernelGGL(k_cndmask_s, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("cmp_e64_s", [&] { hipLaunchKernelGGL(k_cmp_s, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("cndmask_e32_vcc", [&] { hipLaunchKernelGGL(k_cndmask_e32, g, blk, 0, 0, d, 3u); }, 9, cus, clk);
    time_it("cmp_e32_vcc", [&] { hipLaunchKernelGGL(k_cmp_e32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("sel_e64_vcc", [&] { hipLaunchKernelGGL(k_sel_e64_vcc, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("sel_e32_svcc", [&] { hipLaunchKernelGGL(k_sel_e32_svcc, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    time_it("sel_e32_mix", [&] { hipLaunchKernelGGL(k_sel_e32_mix, g, blk, 0, 0, d, 3u); }, 16, cus, clk);
    time_it("sel_xor_only", [&] { hipLaunchKernelGGL(k_sel_xor_only, g, blk, 0, 0, d, 3u); }, 16, cus, clk);
    time_it("addc_e32_vcc", [&] { hipLaunchKernelGGL(k_addc_e32, g, blk, 0, 0, d, 3u); }, 8, cus, clk);
    return 0;
}
