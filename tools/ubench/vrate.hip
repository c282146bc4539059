// VALU issue cost per wave64 instruction on gfx950, by instruction class: each kernel runs ITER
// iterations of 8 independent chains of one instruction per lane (inline asm, so the compiler cannot
// fold them), enough waves to fill every SIMD; cycles per instruction per SIMD =
// time x clock x SIMDs / (waves x instructions). Run: hipcc --offload-arch=gfx950 -O2 vrate.hip && ./a.out
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int ITER = 4096;
#define CH8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

#define K32(name, ins)                                                                  \
    __global__ void name(uint32_t *out, uint32_t seed) {                                \
        uint32_t v0 = seed ^ threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7; \
        for (int i = 0; i < ITER; ++i) {                                                \
            asm volatile(ins " %0, %0, %0\n" ins " %1, %1, %1\n" ins " %2, %2, %2\n" ins " %3, %3, %3\n" \
                         ins " %4, %4, %4\n" ins " %5, %5, %5\n" ins " %6, %6, %6\n" ins " %7, %7, %7" \
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)); \
        }                                                                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7; \
    }
#define K32_3(name, ins)                                                                \
    __global__ void name(uint32_t *out, uint32_t seed) {                                \
        uint32_t v0 = seed ^ threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7; \
        for (int i = 0; i < ITER; ++i) {                                                \
            asm volatile(ins " %0, %0, %0, %0\n" ins " %1, %1, %1, %1\n" ins " %2, %2, %2, %2\n" ins " %3, %3, %3, %3\n" \
                         ins " %4, %4, %4, %4\n" ins " %5, %5, %5, %5\n" ins " %6, %6, %6, %6\n" ins " %7, %7, %7, %7" \
                         : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7)); \
        }                                                                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7; \
    }
#define K64(name, ins, args)                                                            \
    __global__ void name(uint32_t *out, uint32_t seed) {                                \
        uint64_t v0 = seed ^ threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7; \
        for (int i = 0; i < ITER; ++i) {                                                \
            asm volatile(ins " %0, " args "\n" ins " %1, " args "\n"                   \
                         : "+v"(v0), "+v"(v1)); asm volatile(ins " %0, " args "\n" ins " %1, " args "\n" : "+v"(v2), "+v"(v3)); \
            asm volatile(ins " %0, " args "\n" ins " %1, " args "\n" : "+v"(v4), "+v"(v5)); asm volatile(ins " %0, " args "\n" ins " %1, " args "\n" : "+v"(v6), "+v"(v7)); \
        }                                                                               \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7); \
    }

K32(k_add_u32, "v_add_u32")
K32(k_add_f32, "v_add_f32")
K32(k_mul_lo_u32, "v_mul_lo_u32")
K32(k_mul_u32_u24, "v_mul_u32_u24")
K32(k_mul_hi_u32_u24, "v_mul_hi_u32_u24")
K32_3(k_fma_f32, "v_fma_f32")
K32_3(k_bitop3, "v_xad_u32")
K64(k_add_f64, "v_add_f64", "%0, %0")
K64(k_mul_f64, "v_mul_f64", "%0, %0")
K64(k_fma_f64, "v_fma_f64", "%0, %0, %0")
K64(k_lshl_add_u64, "v_lshl_add_u64", "%0, 0, %0")
K64(k_rcp_f64, "v_rcp_f64", "%0")
K64(k_sqrt_f64, "v_sqrt_f64", "%0")

__global__ void k_mad_u64_u32(uint32_t *out, uint32_t seed) {
    uint64_t v0 = seed ^ threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6, v7 = v0 + 7;
    uint32_t a = seed + threadIdx.x;
    for (int i = 0; i < ITER; ++i) {
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %2, %0\nv_mad_u64_u32 %1, vcc, %2, %2, %1" : "+v"(v0), "+v"(v1) : "v"(a) : "vcc");
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %2, %0\nv_mad_u64_u32 %1, vcc, %2, %2, %1" : "+v"(v2), "+v"(v3) : "v"(a) : "vcc");
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %2, %0\nv_mad_u64_u32 %1, vcc, %2, %2, %1" : "+v"(v4), "+v"(v5) : "v"(a) : "vcc");
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %2, %0\nv_mad_u64_u32 %1, vcc, %2, %2, %1" : "+v"(v6), "+v"(v7) : "v"(a) : "vcc");
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7);
}

typedef void (*K)(uint32_t *, uint32_t);
int main() {
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    int clk_khz = 0;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8, threads = 256;  // 8 blocks x 4 waves per CU = 8 waves per SIMD
    uint32_t *out;
    (void)hipMalloc(&out, (size_t)blocks * threads * 4);
    struct { const char *n; K k; } ks[] = {
        {"v_add_u32", k_add_u32}, {"v_add_f32", k_add_f32}, {"v_fma_f32", k_fma_f32}, {"v_xad_u32", k_bitop3},
        {"v_mul_lo_u32", k_mul_lo_u32}, {"v_mul_u32_u24", k_mul_u32_u24}, {"v_mul_hi_u32_u24", k_mul_hi_u32_u24},
        {"v_mad_u64_u32", k_mad_u64_u32}, {"v_lshl_add_u64", k_lshl_add_u64}, {"v_add_f64", k_add_f64},
        {"v_rcp_f64", k_rcp_f64}, {"v_sqrt_f64", k_sqrt_f64}};
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    printf("CUs %d clock %d MHz\n", cus, clk_khz / 1000);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        (void)hipEventRecord(a);
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.k, dim3(blocks), dim3(threads), 0, 0, out, 1u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        const double waves = 3.0 * blocks * threads / 64.0;
        const double insts = waves * ITER * 8.0;
        const double cyc = ms * 1e-3 * clk_khz * 1e3 * cus * 4 / insts;
        printf("%-18s %8.3f ms  %.2f cycles per wave64 instruction per SIMD\n", k.n, ms / 3, cyc);
    }
    return 0;
}
