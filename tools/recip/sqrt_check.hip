// Exhaustive device check of a short square root against the correctly rounded one
// (-fhip-fp32-correctly-rounded-divide-sqrt): s = v_sqrt_f32(x), then the one-ulp neighbours chosen
// by the sign of the fma remainders (the compiler's own correction, without its small-input scaling
// and class fix-up). Mismatch counts by range of x.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float sqrt_short(float x) {
    float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    s = rm <= 0.0f ? sm : s;
    s = rp > 0.0f ? sp : s;
    return s;
}
__device__ __forceinline__ bool same(float a, float b) { return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b); }

__global__ void check(unsigned long long *bad, uint32_t *lo_bad, uint32_t *hi_bad) {
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < (1ull << 32); k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)k;
        const float x = __uint_as_float(u);
        if (!same(sqrt_short(x), __builtin_sqrtf(x))) {
            const int c = (u >> 31) ? 2 : ((u & 0x7fffffffu) < 0x0f800000u ? 0 : 1);  // x<0 | x<2^-96 | rest
            atomicAdd(&bad[c], 1ull);
            if (c == 1) { atomicMin(lo_bad, u); atomicMax(hi_bad, u); }
        }
    }
}

int main() {
    unsigned long long *bad;
    uint32_t *lo, *hi;
    if (hipMalloc(&bad, 24) != hipSuccess || hipMalloc(&lo, 4) != hipSuccess || hipMalloc(&hi, 4) != hipSuccess) return 2;
    hipMemset(bad, 0, 24);
    hipMemset(lo, 0xff, 4);
    hipMemset(hi, 0, 4);
    hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, bad, lo, hi);
    unsigned long long hb[3];
    uint32_t hl, hh;
    if (hipMemcpy(hb, bad, 24, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    hipMemcpy(&hl, lo, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&hh, hi, 4, hipMemcpyDeviceToHost);
    printf("x < 2^-96 (non-negative): %llu mismatches\nx >= 2^-96: %llu mismatches (bits 0x%08x..0x%08x)\nx < 0: %llu mismatches\n", hb[0], hb[1], hl, hh, hb[2]);
    return 0;
}
