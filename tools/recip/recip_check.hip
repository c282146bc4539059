// Exhaustive device check of rrt_kernel.hip's recip_rn against the IEEE quotient 1.0f / s
// (-fhip-fp32-correctly-rounded-divide-sqrt) over all 2^32 f32 bit patterns:
//   recip_rn(s): r = v_rcp_f32(s); e = fma(-s, r, 1); e == e ? fma(e, r, r) : r
// Counts mismatches (NaN results compare as equal) by class: normal |s| in [2^-126, 2^126), other
// finite (subnormal or |s| >= 2^126), and the clamped ray-constant form clamp(recip, +-2^64).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float recip_rn(float s) {
    const float r = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r, 1.0f);
    return e == e ? __builtin_fmaf(e, r, r) : r;
}
__device__ __forceinline__ float clamp_inv(float v) { return __builtin_fmaxf(__builtin_fminf(v, 0x1.0p64f), -0x1.0p64f); }
__device__ __forceinline__ bool same(float a, float b) { return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b); }

__global__ void check(unsigned long long *bad, uint32_t *first) {
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < (1ull << 32); k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)k;
        const float s = __uint_as_float(u);
        const float ref = 1.0f / s, got = recip_rn(s);
        const uint32_t a = u & 0x7fffffffu;
        const int cls = (a >= 0x00800000u && a < 0x7e800000u) ? 0 : 1;
        if (!same(got, ref)) { atomicAdd(&bad[cls], 1ull); atomicMin(&first[cls], u); }
        if (!same(clamp_inv(got), clamp_inv(ref))) { atomicAdd(&bad[2], 1ull); atomicMin(&first[2], u); }
    }
}

int main() {
    unsigned long long *bad;
    uint32_t *first;
    if (hipMalloc(&bad, 24) != hipSuccess || hipMalloc(&first, 12) != hipSuccess) return 2;
    if (hipMemset(bad, 0, 24) != hipSuccess || hipMemset(first, 0xff, 12) != hipSuccess) return 2;
    hipLaunchKernelGGL(check, dim3(16384), dim3(256), 0, 0, bad, first);
    unsigned long long hb[3];
    uint32_t hf[3];
    if (hipMemcpy(hb, bad, 24, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    if (hipMemcpy(hf, first, 12, hipMemcpyDeviceToHost) != hipSuccess) return 3;
    const char *names[3] = {"normal", "other", "clamped"};
    for (int c = 0; c < 3; ++c) printf("%s mismatches %llu first 0x%08x\n", names[c], hb[c], hb[c] ? hf[c] : 0u);
    return 0;
}
