// rrt_device.h — device helpers shared by the f32 megakernel (rrt_kernel.hip) and the f64
// books-arithmetic kernel (rrt_books64.hip): the per-path RNG stream (both kernels draw the same
// numbers for the same (seed, pixel, sample)), the kernarg-segment parameter view, the LDS
// traversal stack, the postponed-leaf record, the accumulation chunk schedule and wave reductions.
// Included inside namespace rrt { namespace { ... } } by each kernel file.
#pragma once

// 64 if the calling lane is the wave's first active lane, else 0 (wave-level event count).
__device__ __forceinline__ uint32_t wave_slot() {
    return (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x ? 64u : 0u;
}

// ---- RNG: xoshiro128+ per path, keyed by (seed, pixel, sample) ------------------------------
// Counter-based in effect: the i-th draw of a path is a pure function of
// (seed, global pixel index, sample index, i); nothing depends on lane or launch shape.
// xoshiro128+ (Blackman & Vigna) is all full-rate 32-bit VALU (add, shift, xor, alignbit):
// 8 instructions per draw against ~17 with three quarter-rate multiplies for the 64-bit LCG
// of a PCG32 (+4.3 % on C2, same-box A/B). Only the top 24 bits of each output are used
// (random_double), the bits the authors recommend for floating-point generation.
// f16 planes of a GNodeH (exact conversions; in an FMA operand they become v_fma_mix_f32)
__device__ __forceinline__ float lo16(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu)); }
__device__ __forceinline__ float hi16(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16)); }

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
struct RngState {
    uint32_t a, b, c, d;
};
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
// x ^ y ^ z in one gfx950 V_BITOP3_B32 (truth table 0x96)
// (gfx950 only: on another --offload-arch the same value by two xors)
__device__ __forceinline__ uint32_t xor3_32(uint32_t x, uint32_t y, uint32_t z) {
#if defined(__gfx950__)
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
#else
    return x ^ y ^ z;
#endif
}
// xoshiro128+ (c ^= a; d ^= b; b ^= c; a ^= d; c ^= b << 9; d = rotl(d, 11); result a + d before
// the step), its two chained xors per word folded into three-input xors: 7 VALU instructions per
// draw instead of 8, the same state sequence (tests/test_rng_bitop3.py checks the algebra).
// RRT_RNG_BITOP3=0: the two-input form.
#ifndef RRT_RNG_BITOP3
#define RRT_RNG_BITOP3 1
#endif
__device__ __forceinline__ uint32_t rng_next(RngState &s) {
    const uint32_t r = s.a + s.d;
    const uint32_t t = s.b << 9;
    if (RRT_RNG_BITOP3) {
        const uint32_t db = s.d ^ s.b;
        const uint32_t b = xor3_32(s.b, s.c, s.a);
        const uint32_t c = xor3_32(s.c, s.a, t);
        s.a ^= db;
        s.b = b;
        s.c = c;
        s.d = rotl32(db, 11);
        return r;
    }
    s.c ^= s.a;
    s.d ^= s.b;
    s.b ^= s.c;
    s.a ^= s.d;
    s.c ^= t;
    s.d = rotl32(s.d, 11);
    return r;
}
// state = (z, pixel key); the low bit of the last word is forced so the state is never zero
__device__ __forceinline__ RngState rng_seed(uint64_t z, uint64_t key) {
    return RngState{(uint32_t)z, (uint32_t)(z >> 32), (uint32_t)key, (uint32_t)(key >> 32) | 1u};
}
// 64 bits of the state (the media draws' key at a segment start)
__device__ __forceinline__ uint64_t rng_key(const RngState &s) { return (uint64_t)s.a | ((uint64_t)s.b << 32); }
// random_double(): 24-bit uniform in [0,1) (exact in f32 and f64).
__device__ __forceinline__ float rnd(RngState &s) { return (float)(rng_next(s) >> 8) * 0x1.0p-24f; }
// random_double_range(lo,hi) = u*(hi-lo) + lo  (rand 0.8 UniformFloat::sample_single order)
__device__ __forceinline__ float rnd_range(RngState &s, float lo, float hi) { return rnd(s) * (hi - lo) + lo; }
// rnd_range(s, -1, 1) in one rounding less work: u * 2^-24 * 2 is exact (power-of-two scalings
// of a 24-bit integer), so u * 2^-23 - 1 rounds once, at the add — and fma(u, 2^-23, -1) rounds
// the same exact product once: identical bits in one instruction.
__device__ __forceinline__ float rnd_pm1(RngState &s) {
    return __builtin_fmaf((float)(rng_next(s) >> 8), 0x1.0p-23f, -1.0f);
}

// Per-lane work counts of the instrumented (counting) kernel variant (+ debug statistics).
struct Counters {
    uint32_t nodes, boxes, spheres;
    uint32_t d0, d1, d2;
};

// Traversal stack in LDS. 16-bit entries: the dword at (depth, wave, k) holds lanes k and
// k+32, which the LDS serves in different cycles (2 x 32-lane groups), so no bank conflicts.
template <typename StackT, int kBlk>
struct LdsStack {
    StackT *base;
    __device__ __forceinline__ void init(StackT *lds, uint32_t tid) {
        if constexpr (sizeof(StackT) == 2) {
            const uint32_t lane = tid & 63u;
            base = lds + (tid & ~63u) + ((lane & 31u) << 1) + (lane >> 5);
        } else {
            base = lds + tid;
        }
    }
    __device__ __forceinline__ void store(int sp, int v) { base[sp * kBlk] = (StackT)v; }
    __device__ __forceinline__ int load(int sp) const { return (int)base[sp * kBlk]; }
};

// A lane's postponed leaf tests: primitives [first, first + count), packed first | count << 28
// like a GNode leaf link (count <= 2 x kMaxLeafPrims = 14, primitive indices < 2^28).
using Leaves = uint32_t;

// The camera block re-read from the kernarg segment at each use (scalar loads through the scalar
// cache) rather than 19 values the compiler would hold in SGPRs across the whole work loop: the
// asm makes the pointer opaque, so the loads cannot be hoisted out of the loop.
__device__ __forceinline__ const __attribute__((address_space(4))) KParams *kernarg_params() {
    auto q = (const __attribute__((address_space(4))) KParams *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(q));
    return q;
}
// a FastDiv member read through either view of the parameters
template <class FD>
__device__ __forceinline__ FastDiv fdiv(const FD &f) { return FastDiv{f.m, f.s}; }

// The path's RNG stream for sample s of global pixel (x, y): xoshiro128+ state
// (z, key | 1 << 32) with key = splitmix64((seed << 32) ^ pixel) and z = splitmix64(key + s).
// The key is computed once per work unit (pixel, sample chunk) and held (+0.6 % on C2).
template <class KP>
__device__ __forceinline__ uint64_t pixel_key(const KP &P, uint32_t x, uint32_t y) {
    return splitmix64(((uint64_t)P.seed << 32) ^ (uint64_t)(y * P.width + x));
}
__device__ __forceinline__ RngState path_rng_k(uint64_t key, uint32_t s) { return rng_seed(splitmix64(key + s), key); }

// First sample (relative to sample_begin) of chunk c of a pixel (rrt_accum_chunk's schedule).
template <class KP>
__host__ __device__ __forceinline__ uint32_t chunk_first(const KP &P, uint32_t c) {
    return c < P.n_big ? c * P.chunk : P.n_big * P.chunk + (c - P.n_big) * P.chunk_small;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
