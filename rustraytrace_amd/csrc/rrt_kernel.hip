// rrt_kernel.hip — gfx950 (CDNA4) path-tracing megakernel.
//
// One lane owns one pixel and runs that pixel's samples [sample_begin, sample_end) in
// order, regenerating a new camera ray in place whenever a path ends (path
// regeneration), so no lane idles while others finish long paths and the per-pixel sum
// is accumulated in fixed sample order (deterministic, no float atomics).
// Each 64-lane wave covers one 8x8 pixel tile (coherent camera rays); a 256-thread block
// holds 4 tiles. BVH2 traversal is iterative, nearest-child-first, with the node stack in
// LDS laid out [depth][lane] (conflict-free: consecutive lanes hit consecutive banks).
//
// Semantics follow the reference's CPU "books" path (NOT src/cuda, Appendix A of SURVEY):
//   camera ray       in_one_weekend/camera.rs:152-180  (+ time draw the_next_week/camera.rs:160)
//   closest hit      camera.rs:187 over (0.001, +inf), sphere.rs:24-51 open interval
//   Aabb slab test   aabb.rs:52-85
//   scatter          material.rs:28-40 / 53-64 / 83-102, vec3.rs:181-189, 201-210
//   Russian roulette camera.rs:189-200 (this bounce's attenuation, clamp [.05,.95])
//   sky / background camera.rs:206-208 / the_next_week/camera.rs:179-181
//   emission, texture the_next_week/material.rs:41-53,131-135, texture.rs:89-109, sphere.rs:46-52
// in f32 with every operation in the reference's order (built with -ffp-contract=off and
// correctly rounded f32 div/sqrt; the only fused multiply-adds are explicit: dot products and
// sums of squares, the sphere discriminant h*h - a*c, Ray::at of the hit point, the slab test)
// so the CPU oracle (oracle/) can reproduce each sample bit for bit. Throughput is carried front-to-back
// (T <- T*att[*1/p]); the reference multiplies back-to-front through its recursion —
// equal in exact arithmetic (documented in DESIGN.md).
#include "rrt_internal.h"

#include <algorithm>
#include <type_traits>

namespace rrt {
namespace {

// Debug builds only (-DRRT_PHASE_TIMING=1..9, never the shipped library): per-wave phase
// statistics written into counter slots 2..4 by the non-counting kernel.
//   1: s_memtime cycles spent in refill+ray start / traversal loop / shading
//   2: traversal wave-iterations x 64 / sum of tracing lanes per iteration / outer iterations
//   3: leaf-loop wave-iterations x 64 / active lanes per leaf iteration / lanes taking the root branch
//   4: shade entries x 64 / shading lanes / rejection-loop wave-iterations x 64
//   5: dielectric-branch wave entries x 64 / dielectric lanes / metal-branch wave entries x 64
//   6: metal lanes / miss (sky) wave entries x 64 / miss lanes
//   7: camera-ray wave entries x 64 (after a path ends) / their lanes / disk-loop wave-iterations x 64
//   8: node-step wave-iterations x 64 / those whose stepping lanes all visit one node x 64 / their lanes
//   9: noise-texture wave entries x 64 / noise lanes / shade entries x 64
#ifndef RRT_PHASE_TIMING
#define RRT_PHASE_TIMING 0
#endif
// Debug builds only: random_unit_vector takes its first candidate (wrong images; prices the
// rejection loop's wave-iterations in an A/B)
#ifndef RRT_DEBUG_NOREJECT
#define RRT_DEBUG_NOREJECT 0
#endif
#ifndef RRT_DEBUG_EXTRA_NODE_LOAD
#define RRT_DEBUG_EXTRA_NODE_LOAD 0
#endif
// Wave issue priority per loop phase (s_setprio levels 0-3; see the work loop's head).
#ifndef RRT_PRIO_REFILL
#define RRT_PRIO_REFILL 2
#endif
#ifndef RRT_PRIO_NODE
#define RRT_PRIO_NODE 1
#endif
#ifndef RRT_PRIO_LEAF
#define RRT_PRIO_LEAF 2
#endif
#ifndef RRT_PRIO_SHADE
#define RRT_PRIO_SHADE 0
#endif

#include "rrt_device.h"



struct V3 {
    float x, y, z;
};

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ V3 muls(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
// vec3.rs:156-158 dot = (u0*v0 + u1*v1) + u2*v2, here with the two adds fused into the products
// (u0*v0, then fma, fma: one rounding per term instead of two, 3 VALU ops instead of 5 under
// -ffp-contract=off; the oracle's f32 modes use the same form, oracle/rrt_oracle.cpp dot3).
__device__ __forceinline__ float dot(V3 a, V3 b) { return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x)); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {  // vec3.rs cross
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// vec3.rs:168-170 unit_vector = v * (1/len)  (Div<f64> is `(1.0/rhs) * self`, vec3.rs:142-148)
// 1 / s correctly rounded in three instructions instead of the IEEE expansion's twelve: v_rcp_f32
// (1 ulp) and one Newton step by fma. It is the IEEE quotient for every s with |s| in [2^-126,
// 2^126) (exhaustive on the device: rrt_testing_recip_check, tests/test_gpu_recip.py); for s = +-0,
// +-inf and NaN the step's residual is NaN and the estimate, exact there, is kept. The kernel takes
// it for reciprocals of square roots of |v|^2 (>= 2^-75) and of probabilities in [0.05, 0.95].
// RRT_RCP=0: the IEEE division.
#ifndef RRT_RCP
#define RRT_RCP 1
#endif
__device__ __forceinline__ float recip_rn(float s) {
    if (!RRT_RCP) return 1.0f / s;
    const float r = __builtin_amdgcn_rcpf(s);
    const float e = __builtin_fmaf(-s, r, 1.0f);
    return e == e ? __builtin_fmaf(e, r, r) : r;
}

// sqrt(x) correctly rounded for x = +-0 or |x| >= 2^-96 (negative x: NaN, as IEEE; +-inf, NaN): v_sqrt_f32 and the choice
// between its one-ulp neighbours by the sign of the fma remainders — the compiler's own correction
// without the rescaling of small arguments (exhaustive on the device, rrt_testing_recip_check). The
// kernel takes it where the argument is provably 0 or >= 2^-46: |p|^2 of the rejection loop, and
// 1 - c^2 / |1 - |perp|^2| (0 or multiples of 2^-24 near 1). RRT_RCP=0: the library sqrt.
__device__ __forceinline__ float sqrt_rn_big(float x) {
    if (!RRT_RCP) return __builtin_sqrtf(x);
    float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    s = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : s;
}

// sqrt(x) correctly rounded for any x: sqrt_rn_big unless an active lane of the wave holds a
// nonzero |x| < 2^-96 (a wave-uniform branch to the library sequence; sqrt_rn_big differs from the
// IEEE root only on positive and negative arguments below 2^-96 other than +-0, per the device check)
__device__ __forceinline__ float sqrt_rn(float x) {
    if (!RRT_RCP) return __builtin_sqrtf(x);
    if (__ballot(__builtin_fabsf(x) < 0x1.0p-96f && x != 0.0f) == 0) return sqrt_rn_big(x);
    return __builtin_sqrtf(x);
}

__device__ __forceinline__ V3 unit(V3 v) {
    const float inv = recip_rn(sqrt_rn(dot(v, v)));
    return muls(v, inv);
}


// vec3.rs:181-189 random_unit_vector: rejection in [-1,1)^3, accept 1e-160 < |p|^2 <= 1
// (1e-160 underflows to 0 in f32: the one intentional f32 deviation).
// The loop only draws and tests; the normalisation runs once after it, with the wave
// converged (inside the loop it would run in every iteration in which any lane accepts).
template <typename C>
__device__ __forceinline__ V3 random_unit_vector(RngState &s, C &cnt) {
    float px, py, pz, lensq;
    for (;;) {
        if constexpr (RRT_PHASE_TIMING == 4) cnt.d2 += wave_slot();
        px = rnd_pm1(s);
        py = rnd_pm1(s);
        pz = rnd_pm1(s);
        lensq = __builtin_fmaf(pz, pz, __builtin_fmaf(py, py, px * px));
        if (RRT_DEBUG_NOREJECT || (0.0f < lensq && lensq <= 1.0f)) break;  // (debug: first candidate)
    }
    const float inv = recip_rn(sqrt_rn_big(lensq));  // lensq >= 2^-46
    return v3(px * inv, py * inv, pz * inv);
}

// vec3.rs:201-203 reflect = v - n*(2*dot(v,n))
__device__ __forceinline__ V3 reflect(V3 v, V3 n) { return sub(v, muls(n, 2.0f * dot(v, n))); }

// vec3.rs:205-210 refract
__device__ __forceinline__ V3 refract(V3 uv, V3 n, float e) {
    float c = -dot(uv, n);
    c = (c < 1.0f) ? c : 1.0f;
    const V3 perp = muls(add(uv, muls(n, c)), e);
    const float k = __builtin_fabsf(1.0f - dot(perp, perp));
    const V3 par = muls(n, -sqrt_rn_big(k));  // k = 0 or >= 2^-24
    return add(perp, par);
}

// material.rs:75-80 Schlick at a given r0 = ((1 - ri) / (1 + ri))^2; powi(5) expands to x*((x*x)*(x*x)).
__device__ __forceinline__ float reflectance_r0(float cosine, float r0) {
    const float x = 1.0f - cosine;
    const float x2 = x * x;
    const float x4 = x2 * x2;
    const float x5 = x * x4;
    return r0 + (1.0f - r0) * x5;
}

// A dielectric hit's (ri, r0): from the material record the host formed (rrt_host.cpp
// dielectric_consts: a = (1 / eta, r0(1 / eta), r0(eta)), the same f32 operations), or divided here
#ifndef RRT_DIEL_HOST
#define RRT_DIEL_HOST 1
#endif
__device__ __forceinline__ void dielectric_ri_r0(const GMaterial &m, bool front, float &ri, float &r0) {
    const float eta = __int_as_float(m.b.y);
    if (RRT_DIEL_HOST) {
        ri = front ? m.a.x : eta;
        r0 = front ? m.a.y : m.a.z;
    } else {
        ri = front ? (1.0f / eta) : eta;
        const float q = (1.0f - ri) / (1.0f + ri);
        r0 = q * q;
    }
}

// ---- deterministic f32 acos / atan2 for sphere UV (sphere.rs:46-52) -------------------------
// Cephes single-precision polynomials, only + - * / sqrt, replicated bit-for-bit by the oracle.
constexpr float kPi = 3.14159265358979323846f;
constexpr float kPiO2 = 1.57079632679489661923f;
constexpr float kPiO4 = 0.78539816339744830962f;
// x / c for the texture coordinates' constant divisors (2 pi, pi; the_next_week/sphere.rs:50-51):
// q = x RN(1/c), then one fma correction of the remainder (Markstein's step), three instructions
// against the IEEE expansion's ten. It returns the IEEE quotient for x = 0 and every f32 x in
// [2^-100, 8] (exhaustive for both divisors, tests/test_div_const.py; over all positive floats the
// only differences lie below 3.1e-32, where the remainder underflows); phi is 0 or >= 2^-22
// (atan2 + pi), theta 0 or >= 3e-4 (acos). RRT_DIV_CONST=0: the IEEE division.
#ifndef RRT_DIV_CONST
#define RRT_DIV_CONST 1
#endif
__device__ __forceinline__ float div_by_const(float x, float c) {
    if (!RRT_DIV_CONST) return x / c;
    const float rc = 1.0f / c;  // folded: RN(1/c)
    const float q = x * rc;
    return __builtin_fmaf(__builtin_fmaf(-q, c, x), rc, q);
}

__device__ __forceinline__ float asin_core(float x) {  // |x| <= 0.5 polynomial, z = x*x
    const float z = x * x;
    return ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
            1.6666752422e-1f) * z * x + x;
}
__device__ __forceinline__ float rrt_acosf(float x) {
    if (x < -0.5f) return kPi - 2.0f * asin_core(__builtin_sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_core(__builtin_sqrtf(0.5f * (1.0f - x)));
    return kPiO2 - asin_core(x);
}
__device__ __forceinline__ float rrt_atanf(float x) {
    float sgn = 1.0f;
    if (x < 0.0f) { sgn = -1.0f; x = -x; }
    float y = 0.0f;
    if (x > 2.414213562373095f) { y = kPiO2; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y = kPiO4; x = (x - 1.0f) / (x + 1.0f); }
    const float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x);
    return sgn * y;
}
__device__ __forceinline__ float rrt_atan2f(float y, float x) {
    if (x == 0.0f) {
        if (y > 0.0f) return kPiO2;
        if (y < 0.0f) return -kPiO2;
        return 0.0f;
    }
    float z = rrt_atanf(y / x);
    if (x < 0.0f) z = (y < 0.0f) ? z - kPi : z + kPi;
    return z;
}

// ---- ray/box slab test (role of Aabb::hit, aabb.rs:52-85) -----------------------------------
// A box test only prunes: which sphere is hit, and at which t, is decided by the sphere test
// alone (sphere.rs:24-51 against the running closest hit), so the slab arithmetic need not be
// the reference's op for op. This is the standard GPU form: t = lo*inv - o*inv as one FMA per
// plane, near/far via min/max, entry = max3, exit = min3. It can only differ from the
// reference's slab in grazing cases at the last ulp, where the reference's own result already
// depends on its BVH topology ("Parity"); the host grows every stored box by the
// rounding bound of this arithmetic (rrt_host.cpp BoxSlack), so the test is conservative. A
// zero direction component gives inv = +-2^64 (ray_consts), i.e. plane distances of +-huge
// with the sign of (P - o): the ray is inside that slab for all t, or outside it.
__device__ __forceinline__ bool box_hit(float lx, float hx, float ly, float hy, float lz, float hz,
                                        V3 inv, V3 oi, float tmin, float tmax, float &tnear) {
    const float x0 = __builtin_fmaf(lx, inv.x, -oi.x), x1 = __builtin_fmaf(hx, inv.x, -oi.x);
    const float y0 = __builtin_fmaf(ly, inv.y, -oi.y), y1 = __builtin_fmaf(hy, inv.y, -oi.y);
    const float z0 = __builtin_fmaf(lz, inv.z, -oi.z), z1 = __builtin_fmaf(hz, inv.z, -oi.z);
    const float nr = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(x0, x1), __builtin_fminf(y0, y1)),
                                     __builtin_fmaxf(__builtin_fminf(z0, z1), tmin));
    const float fr = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(x0, x1), __builtin_fmaxf(y0, y1)),
                                     __builtin_fminf(__builtin_fmaxf(z0, z1), tmax));
    tnear = nr;
    return nr < fr;
}

// box_hit on planes given in (entry, exit) order per axis (GNode's lo, hi, lo layout read at
// the ray's sign offsets): fma is monotonic in P for a fixed multiplier, so the entry plane's
// distance is exactly min(t_lo, t_hi) and the exit plane's exactly the max — the same values
// and decisions as box_hit, without its six min/max.
__device__ __forceinline__ bool box_hit_ordered(float nx, float fx, float ny, float fy, float nz, float fz, V3 inv,
                                                V3 oi, float tmin, float tmax, float &tnear) {
    const float x0 = __builtin_fmaf(nx, inv.x, -oi.x), x1 = __builtin_fmaf(fx, inv.x, -oi.x);
    const float y0 = __builtin_fmaf(ny, inv.y, -oi.y), y1 = __builtin_fmaf(fy, inv.y, -oi.y);
    const float z0 = __builtin_fmaf(nz, inv.z, -oi.z), z1 = __builtin_fmaf(fz, inv.z, -oi.z);
    const float nr = __builtin_fmaxf(__builtin_fmaxf(x0, y0), __builtin_fmaxf(z0, tmin));
    const float fr = __builtin_fminf(__builtin_fminf(x1, y1), __builtin_fminf(z1, tmax));
    tnear = nr;
    return nr < fr;
}


// Per-ray constants of the box and sphere tests. Recomputed from (o, d) each time a wave
// enters its traversal loop rather than kept alive across shading (same IEEE ops, so the
// same values): 7 fewer registers held by lanes parked mid-tree.
struct RayK {
    V3 inv;
    V3 oi;     // o * inv
    float a;
    float ra;  // refined reciprocal of a (0 when a is outside [2^-64, 2^64])
    // byte offsets of the ray's (entry, exit) plane pair of each axis in a GNode child box:
    // 12a + 4 when 1/d_a < 0 (hi, lo), else 12a (lo, hi)
    uint32_t ox, oy, oz;
};

// minNum / maxNum semantics (a NaN direction gives +2^64, as in the oracle's std::fmin/fmax)
__device__ __forceinline__ float clamp_inv(float v) { return __builtin_fmaxf(__builtin_fminf(v, 0x1.0p64f), -0x1.0p64f); }
// clamp_inv(1 / s) through recip_rn: |s| below 2^-126 (subnormal or zero, where the hardware
// estimate is flushed) has |1 / s| > 2^126 and takes +-2^64 by its sign. Equal to
// clamp_inv(1.0f / s) for every s with |s| < 2^126, NaN included (rrt_testing_recip_check).
__device__ __forceinline__ float clamped_slope(float s) {
    if (!RRT_RCP) return clamp_inv(1.0f / s);
    return __builtin_fabsf(s) < 0x1.0p-126f ? __builtin_copysignf(0x1.0p64f, s) : clamp_inv(recip_rn(s));
}

// kLdsNodes: ox, oy, oz are the byte offsets of the (entry, exit) plane pairs in an LDS GNode; for
// the 32-B f16 nodes read from global memory (RRT_F16_ORDERED) ox packs the rotations that put each
// axis's lo | hi << 16 word in (entry, exit) order — 16 when 1/d_a < 0, else 0 — at bits 0, 5 and 10
// (v_alignbit reads the low 5 bits of its shift), so the traversal holds one register, not three.
#ifndef RRT_F16_ORDERED
#define RRT_F16_ORDERED 1
#endif
// the ordered f16 slab for kernel classes up to this one (book 1 <= 0, book 2 1-3; all by default):
// C5 +7.9 %, bouncing spheres +4.7 %, final_scene +3.0 % same-box (profiles/r6_f16_ordered_ab.log).
// The media class (3: final_scene) forms ra per leaf batch to hold the rotation register within its
// 96-VGPR bound (kHoldRa; with ra held it spilled 20 VGPRs and lost 0.4 %, at 4 waves 8.5 %).
#ifndef RRT_F16_ORDERED_MAX_CLASS
#define RRT_F16_ORDERED_MAX_CLASS 3
#endif
// waves per SIMD and block size of the book-1 untextured class (C2) staged in LDS (6: 512 threads).
// Each block stages its own scene copy (C2: 37 KB), which held C2 at three 512-thread blocks per CU;
// two 1024-thread blocks hold two copies and reach 8 waves/SIMD (64 VGPRs, 28 spilled): C2 +4.6 %
// same-box (round 6). 896 x 7 loses 24 %: 14-wave blocks do not pack onto 4 SIMDs twice.
#ifndef RRT_B1U_WAVES
#define RRT_B1U_WAVES 8
#endif
#ifndef RRT_B1U_BLOCK
#define RRT_B1U_BLOCK 1024
#endif
// waves per SIMD of the book-1 diffuse-only class (C4) staged in LDS (6: 512-thread blocks); its
// small scenes leave LDS for 8 blocks of 256: C4 +3.1 % at 256 x 8, +2.4 % at 256 x 7 (round 6)
#ifndef RRT_B1D_WAVES
#define RRT_B1D_WAVES 8
#endif
// waves per SIMD of the book-2 classes 1-2 for scenes without noise textures
#ifndef RRT_B2_NF_WAVES
#define RRT_B2_NF_WAVES 6
#endif
// waves per SIMD of the book-2 media class (3) for scenes read from L2 (0: kBook2Waves)
#ifndef RRT_B2_MEDIA_GLOBAL_WAVES
#define RRT_B2_MEDIA_GLOBAL_WAVES 0
#endif
// The reciprocal step of the IEEE f32 division expansion (v_rcp + one Newton step) of a = |d|^2, done
// once per ray (or per leaf batch) instead of in every root division (div_by_a); 0 outside
// [2^-64, 2^64].
__device__ __forceinline__ float refine_ra(float a) {
    const float r0 = __builtin_amdgcn_rcpf(a);
    const float e = __builtin_fmaf(-a, r0, 1.0f);
    return (a >= 0x1.0p-64f && a <= 0x1.0p64f) ? __builtin_fmaf(e, r0, r0) : 0.0f;
}
// kHoldRa = false: ra is formed per leaf batch (trav_leaves) from a, so the node steps hold one
// register less (the media class with the ordered f16 slab, which spills at its 96-VGPR bound).
template <bool kLdsNodes = true, bool kHoldRa = true>
__device__ __forceinline__ RayK ray_consts(V3 o, V3 d) {
    RayK r;
    // aabb.rs:58 adinv, hoisted per ray, clamped to +-2^64: a zero component then gives a huge
    // finite slope, so fma(P, inv, -o*inv) keeps the sign of (P - o). Unclamped, inf * P - inf * o
    // is NaN or -inf, and a slab that straddles o (lo < 0 < hi about o's sign) rejects the ray.
    r.inv = v3(clamped_slope(d.x), clamped_slope(d.y), clamped_slope(d.z));
    r.oi = v3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
    if (kLdsNodes) {
        r.ox = r.inv.x < 0.0f ? 4u : 0u;
        r.oy = r.inv.y < 0.0f ? 16u : 12u;
        r.oz = r.inv.z < 0.0f ? 28u : 24u;
    } else {
        r.ox = (r.inv.x < 0.0f ? 16u : 0u) | (r.inv.y < 0.0f ? 16u << 5 : 0u) | (r.inv.z < 0.0f ? 16u << 10 : 0u);
        r.oy = r.oz = 0u;
    }
    r.a = dot(d, d);                                  // sphere.rs:27, hoisted per ray
    r.ra = kHoldRa ? refine_ra(r.a) : 0.0f;
    return r;
}

// n / a, correctly rounded: the quotient steps of the compiler's IEEE f32 division expansion
// (q = n*r, two remainder corrections by fma) on the per-ray reciprocal. For a in
// [2^-64, 2^64] the expansion's v_div_scale / v_div_fmas / v_div_fixup are identities except
// when |n| < 2^-103, where both results are below the 0.001 acceptance bound, so every
// accept/reject decision and every accepted root equals the IEEE quotient (the oracle's).
template <bool kFast = false>
__device__ __forceinline__ float div_by_a(float n, const RayK &rk) {
    if (!kFast && rk.ra == 0.0f) return n / rk.a;
    const float q0 = n * rk.ra;
    const float e0 = __builtin_fmaf(-rk.a, q0, n);
    const float q1 = __builtin_fmaf(e0, rk.ra, q0);
    const float e1 = __builtin_fmaf(-rk.a, q1, n);
    return __builtin_fmaf(e1, rk.ra, q1);
}

// Sphere centers as the sphere test sees them: static, or (book-2 scenes) a moving sphere's
// center at the ray's time, center1 + time * (center2 - center1) (the_next_week/sphere.rs:44:
// Ray::at; static book-2 spheres carry a zero motion).
// kBook2: 0 = book-1 scenes, 1 = book 2 (motion, procedural textures), 2 = book 2 with quads,
// 3 = book 2 with quads and media, 4 = book 3 (all of book 2 + the MIS integrator);
// kBook1Untextured (-1) = book-1 scenes without an image-textured material: the texture path
// (acos, atan2, the texel fetch) is compiled out. It is dead code at run time in such scenes, but
// it costs registers: the C2 kernel spills 19 SGPRs instead of 33 without it, C2 +1.0 % same-box.
constexpr int kBook1Untextured = -1;
// kBook1Diffuse (-2) = book-1 scenes whose materials are all Lambertian (plain or image-textured)
// or emissive: the metal and dielectric branches are compiled out (C4, C1).
constexpr int kBook1Diffuse = -2;
template <int kBook2>
struct Prims {
    const float4 *cr;
    const float4 *mo;
    float time;
    const GQuad *qd;  // book-2 scenes: quads, tagged in cr by a negative w (-(1 + index))
    const GMedium *md;  // media, tagged -(1 + n_quads + index)
    uint32_t n_quads;
    uint64_t seg;  // the path's RNG state at this segment ^ (bounce << 32): key of the media draws
    const GPerlin *perlin;  // Perlin tables (LDS copy when staged, else KParams.perlin)
    static constexpr bool kHasQuads = kBook2 >= 2;
    static constexpr bool kHasMedia = kBook2 >= 3;
    // Book-1 scenes store r * r (f32, rounded as the test would round it) in the record's w and
    // 1 / r (the normal's IEEE quotient, sphere.rs:48 through vec3.rs:142-148) in the material
    // record's b.w (rrt_host.cpp): one multiply less per sphere test, one division less per hit.
    static constexpr bool kR2 = kBook2 <= 0;
    __device__ __forceinline__ float4 at(int i) const {
        float4 m;
        return at(i, m);
    }
    // also returns the motion record: a quad's (normal, D)
    __device__ __forceinline__ float4 at(int i, float4 &m) const {
        float4 c = cr[i];
        if constexpr (kBook2 > 0) {
            m = mo[i];
            c.x = c.x + time * m.x;
            c.y = c.y + time * m.y;
            c.z = c.z + time * m.z;
        }
        return c;
    }
};

// Quad::hit (the_next_week/quad.rs:61-87) in f32: plane distance, then the hit point's (alpha,
// beta) in the (u, v) frame. The t acceptance is Interval::contains (closed: a quad at exactly
// the running closest t replaces the earlier hit), unlike the sphere's open `surrounds`.
__device__ __forceinline__ bool quad_hit(const GQuad &g, V3 o, V3 d, float tmin, float closest, float &t_out) {
    const V3 n = v3(g.n.x, g.n.y, g.n.z);
    const float denom = dot(n, d);
    if (__builtin_fabsf(denom) < 1e-8f) return false;
    const float t = (g.q.w - dot(n, o)) / denom;
    if (!(tmin <= t && t <= closest)) return false;
    const V3 p = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);  // Ray::at
    const V3 hp = v3(p.x - g.q.x, p.y - g.q.y, p.z - g.q.z);
    const V3 w = v3(g.w.x, g.w.y, g.w.z);
    const float alpha = dot(w, cross(hp, v3(g.v.x, g.v.y, g.v.z)));
    const float beta = dot(w, cross(v3(g.u.x, g.u.y, g.u.z), hp));
    if (!(0.0f <= alpha && alpha <= 1.0f && 0.0f <= beta && beta <= 1.0f)) return false;  // is_interior
    t_out = t;
    return true;
}

// quad_hit on the leaf-order records: q and the tag in the primitive slot, (normal, D) in the
// motion slot, so the plane test needs no further fetch; the quad's u, v, w (GQuad) are read only
// for a t inside the interval.
__device__ __forceinline__ bool quad_hit_leaf(const GQuad *g, float4 c, float4 m, V3 o, V3 d, float closest,
                                              float &t_out) {
    const V3 n = v3(m.x, m.y, m.z);
    const float denom = dot(n, d);
    if (__builtin_fabsf(denom) < 1e-8f) return false;
    const float t = (m.w - dot(n, o)) / denom;
    if (!(0.001f <= t && t <= closest)) return false;
    const float4 u = g->u, v = g->v, w4 = g->w;
    const V3 p = v3(o.x + t * d.x, o.y + t * d.y, o.z + t * d.z);  // Ray::at
    const V3 hp = v3(p.x - c.x, p.y - c.y, p.z - c.z);
    const V3 w = v3(w4.x, w4.y, w4.z);
    const float alpha = dot(w, cross(hp, v3(v.x, v.y, v.z)));
    const float beta = dot(w, cross(v3(u.x, u.y, u.z), hp));
    if (!(0.0f <= alpha && alpha <= 1.0f && 0.0f <= beta && beta <= 1.0f)) return false;  // is_interior
    t_out = t;
    return true;
}

// ln(x) in f32 with only + - * and exponent extraction, bit-reproducible by the oracle: Cephes
// logf (x = m * 2^e, m in [sqrt(1/2), sqrt(2)), minimax polynomial in m - 1, ln 2 in two
// parts). x = 0 gives -inf; only called with the media draws, u in [0, 1) on a 2^-24 grid.
__device__ __forceinline__ float rrt_logf(float x) {
    if (x == 0.0f) return -__builtin_inff();
    const uint32_t b = __float_as_uint(x);
    int e = (int)((b >> 23) & 255u) - 126;
    float m = __uint_as_float((b & 0x807fffffu) | 0x3f000000u);  // frexpf: m in [0.5, 1)
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = m + m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float y = ((((((((7.0376836292e-2f * m - 1.1514610310e-1f) * m + 1.1676998740e-1f) * m - 1.2420140846e-1f) * m +
                   1.4249322787e-1f) * m - 1.6668057665e-1f) * m + 2.0000714765e-1f) * m - 2.4999993993e-1f) * m +
               3.3333331174e-1f) * m * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    r = r + 0.693359375f * fe;
    return r;
}

// ConstantMedium::hit (constant_medium.rs:40-84) in f32: the boundary's first hit over
// (-inf, inf) and its next hit after t1 + 0.0001 (Sphere::hit / HittableList over the boundary
// quads), clipped to [0.001, closest]; a free flight of -ln(u)/density along the ray (u: the
// per-(path, segment, medium) draw, include/rrt_hip.h). Returns the scatter t or false.
template <class PR>
__device__ __forceinline__ bool medium_hit(const PR &pr, int m, V3 o, V3 d, const RayK &rk, float closest, float &t_out) {
    const GMedium g = pr.md[m];
    const float inf = __builtin_inff();
    float t1, t2;
    if (g.kind == 0u) {
        const V3 oc = v3(g.sphere.x - o.x, g.sphere.y - o.y, g.sphere.z - o.z);
        const float h = dot(d, oc);
        const float c = dot(oc, oc) - g.sphere.w * g.sphere.w;
        const float disc = __builtin_fmaf(h, h, -(rk.a * c));
        if (disc < 0.0f) return false;
        const float sq = __builtin_sqrtf(disc);
        const float r0 = div_by_a(h - sq, rk), r1 = div_by_a(h + sq, rk);
        // Sphere::hit over (-inf, inf), then over (t1 + 0.0001, inf)
        if (-inf < r0 && r0 < inf) t1 = r0;
        else if (-inf < r1 && r1 < inf) t1 = r1;
        else return false;
        const float lo = t1 + 0.0001f;
        if (lo < r0 && r0 < inf) t2 = r0;
        else if (lo < r1 && r1 < inf) t2 = r1;
        else return false;
    } else {
        t1 = inf;
        bool h1 = false;
        for (uint32_t k = 0; k < g.count; ++k) {
            float t;
            if (quad_hit(pr.qd[g.first + k], o, d, -inf, t1, t)) t1 = t, h1 = true;
        }
        if (!h1) return false;
        const float lo = t1 + 0.0001f;
        t2 = inf;
        bool h2 = false;
        for (uint32_t k = 0; k < g.count; ++k) {
            float t;
            if (quad_hit(pr.qd[g.first + k], o, d, lo, t2, t)) t2 = t, h2 = true;
        }
        if (!h2) return false;
    }
    if (t1 < 0.001f) t1 = 0.001f;
    if (t2 > closest) t2 = closest;
    if (t1 >= t2) return false;
    if (t1 < 0.0f) t1 = 0.0f;
    const float len = __builtin_sqrtf(rk.a);
    const float inside = (t2 - t1) * len;
    const float u = (float)(uint32_t)(splitmix64(pr.seg ^ (uint64_t)m) >> 40) * 0x1.0p-24f;
    const float hd = g.neg_inv_density * rrt_logf(u);
    if (hd > inside) return false;
    t_out = t1 + hd / len;
    return true;
}

// Sphere::hit (sphere.rs:24-51) root selection; returns true and shrinks `closest`.
template <bool kCount, class PR>
__device__ __forceinline__ void test_prims(const PR &prim_cr, int first, int count, V3 o, V3 d,
                                           float a, int skip, float &closest, int &hit_prim, Counters &cnt) {
    static_assert(!PR::kHasQuads, "book-2 scenes (quads, motion) use the binary BVH");
    for (int i = first; i < first + count; ++i) {
        if (kCount) cnt.spheres++;
        if (i == skip) continue;
        const float4 cr = prim_cr.at(i);
        const V3 oc = v3(cr.x - o.x, cr.y - o.y, cr.z - o.z);
        const float h = dot(d, oc);
        const float c = dot(oc, oc) - (PR::kR2 ? cr.w : cr.w * cr.w);
        const float disc = __builtin_fmaf(h, h, -(a * c));
        if (disc < 0.0f) continue;
        const float sq = sqrt_rn(disc);
        float root = (h - sq) / a;
        if (!(0.001f < root && root < closest)) {
            root = (h + sq) / a;
            if (!(0.001f < root && root < closest)) continue;
        }
        closest = root;
        hit_prim = i;
    }
}

// ---- lazy exact roots (book-1 scenes, the non-counting kernel) -------------------------------------
// The closest hit is the lexicographic minimum of (exact root, test order) over the valid roots
// (sphere.rs:24-51 against the running closest, strictly less: the first of equal roots wins), and
// box tests only prune (conservative boxes, BoxSlack). So the leaf loop need not form every root
// exactly: it brackets each root in an interval from the hardware square root and the per-ray
// reciprocal and keeps the best candidate's interval [lo, closest]. A candidate whose interval lies
// wholly below lo replaces the best, one wholly at or above `closest` is rejected (both decisions
// are the exact ones), and only an overlap (nearly equal roots, or a root near tmin) is resolved on
// the exact roots, as the exact loop forms them. The box tests prune with the upper bound `closest`,
// so they visit a superset of the exact walk's nodes in the same order, whose extra primitives the
// exact comparison would reject anyway. The exact root of the winner is formed once, when the query
// ends (lazy_finish): every decision and every t equal the exact loop's, bit for bit (the GPU parity
// suite with the whole C2 frame passed with it on). Measured and left off (round 6, same-box): C2
// -0.1 %, C5 -0.8 %, C4 -4 % — VALU instructions per ray fell only 0.4 % (the winner's exact root at
// the query's end and the interval bookkeeping cost about what the sparse root code did) and SALU
// rose 4.5 % (profiles/r6_lazy_root_ab.log). RRT_LAZY_ROOT=1 turns it on.
#ifndef RRT_LAZY_ROOT
#define RRT_LAZY_ROOT 0
#endif
// The exact root the leaf loop forms (test_range's arithmetic): the near root if above tmin, else the far.
template <bool kFastDiv, class PR>
__device__ __forceinline__ float exact_root(const PR &prim_cr, int i, V3 o, V3 d, const RayK &rk) {
    const float4 cr = prim_cr.at(i);
    const V3 oc = v3(cr.x - o.x, cr.y - o.y, cr.z - o.z);
    const float h = dot(d, oc);
    const float c = dot(oc, oc) - (PR::kR2 ? cr.w : cr.w * cr.w);
    const float disc = __builtin_fmaf(h, h, -(rk.a * c));
    const float sq = sqrt_rn(disc);
    float root = div_by_a<kFastDiv>(h - sq, rk);
    if (!(0.001f < root)) root = div_by_a<kFastDiv>(h + sq, rk);
    return root;
}
// An ambiguous candidate i (its interval overlaps the best's, or its root may lie at tmin): the exact
// loop's decision on the exact roots. hit_prim < 0 or lo == closest: the best is exact already.
template <bool kFastDiv, class PR>
__device__ __forceinline__ void lazy_resolve(const PR &prim_cr, int i, V3 o, V3 d, const RayK &rk, float &lo,
                                             float &closest, int &hit_prim) {
    const float rc = exact_root<kFastDiv>(prim_cr, i, o, d, rk);
    if (0.001f < rc && rc < closest) {  // else rc >= closest >= the best's root: rejected
        const float rb = (hit_prim >= 0 && lo != closest) ? exact_root<kFastDiv>(prim_cr, hit_prim, o, d, rk) : closest;
        if (rc < rb) {
            hit_prim = i;
            lo = closest = rc;
        } else {
            lo = closest = rb;
        }
    }
}
// The query's exact t: the winner's exact root when its interval is still open.
template <class PR>
__device__ __forceinline__ void lazy_finish(const PR &prim_cr, V3 o, V3 d, const RayK &rk, float &lo, float &closest,
                                            int hit_prim) {
    if (hit_prim >= 0 && lo != closest) {
        closest = rk.ra != 0.0f ? exact_root<true>(prim_cr, hit_prim, o, d, rk) : exact_root<false>(prim_cr, hit_prim, o, d, rk);
        lo = closest;
    }
}

// Leaf primitives [first, first + count): the hit leaf children of one node visit, which are
// adjacent in primitive order (sibling leaves split one range, rrt_host.cpp flatten2).
// `skip` is the primitive the ray is leaving (exit_skip): it can never be accepted, so it is left
// out of the loop — a lane whose range holds it runs one iteration less — but the counting
// variant still counts it as a test, like the oracle's hit_prim (tests count every primitive of
// the range). kFastDiv: every active lane's |d|^2 is in the range of the per-ray reciprocal (the
// caller checked it wave-wide), so the root divisions take no branch.
template <bool kCount, bool kFastDiv, class PR>
__device__ __forceinline__ void test_range(const PR &prim_cr, int first, int count, V3 o, V3 d, const RayK &rk,
                                           int skip, float &closest, int &hit_prim, float &lo, Counters &cnt) {
    // lazy roots: book-1 spheres in the non-counting kernel (the counting twin keeps the exact
    // walk, so its test counts stay the oracle's), the per-ray reciprocal in range (kFastDiv)
    constexpr bool kLazy = RRT_LAZY_ROOT && !kCount && kFastDiv && PR::kR2 && !PR::kHasQuads;
    const float a = rk.a;
    const bool trim = (uint32_t)(skip - first) < (uint32_t)count;
    const int n = count - (trim ? 1 : 0);
    const int gap = trim ? skip : 0x7fffffff;
    if (kCount && trim) cnt.spheres++;
    for (int k = 0; k < n; ++k) {
        const int i = first + k + (first + k >= gap ? 1 : 0);
        if (kCount) cnt.spheres++;
        if constexpr (RRT_PHASE_TIMING == 3) {
            cnt.d0 += wave_slot();
            cnt.d1 += 1;
        }
        float4 cr;
        if constexpr (PR::kHasQuads) {
            cr = prim_cr.cr[i];
            const float4 m = prim_cr.mo[i];
            if (cr.w < 0.0f) {
                const int j = (int)(-cr.w) - 1;
                float tq;
                bool hit;
                if (PR::kHasMedia && j >= (int)prim_cr.n_quads) hit = medium_hit(prim_cr, j - (int)prim_cr.n_quads, o, d, rk, closest, tq);
                else hit = quad_hit_leaf(prim_cr.qd + j, cr, m, o, d, closest, tq);
                if (hit) {
                    closest = tq;
                    hit_prim = i;
                }
                continue;
            }
            cr.x = cr.x + prim_cr.time * m.x;  // Prims::at
            cr.y = cr.y + prim_cr.time * m.y;
            cr.z = cr.z + prim_cr.time * m.z;
        } else {
            cr = prim_cr.at(i);
        }
        const V3 oc = v3(cr.x - o.x, cr.y - o.y, cr.z - o.z);
        const float h = dot(d, oc);
        const float c = dot(oc, oc) - (PR::kR2 ? cr.w : cr.w * cr.w);
        const float disc = __builtin_fmaf(h, h, -(a * c));
        // The far root (h + sq) / a is needed only when the near one is at or behind tmin (the
        // ray starts inside the sphere): r1 >= r0 always (sq >= 0, a > 0, correctly rounded
        // quotients are monotone), so r0 >= closest rejects both. A wave skips that rare branch
        // when no lane takes it.
        if (disc < 0.0f) continue;
        if constexpr (RRT_PHASE_TIMING == 3) cnt.d2 += 1;
        if constexpr (kLazy) {
            // Interval of the exact near root r0 = RN(RN(h - RN(sqrt disc)) / a): the hardware root s
            // is within 2 ulp of sqrt(disc) (the exhaustive device check of sqrt_rn_big), so
            // |RN(h - s) - RN(h - sq)| <= 2^-21 s + 2u |h - s| and, with ra within 2u of 1/a,
            // |q - r0| <= 9u ra (|h - s| + s) <= 9u ra (|h| + 2s) (u = 2^-24); e = 2^-20 ra (|h| + 2s)
            // bounds it with 1.7x to spare, which also covers the roundings of e and of q -+ e
            // (e >= 16u |q|). Decided here: the near root surely above tmin, and surely below the
            // best's interval (accept) or surely at or above it (reject). Anything else — a root near
            // tmin, a ray inside the sphere (the far root), overlapping intervals, disc below 2^-96 (the
            // square root's scaled range), an overflow or a NaN — is resolved on the exact roots.
            const float sv = __builtin_amdgcn_sqrtf(disc);
            const float q = (h - sv) * rk.ra;
            const float e = __builtin_fmaf(sv, 2.0f, __builtin_fabsf(h)) * (rk.ra * 0x1.0p-20f);
            const float l = q - e, u = q + e;
            const bool valid = (disc >= 0x1.0p-96f) & (l > 0.001f);
            const bool acc = valid & (u < lo);
            const bool rej = valid & (l >= closest);
            lo = acc ? l : lo;
            closest = acc ? u : closest;
            hit_prim = acc ? i : hit_prim;
            if (!(acc | rej)) lazy_resolve<kFastDiv>(prim_cr, i, o, d, rk, lo, closest, hit_prim);
        } else {
            const float sq = sqrt_rn(disc);
            float root = div_by_a<kFastDiv>(h - sq, rk);
            if (!(0.001f < root)) root = div_by_a<kFastDiv>(h + sq, rk);
            if (RRT_LAZY_ROOT && !kCount && PR::kR2 && !PR::kHasQuads) {
                // exact root against a best that may be an interval (an earlier lazy batch)
                if (0.001f < root && root < closest) {
                    if (root < lo) {
                        lo = closest = root;
                        hit_prim = i;
                    } else {
                        lazy_resolve<kFastDiv>(prim_cr, i, o, d, rk, lo, closest, hit_prim);
                    }
                }
            } else if (0.001f < root && root < closest) {
                closest = root;
                hit_prim = i;
            }
        }
    }
}


// Resumable BVH traversal: one call = one node. The state lives in registers (+ the LDS stack)
// so a wave can leave the traversal loop while some lanes are still mid-tree.
struct Trav {
    float closest;  // the best hit's root, or (lazy roots) an upper bound of it
    int hit_prim;
    int node;
    int sp;
    float lo;       // lazy roots: a lower bound of the best hit's root (== closest when exact)
};

__device__ __forceinline__ void trav_begin(Trav &t) {
    t.closest = __builtin_inff();  // camera.rs:187 Interval(0.001, INFINITY)
    t.lo = __builtin_inff();
    t.hit_prim = -1;
    t.node = 0;
    t.sp = 0;
}


// BVH2 node visit with postponed leaf tests: tests both child boxes against the current
// closest hit, records leaf children in `lv` (tested later, before this lane's next node
// visit), descends into the nearer internal child and pushes the farther one; t.node = -1
// when nothing is left to visit. The next node depends only on these box results, so
// testing the leaves later keeps every ray's sequence of operations unchanged. Returns
// true when leaf tests are pending.
template <bool kCount, bool kOrd16, typename Node, typename Stack>
__device__ __forceinline__ bool trav_node(const Node *__restrict__ nodes, Stack &stack, const RayK &rk, Trav &t,
                                          Leaves &lv, Counters &cnt) {
    if (kCount) { cnt.nodes++; cnt.boxes += 2; }
    float tn0 = 0.0f, tn1 = 0.0f;
    bool h0, h1;
    uint32_t l0, l1;
    if constexpr (std::is_same<Node, GNode>::value) {
        // node * 80 as a 24-bit multiply (full rate; node indices < 2^24)
        const GNode &n = *reinterpret_cast<const GNode *>(reinterpret_cast<const char *>(nodes) +
                                                           __umul24((uint32_t)t.node, (uint32_t)sizeof(GNode)));
        // LDS: each plane pair read at the ray's sign offset (ds_read2_b32), no min/max
        const char *bx = reinterpret_cast<const char *>(&n.box[0][0]);
        auto plane = [&](uint32_t byte_off) { return *reinterpret_cast<const float *>(bx + byte_off); };
        h0 = box_hit_ordered(plane(rk.ox), plane(rk.ox + 4), plane(rk.oy), plane(rk.oy + 4), plane(rk.oz),
                             plane(rk.oz + 4), rk.inv, rk.oi, 0.001f, t.closest, tn0);
        h1 = box_hit_ordered(plane(rk.ox + 36), plane(rk.ox + 40), plane(rk.oy + 36), plane(rk.oy + 40),
                             plane(rk.oz + 36), plane(rk.oz + 40), rk.inv, rk.oi, 0.001f, t.closest, tn1);
        l0 = n.link[0];
        l1 = n.link[1];
    } else {
        // global memory (scenes beyond the LDS budget): the 32-B f16 node in two 16-B loads and
        // the min/max slab (per-lane dword gathers cost more there than the min/max)
        const uint4 *q = reinterpret_cast<const uint4 *>(nodes + t.node);
        const uint4 a = q[0], b = q[1];
#if RRT_DEBUG_EXTRA_NODE_LOAD == 1  // debug builds only: one more 16-B load of the same node (prices node bytes)
        {
            const uint4 *q2 = q;
            asm volatile("" : "+v"(q2));
            const uint4 c = q2[0];
            asm volatile("" ::"v"(c.x ^ c.y ^ c.z ^ c.w));
        }
#endif
#if RRT_DEBUG_EXTRA_NODE_LOAD == 2  // debug: a second load that waits for the first and that the next node waits for
        uint32_t dep_zero;  // (prices one more L2 round trip in the node-to-node chain)
        {
            uint32_t z = a.x;
            asm volatile("v_and_b32 %0, 0, %0" : "+v"(z));
            const uint4 c = q[z];
            dep_zero = c.x;
            asm volatile("v_and_b32 %0, 0, %0" : "+v"(dep_zero));
        }
#endif
        if (kOrd16) {
            // each axis's lo | hi << 16 word rotated by 16 bits when 1/d_a < 0 holds the (entry, exit)
            // pair (the f64 kernel's rotation, rrt_books64.hip): the ordered slab, 6 v_alignbit instead
            // of box_hit's 12 min/max; fma is monotone in the plane, so the same values and decisions
            auto ord = [](uint32_t w, uint32_t r) { return __builtin_amdgcn_alignbit(w, w, r); };
            // the y and z rotations unpacked per node step (asm volatile: not hoisted out of the
            // traversal loop, where they would hold two more registers)
            uint32_t ry, rz;
            asm volatile("v_lshrrev_b32 %0, 5, %1" : "=v"(ry) : "v"(rk.ox));
            asm volatile("v_lshrrev_b32 %0, 10, %1" : "=v"(rz) : "v"(rk.ox));
            const uint32_t x0 = ord(a.x, rk.ox), y0 = ord(a.y, ry), z0 = ord(a.z, rz);
            const uint32_t x1 = ord(a.w, rk.ox), y1 = ord(b.x, ry), z1 = ord(b.y, rz);
            h0 = box_hit_ordered(lo16(x0), hi16(x0), lo16(y0), hi16(y0), lo16(z0), hi16(z0), rk.inv, rk.oi, 0.001f,
                                 t.closest, tn0);
            h1 = box_hit_ordered(lo16(x1), hi16(x1), lo16(y1), hi16(y1), lo16(z1), hi16(z1), rk.inv, rk.oi, 0.001f,
                                 t.closest, tn1);
        } else {
            h0 = box_hit(lo16(a.x), hi16(a.x), lo16(a.y), hi16(a.y), lo16(a.z), hi16(a.z), rk.inv, rk.oi, 0.001f, t.closest, tn0);
            h1 = box_hit(lo16(a.w), hi16(a.w), lo16(b.x), hi16(b.x), lo16(b.y), hi16(b.y), rk.inv, rk.oi, 0.001f, t.closest, tn1);
        }
        l0 = b.z;
        l1 = b.w;
#if RRT_DEBUG_EXTRA_NODE_LOAD == 2
        l0 += dep_zero;
        l1 += dep_zero;
#endif
    }
    // Leaf children (count in the link's top bits, 0 = internal) are postponed; the hit ones
    // form one range: sibling leaves are adjacent in primitive order, so l0's first primitive
    // continues into l1's.
    const uint32_t c0 = h0 ? (l0 >> kLinkCountShift) : 0u;
    const uint32_t c1 = h1 ? (l1 >> kLinkCountShift) : 0u;
    lv = c0 ? l0 + (c1 << kLinkCountShift) : l1;
    if (c0) h0 = false;
    if (c1) h1 = false;
    if (h0 && h1) {
        const bool first1 = tn1 < tn0;
        stack.store(t.sp, first1 ? (int)l0 : (int)l1);
        ++t.sp;
        t.node = first1 ? (int)l1 : (int)l0;
    } else if (h0) {
        t.node = (int)l0;
    } else if (h1) {
        t.node = (int)l1;
    } else if (t.sp == 0) {
        t.node = -1;
    } else {
        --t.sp;
        t.node = stack.load(t.sp);
    }
    return (c0 | c1) != 0;
}

// The postponed leaf tests of one node visit (leaf 0's primitives, then leaf 1's).
template <bool kCount, bool kHoldRa, class PR>
__device__ __forceinline__ void trav_leaves(const PR &prims, Leaves lv, V3 o, V3 d, const RayK &rk_, int skip, Trav &t,
                                            Counters &cnt) {
    RayK rk = rk_;
    if (!kHoldRa) rk.ra = refine_ra(rk.a);
    const int first = (int)(lv & kLinkFirstMask), count = (int)(lv >> kLinkCountShift);
    if (__ballot(rk.ra == 0.0f) == 0) {
        test_range<kCount, true>(prims, first, count, o, d, rk, skip, t.closest, t.hit_prim, t.lo, cnt);
        return;
    }
    test_range<kCount, false>(prims, first, count, o, d, rk, skip, t.closest, t.hit_prim, t.lo, cnt);
}

// BVH4 step: test the 4 child boxes, test leaf children's spheres in place, then descend
// into the nearest internal child and push the others farthest-first (5-exchange sort).
template <bool kCount, typename Stack, class PR>
__device__ __forceinline__ bool trav_step4(const GNode4 *__restrict__ nodes, const PR &prims,
                                           Stack &stack, V3 o, V3 d, const RayK &rk, int skip, Trav &t, Counters &cnt) {
    const GNode4 n = nodes[t.node];
    if (kCount) { cnt.nodes++; cnt.boxes += 4; }
    const float lox[4] = {n.lox.x, n.lox.y, n.lox.z, n.lox.w}, hix[4] = {n.hix.x, n.hix.y, n.hix.z, n.hix.w};
    const float loy[4] = {n.loy.x, n.loy.y, n.loy.z, n.loy.w}, hiy[4] = {n.hiy.x, n.hiy.y, n.hiy.z, n.hiy.w};
    const float loz[4] = {n.loz.x, n.loz.y, n.loz.z, n.loz.w}, hiz[4] = {n.hiz.x, n.hiz.y, n.hiz.z, n.hiz.w};
    const int child[4] = {n.child.x, n.child.y, n.child.z, n.child.w};
    const int count[4] = {n.count.x, n.count.y, n.count.z, n.count.w};
    float key[4];
    int idx[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float tn = 0.0f;
        const bool h = box_hit(lox[c], hix[c], loy[c], hiy[c], loz[c], hiz[c], rk.inv, rk.oi, 0.001f, t.closest, tn);
        key[c] = h ? tn : __builtin_inff();
        idx[c] = child[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        if (count[c] > 0) {
            if (key[c] < __builtin_inff())
                test_prims<kCount>(prims, child[c], count[c], o, d, rk.a, skip, t.closest, t.hit_prim, cnt);
            key[c] = __builtin_inff();
        }
    }
    // a child whose entry lies beyond the (possibly shrunk) closest hit cannot contain a closer hit
#pragma unroll
    for (int c = 0; c < 4; ++c) key[c] = (key[c] < t.closest) ? key[c] : __builtin_inff();
    auto cswap = [&](int i, int j) {
        const bool sw = key[j] < key[i];
        const float ki = key[i], kj = key[j];
        const int ii = idx[i], ij = idx[j];
        key[i] = sw ? kj : ki;
        key[j] = sw ? ki : kj;
        idx[i] = sw ? ij : ii;
        idx[j] = sw ? ii : ij;
    };
    cswap(0, 1);
    cswap(2, 3);
    cswap(0, 2);
    cswap(1, 3);
    cswap(1, 2);
    const float kInf = __builtin_inff();
    if (key[3] < kInf) { stack.store(t.sp, idx[3]); ++t.sp; }
    if (key[2] < kInf) { stack.store(t.sp, idx[2]); ++t.sp; }
    if (key[1] < kInf) { stack.store(t.sp, idx[1]); ++t.sp; }
    if (key[0] < kInf) {
        t.node = idx[0];
        return false;
    }
    if (t.sp == 0) {
        t.node = -1;
        return true;
    }
    --t.sp;
    t.node = stack.load(t.sp);
    return false;
}

// Radiance is only ever added when a path ends (sky/background or an emitter, camera.rs:
// 182-209), so the path carries no running sum: the terminating contribution T*Le goes
// straight into the pixel's sample sum. Bit-identical to L = 0 + T*Le; sum += L, since
// the sum starts at +0 and therefore never becomes -0.
struct PathState {
    V3 o, d, T;
    RngState rng;
    uint32_t k;  // bounce index (camera ray = 0)
    float time;  // the camera ray's time draw, kept by every bounce (book 2, moving spheres)
    int skip;    // leaf-order primitive the current segment leaves (exit_skip), -1 none
};

// The primitive a scattered ray cannot meet again in exact arithmetic, skipped by its next
// closest-hit query (the oracle's exit_skip, oracle/rrt_oracle.cpp): a sphere it leaves
// outward (convex: a ray from its surface with d.n_out > 0 meets it only at t = 0), or the
// quad it leaves (a plane is met once). In f32 the hit point lies up to ~ulp(|center|) off the
// surface and |oc|^2 - r^2 cancels two ~|oc|^2 values (the r = 1000 ground sphere: ulp 0.0625),
// so a grazing bounce would re-hit the surface it leaves past tmin = 0.001 and be trapped
// inside the ground sphere: +0.71 % rays and -0.21 % radiance on C2 against the f64 books
// path, which never does. -1 for a medium, or a ray entering / staying inside a sphere.
// `nrm` faces the incoming ray, so d.nrm > 0 keeps the ray on the side it came from.
__device__ __forceinline__ int exit_skip(bool is_quad, bool is_medium, bool front, V3 dir, V3 nrm, int prim) {
    if (is_medium) return -1;
    if (is_quad) return prim;
    return ((dot(dir, nrm) > 0.0f) == front) ? prim : -1;
}

// Camera::get_ray (camera.rs:152-180) for global pixel (x, y) and the path's RNG.
template <bool kStrat>
__device__ __forceinline__ void camera_ray(const KParams &P, uint32_t x, uint32_t y, uint32_t s, PathState &ps,
                                           Counters &cnt) {
    const auto &C = *kernarg_params();
    float ox, oy;
    if constexpr (kStrat) {  // sample_square_stratified (the_rest_of_your_life/camera.rs:173-177)
        const uint32_t sj = fast_div(s, P.fd_sqrt_spp), si = s - sj * P.sqrt_spp;
        ox = (((float)si + rnd(ps.rng)) * P.recip_sqrt_spp) - 0.5f;
        oy = (((float)sj + rnd(ps.rng)) * P.recip_sqrt_spp) - 0.5f;
    } else {
        // rnd - 0.5 (sample_square): the product u * 2^-24 is exact, so one fma rounds as the sub does
        ox = __builtin_fmaf((float)(rng_next(ps.rng) >> 8), 0x1.0p-24f, -0.5f);
        oy = __builtin_fmaf((float)(rng_next(ps.rng) >> 8), 0x1.0p-24f, -0.5f);
    }
    const float fi = (float)x + ox;
    const float fj = (float)y + oy;
    const V3 sample = v3(C.p00[0] + C.du[0] * fi + C.dv[0] * fj,
                         C.p00[1] + C.du[1] * fi + C.dv[1] * fj,
                         C.p00[2] + C.du[2] * fi + C.dv[2] * fj);
    V3 origin = v3(C.center[0], C.center[1], C.center[2]);
    if (C.defocus_radius > 0.0f) {
        float px, py;
        for (;;) {  // vec3.rs:172-179 random_in_unit_disk
            if constexpr (RRT_PHASE_TIMING == 7) cnt.d2 += wave_slot();
            px = rnd_pm1(ps.rng);
            py = rnd_pm1(ps.rng);
            if (__builtin_fmaf(py, py, px * px) < 1.0f) break;
        }
        origin = v3(C.center[0] + C.disk_u[0] * px + C.disk_v[0] * py,
                    C.center[1] + C.disk_u[1] * px + C.disk_v[1] * py,
                    C.center[2] + C.disk_u[2] * px + C.disk_v[2] * py);
    }
    ps.time = 0.0f;
    if (C.flags & 0x1u) ps.time = rnd(ps.rng);  // RRT_FLAG_RAY_TIME (the_next_week/camera.rs:160)
    ps.skip = -1;
    ps.o = origin;
    ps.d = sub(sample, origin);
    ps.T = v3(1.0f, 1.0f, 1.0f);
    ps.k = 0;
}

__device__ __forceinline__ RngState path_rng(const KParams &P, uint32_t x, uint32_t y, uint32_t s) {
    const uint64_t key = pixel_key(P, x, y);
    return rng_seed(splitmix64(key + s), key);
}

// ---- book-2 procedural textures (the_next_week/texture.rs:39-77, 111-126; perlin.rs) --------
// f32 sin with only + - * and truncation, bit-reproducible by the oracle: Cephes sinf (octant
// reduction by 4/pi with the three-part pi/4 of DP1..DP3, minimax polynomials on [0, pi/4]).
// Arguments >= 2^24 - 1 return 0 (Cephes' total-loss bound); NaN propagates.
__device__ __forceinline__ float rrt_sinf(float xx) {
    float x = xx;
    float sign = 1.0f;
    if (x < 0.0f) { sign = -1.0f; x = -x; }
    if (x > 16777215.0f) return 0.0f;
    if (!(x == x)) return xx;
    int j = (int)(1.27323954473516f * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { sign = -sign; j -= 4; }
    if (x > 8192.0f) x = x - y * 0.7853981633974483096f;
    else x = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    const float z = x * x;
    if (j == 1 || j == 2) {
        y = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
        y = y - 0.5f * z;
        y = y + 1.0f;
    } else {
        y = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x;
        y = y + x;
    }
    return sign < 0.0f ? -y : y;
}

// Cephes cosf: rrt_sinf's reduction, the octant's sign and polynomial for cos.
__device__ __forceinline__ float rrt_cosf(float xx) {
    float x = xx < 0.0f ? -xx : xx;
    if (x > 16777215.0f) return 0.0f;
    if (!(x == x)) return xx;
    float sign = 1.0f;
    int j = (int)(1.27323954473516f * x);
    float y = (float)j;
    if (j & 1) { j += 1; y += 1.0f; }
    j &= 7;
    if (j > 3) { j -= 4; sign = -sign; }
    if (j > 1) sign = -sign;
    if (x > 8192.0f) x = x - y * 0.7853981633974483096f;
    else x = ((x - y * 0.78515625f) - y * 2.4187564849853515625e-4f) - y * 3.77489497744594108e-8f;
    const float z = x * x;
    if (j == 1 || j == 2) {
        y = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f) * z * x;
        y = y + x;
    } else {
        y = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f) * z * z;
        y = y - 0.5f * z;
        y = y + 1.0f;
    }
    return sign < 0.0f ? -y : y;
}

#ifndef RRT_NOISE_UNROLL
#define RRT_NOISE_UNROLL 1
#endif
#ifndef RRT_PERLIN_LDS_PTR
#define RRT_PERLIN_LDS_PTR 1
#endif
#ifndef RRT_DEBUG_NOISE_FIXED  // debug builds only: a constant-time stand-in (prices the texture; wrong images)
#define RRT_DEBUG_NOISE_FIXED 0
#endif

// Rust `f32 as i32` of a floored value: saturating, NaN -> 0.
__device__ __forceinline__ int floor_i32(float x) {
    const float f = __builtin_floorf(x);
    if (!(f == f)) return 0;
    if (f <= -2147483648.0f) return (int)0x80000000;
    if (f >= 2147483647.0f) return 0x7fffffff;
    return (int)f;
}

// The Perlin tables are read through a pointer of type PP: an LDS (address space 3) pointer when
// the block staged them (ds_read, 32-bit addresses), else the generic one.
using LdsPerlin = const __attribute__((address_space(3))) GPerlin *;

template <class Q>
__device__ __forceinline__ V3 gradient(Q randvec, uint32_t idx) { return v3(randvec[idx].x, randvec[idx].y, randvec[idx].z); }

// Perlin::noise (perlin.rs:25-48) + perlin_interp (perlin.rs:79-98), operation order kept:
// the (i*uu + (1-i)*(1-uu)) factors are exactly uu or 1-uu for i in {0,1}.
template <class PP, bool kUnroll = RRT_NOISE_UNROLL>
__device__ __forceinline__ float perlin_noise(PP pt, V3 p) {
    const float fx = __builtin_floorf(p.x), fy = __builtin_floorf(p.y), fz = __builtin_floorf(p.z);
    const float u = p.x - fx, v = p.y - fy, w = p.z - fz;
    const int i = floor_i32(p.x), j = floor_i32(p.y), k = floor_i32(p.z);
    const float uu = u * u * (3.0f - 2.0f * u);
    const float vv = v * v * (3.0f - 2.0f * v);
    const float ww = w * w * (3.0f - 2.0f * w);
    // the two permutation entries per axis, read once (the corner loop indexes them by its bits)
    const uint32_t px0 = pt->perm[(uint32_t)i & 255u] & 0xffu, px1 = pt->perm[(uint32_t)(i + 1) & 255u] & 0xffu;
    const uint32_t py0 = (pt->perm[(uint32_t)j & 255u] >> 8) & 0xffu, py1 = (pt->perm[(uint32_t)(j + 1) & 255u] >> 8) & 0xffu;
    const uint32_t pz0 = (pt->perm[(uint32_t)k & 255u] >> 16) & 0xffu, pz1 = (pt->perm[(uint32_t)(k + 1) & 255u] >> 16) & 0xffu;
    float accum = 0.0f;
    if constexpr (!kUnroll) {
#pragma unroll 1
        for (int corner = 0; corner < 8; ++corner) {  // (di, dj, dk) in perlin_interp's nested order
            const int di = corner >> 2, dj = (corner >> 1) & 1, dk = corner & 1;
            const V3 c = gradient(pt->randvec, (di ? px1 : px0) ^ (dj ? py1 : py0) ^ (dk ? pz1 : pz0));
            const float wx = u - (float)di, wy = v - (float)dj, wz = w - (float)dk;
            const float fi = di ? uu : 1.0f - uu;
            const float fj = dj ? vv : 1.0f - vv;
            const float fk = dk ? ww : 1.0f - ww;
            accum = accum + fi * fj * fk * dot(c, v3(wx, wy, wz));
        }
        return accum;
    }
    // RRT_NOISE_UNROLL: the corner loop unrolled. The corner offsets are constants (u - 0 = u and
    // 0 * uu + 1 * (1 - uu) = 1 - uu exactly, as above), each (fi * fj) is formed once per pair
    // (perlin_interp multiplies left to right: (fi * fj) * fk * dot is the loop's product), and a
    // face's four gradient reads are independent loads in flight together instead of one round
    // trip per corner. Same operations on the same values in the same order: bit-identical.
    const float v1 = v - 1.0f, w1 = w - 1.0f;
    const float fv0 = 1.0f - vv, fw0 = 1.0f - ww;
    const uint32_t q00 = py0 ^ pz0, q01 = py0 ^ pz1, q10 = py1 ^ pz0, q11 = py1 ^ pz1;
#pragma unroll 1
    for (int di = 0; di < 2; ++di) {  // one x face per pass: four reads in flight, not eight
        const uint32_t px = di ? px1 : px0;
        const float wx = di ? u - 1.0f : u;
        const float fi = di ? uu : 1.0f - uu;
        const V3 c0 = gradient(pt->randvec, px ^ q00), c1 = gradient(pt->randvec, px ^ q01);
        const V3 c2 = gradient(pt->randvec, px ^ q10), c3 = gradient(pt->randvec, px ^ q11);
        const float f0 = fi * fv0, f1 = fi * vv;
        accum = accum + f0 * fw0 * dot(c0, v3(wx, v, w));
        accum = accum + f0 * ww * dot(c1, v3(wx, v, w1));
        accum = accum + f1 * fw0 * dot(c2, v3(wx, v1, w));
        accum = accum + f1 * ww * dot(c3, v3(wx, v1, w1));
    }
    return accum;
}

// NoiseTexture::value (texture.rs:122-126): 0.5 * (1 + sin(scale * p.z + 10 * turb(p, 7))),
// turb (perlin.rs:50-62): |sum of weight * noise(p * 2^i)|, weight halving. The octave loop stays
// rolled: unrolled (56 corner evaluations) it swamps the megakernel's register allocation.
#ifndef RRT_NOISE_CALL
#define RRT_NOISE_CALL 1
#endif
#if RRT_NOISE_CALL
#define RRT_NOISE_FN __attribute__((noinline))
#else
#define RRT_NOISE_FN __forceinline__
#endif
template <class PP>
__device__ RRT_NOISE_FN float noise_value(PP pt, float scale, V3 p) {
    if (RRT_DEBUG_NOISE_FIXED) return 0.5f + p.z * 0x1.0p-30f;
    float accum = 0.0f, weight = 1.0f;
    V3 tp = p;
#pragma unroll 1
    for (int o = 0; o < 7; ++o) {
        accum = accum + weight * perlin_noise(pt, tp);
        weight = weight * 0.5f;
        tp = muls(tp, 2.0f);
    }
    const float turb = __builtin_fabsf(accum);
    return 0.5f * (1.0f + rrt_sinf(scale * p.z + 10.0f * turb));
}
// Noise texture `table` at p: a wave-uniform branch on where the block keeps the tables.
template <class KP>
__device__ __forceinline__ float noise_at(const KP &P, const GPerlin *perlin, int table, float scale, V3 p) {
    if (RRT_PERLIN_LDS_PTR && P.perlin_in_lds) return noise_value((LdsPerlin)(perlin + table), scale, p);
    return noise_value(perlin + table, scale, p);
}

#ifndef RRT_NOISE_WAVE
#define RRT_NOISE_WAVE 0
#endif
// x from lane (this lane + n) of the same 16-lane row (DPP row_shl:n; 0 past the row's end)
template <int n>
__device__ __forceinline__ float row_shl(float x) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x100 | n, 0xf, 0xf, true));
}

// NoiseTexture::value for the lanes in `want` (a ballot), evaluated by the whole wave together (every lane
// of the wave must be active). In final_scene a shading pass that meets the noise texture has 3.3
// such lanes on average, and the per-lane evaluation costs the wave all 7 x 8 corners for them.
// Here a pass takes up to 8 noise lanes: lane 8k + o (o < 7) evaluates octave o of the k-th one,
// perlin_noise at p * 2^o (turb's doublings are exact, so that is the value its loop reaches) times
// weight 2^-o (its halvings, exact too); lane 8k folds the seven terms in octave order by DPP row
// shifts, ((0 + t0) + t1) + ... + t6, turb's own left fold; the noise lane pulls the sum back and
// finishes value(). The same operations on the same values: bit-identical to noise_value.
#ifndef RRT_NOISE_WAVE_MAX  // noise lanes per shading pass the wave evaluates together (above: per lane)
#define RRT_NOISE_WAVE_MAX 64
#endif
#ifndef RRT_NOISE_WAVE_CALL
#define RRT_NOISE_WAVE_CALL 0
#endif
#ifndef RRT_WAVE_NOISE_UNROLL  // the corner loop inside the wave pass (rolled: fewer live registers)
#define RRT_WAVE_NOISE_UNROLL 0
#endif
#if RRT_NOISE_WAVE_CALL
#define RRT_WAVE_NOISE_FN __attribute__((noinline))
#else
#define RRT_WAVE_NOISE_FN __forceinline__
#endif
template <class KP>
__device__ RRT_WAVE_NOISE_FN float wave_noise(const KP &P, const GPerlin *perlin, uint64_t want, V3 p, int table,
                                              float scale) {
    const uint32_t lane = __lane_id();
    const uint32_t slot = lane >> 3, oct = lane & 7u;
    const uint64_t below = (1ull << lane) - 1ull;
    float g = 0.0f;
    for (uint64_t need = want; need != 0;) {
        // this pass's source lanes: the first (up to) 8 noise lanes, slot k = the k-th
        uint64_t rest = need;
        int src = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const int b = rest ? __builtin_ctzll(rest) : 0;
            src = slot == (uint32_t)k ? b : src;
            rest &= rest - 1ull;
        }
        const uint64_t pass = need ^ rest;
        const uint32_t n_slots = (uint32_t)__popcll(pass);
        const float qx = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(p.x)));
        const float qy = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(p.y)));
        const float qz = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(p.z)));
        const int tbl = __builtin_amdgcn_ds_bpermute(src << 2, table);
        float term = 0.0f;
        if (oct < 7u && slot < n_slots) {
            const float up = __int_as_float((int)(127u + oct) << 23);    // 2^oct
            const float down = __int_as_float((int)(127u - oct) << 23);  // 2^-oct
            const V3 tp = v3(qx * up, qy * up, qz * up);
            const float nz = (RRT_PERLIN_LDS_PTR && P.perlin_in_lds)
                                 ? perlin_noise<LdsPerlin, RRT_WAVE_NOISE_UNROLL>((LdsPerlin)(perlin + tbl), tp)
                                 : perlin_noise<const GPerlin *, RRT_WAVE_NOISE_UNROLL>(perlin + tbl, tp);
            term = down * nz;
        }
        float acc = 0.0f + term;
        acc = acc + row_shl<1>(term);
        acc = acc + row_shl<2>(term);
        acc = acc + row_shl<3>(term);
        acc = acc + row_shl<4>(term);
        acc = acc + row_shl<5>(term);
        acc = acc + row_shl<6>(term);
        const uint32_t rank = (uint32_t)__popcll(pass & below);
        const float turb_acc = __int_as_float(__builtin_amdgcn_ds_bpermute((int)(rank << 5), __float_as_int(acc)));
        if ((pass >> lane) & 1ull) g = 0.5f * (1.0f + rrt_sinf(scale * p.z + 10.0f * __builtin_fabsf(turb_acc)));
        need = rest;
    }
    return g;
}

// CheckerTexture::value (texture.rs:66-77) with solid even/odd colours.
__device__ __forceinline__ bool checker_even(float inv_scale, V3 p) {
    const int xi = floor_i32(inv_scale * p.x), yi = floor_i32(inv_scale * p.y), zi = floor_i32(inv_scale * p.z);
    const int sum = (int)((uint32_t)xi + (uint32_t)yi + (uint32_t)zi);  // i32 wrapping add
    return sum % 2 == 0;
}

__device__ __forceinline__ V3 texel(const KParams &P, int tex, float u, float v) {
    const GTexture t = P.texs[tex];
    if (t.height <= 0) return v3(0.0f, 1.0f, 1.0f);  // texture.rs:91-93
    u = (u < 0.0f) ? 0.0f : ((u > 1.0f) ? 1.0f : u);  // Interval::clamp
    v = 1.0f - ((v < 0.0f) ? 0.0f : ((v > 1.0f) ? 1.0f : v));
    int i = (int)(u * (float)t.width);
    int j = (int)(v * (float)t.height);
    i = (i < 0) ? 0 : ((i < t.width) ? i : t.width - 1);  // rtw_image.rs:51-52, 70-78
    j = (j < 0) ? 0 : ((j < t.height) ? j : t.height - 1);
    const uint8_t *px = P.tex_pool + t.offset + ((size_t)j * t.width + i) * 3;
    const float cs = 1.0f / 255.0f;
    return v3(cs * (float)px[0], cs * (float)px[1], cs * (float)px[2]);
}

// After the closest-hit query of the current segment (prim < 0: miss): background, or
// emission / scatter / RR (camera.rs:182-209). Returns true when the path has ended; a
// path ending at the sky or an emitter adds T*Le to `sum`.
template <int kBook2, bool kNoise, typename C, class PR>
__device__ __forceinline__ bool shade(const KParams &P, const PR &prims, const GMaterial *mtl, PathState &ps,
                                      float t, int prim, V3 &sum, C &cnt, float gnoise, bool gnoise_ok) {
    if constexpr (RRT_PHASE_TIMING == 4) {
        cnt.d0 += wave_slot();
        cnt.d1 += 1;
    }
    if constexpr (RRT_PHASE_TIMING == 9) cnt.d2 += wave_slot();
    if (prim < 0) {
        if constexpr (RRT_PHASE_TIMING == 6) {
            cnt.d1 += wave_slot();
            cnt.d2 += 1;
        }
        V3 bg;
        if (P.bg_mode == 1u) {
            bg = v3(P.background[0], P.background[1], P.background[2]);
        } else {
            const V3 ud = unit(ps.d);
            const float a = 0.5f * (ud.y + 1.0f);
            bg = v3((1.0f - a) * 1.0f + a * 0.5f, (1.0f - a) * 1.0f + a * 0.7f, (1.0f - a) * 1.0f + a * 1.0f);
        }
        sum = add(sum, mul(ps.T, bg));
        return true;
    }
    // HitRecord (sphere.rs:47-50, hittable.rs:20-32)
    float4 qn;  // a quad's (normal, D): its motion slot
    const float4 cr = prims.at(prim, qn);  // the sphere's center at the ray's time (sphere.rs:48)
    const V3 p = v3(__builtin_fmaf(ps.d.x, t, ps.o.x), __builtin_fmaf(ps.d.y, t, ps.o.y), __builtin_fmaf(ps.d.z, t, ps.o.z));  // Ray::at, fused
    V3 outward;
    bool is_quad = false, is_medium = false;
    if (PR::kHasQuads && cr.w < 0.0f) {  // a quad's plane normal (quad.rs:79); a medium's (1, 0, 0)
        const int j = (int)(-cr.w) - 1;
        if (PR::kHasMedia && j >= (int)prims.n_quads) {
            is_medium = true;
            outward = v3(1.0f, 0.0f, 0.0f);  // constant_medium.rs:76-82 (front_face true)
        } else {
            is_quad = true;
            outward = v3(qn.x, qn.y, qn.z);
        }
    } else {
#ifndef RRT_INVR_HOST
#define RRT_INVR_HOST 1
#endif
        // 1 / r from the host: book 1 in the material record's b.w, books 2 / 3 in the motion
        // record's w (a sphere's motion is xyz only)
        const float inv_r = !RRT_INVR_HOST ? 1.0f / (PR::kR2 ? __int_as_float(mtl[prim].b.w) : cr.w)
                            : PR::kR2      ? __int_as_float(mtl[prim].b.w)
                                           : qn.w;
        outward = v3((p.x - cr.x) * inv_r, (p.y - cr.y) * inv_r, (p.z - cr.z) * inv_r);
    }
    const bool front = dot(ps.d, outward) < 0.0f;
    const V3 nrm = front ? outward : v3(-outward.x, -outward.y, -outward.z);
    const GMaterial m = mtl[prim];
    const int kind = m.b.x;
    V3 att;
    V3 dir;
    if (kind == 4) {  // DiffuseLight: emitted, scatter None
        sum = add(sum, mul(ps.T, v3(m.a.x, m.a.y, m.a.z)));
        return true;
    }
    // Lambertian and Metal both draw one random_unit_vector and nothing else before RR: one
    // rejection loop for both kinds (a wave mixing them runs it once, not twice).
    V3 r = v3(0.0f, 0.0f, 0.0f);
    if (kBook2 == kBook1Diffuse || kind != 2) r = random_unit_vector(ps.rng, cnt);
    if (kBook2 > 0 && kind == 7) {  // Isotropic (material.rs:153-158): a fresh random_unit_vector
        dir = r;
        att = v3(m.a.x, m.a.y, m.a.z);
    } else if (kBook2 == kBook1Diffuse || (kind != 1 && kind != 2)) {  // Lambertian, plain or textured (material.rs:28-40; book 2 :41-53)
        dir = add(nrm, r);
        if (__builtin_fabsf(dir.x) < 1e-8f && __builtin_fabsf(dir.y) < 1e-8f && __builtin_fabsf(dir.z) < 1e-8f) dir = nrm;
        if (kBook2 != kBook1Untextured && kind == 3) {  // ImageTexture at the sphere's (u, v) (sphere.rs:46-52)
#ifndef RRT_DEBUG_TEXEL_FIXED  // debug builds only: no acos / atan2 (prices them; wrong images)
#define RRT_DEBUG_TEXEL_FIXED 0
#endif
            const float theta = RRT_DEBUG_TEXEL_FIXED ? 1.0f + outward.y * 0x1.0p-30f : rrt_acosf(-outward.y);
            const float phi = RRT_DEBUG_TEXEL_FIXED ? 2.0f + outward.x * 0x1.0p-30f : rrt_atan2f(-outward.z, outward.x) + kPi;
            att = texel(P, m.b.z, div_by_const(phi, 2.0f * kPi), div_by_const(theta, kPi));
        } else if (kBook2 > 0 && kind == 5) {  // CheckerTexture at p
            att = checker_even(m.a.w, p) ? v3(m.a.x, m.a.y, m.a.z)
                                         : v3(__int_as_float(m.b.y), __int_as_float(m.b.z), __int_as_float(m.b.w));
        } else if (kBook2 > 0 && kNoise && kind == 6) {  // NoiseTexture at p
            if constexpr (RRT_PHASE_TIMING == 9) {
                cnt.d0 += wave_slot();
                cnt.d1 += 1;
            }
            // evaluated by the wave before shading (RRT_NOISE_WAVE: gnoise_ok, wave-uniform), or here
            const float g = gnoise_ok ? gnoise : noise_at(P, prims.perlin, m.b.z, m.a.w, p);
            att = v3(g, g, g);
        } else {
            att = v3(m.a.x, m.a.y, m.a.z);
        }
    } else if (kind == 1) {  // Metal (material.rs:53-64)
        if constexpr (RRT_PHASE_TIMING == 5) cnt.d2 += wave_slot();
        if constexpr (RRT_PHASE_TIMING == 6) cnt.d0 += 1;
        const V3 refl = unit(reflect(ps.d, nrm));
        dir = add(refl, muls(r, m.a.w));
        if (!(dot(dir, nrm) > 0.0f)) return true;  // absorbed
        att = v3(m.a.x, m.a.y, m.a.z);
    } else {  // Dielectric (material.rs:83-102)
        if constexpr (RRT_PHASE_TIMING == 5) {
            cnt.d0 += wave_slot();
            cnt.d1 += 1;
        }
        float ri, r0;
        dielectric_ri_r0(m, front, ri, r0);
        const V3 ud = unit(ps.d);
        float c = -dot(ud, nrm);
        c = (c < 1.0f) ? c : 1.0f;
        const float sn = sqrt_rn_big(1.0f - c * c);  // 0 or >= 2^-24
        const bool cannot = ri * sn > 1.0f;
        if (cannot || reflectance_r0(c, r0) > rnd(ps.rng)) dir = reflect(ud, nrm);
        else dir = refract(ud, nrm, ri);
        att = v3(1.0f, 1.0f, 1.0f);
    }
    if (ps.k >= 5u) {  // camera.rs:189-200
        float pr = att.x;
        if (att.y > pr) pr = att.y;
        if (att.z > pr) pr = att.z;
        if (pr < 0.05f) pr = 0.05f;
        if (pr > 0.95f) pr = 0.95f;
        if (rnd(ps.rng) > pr) return true;
        // Book-1 scenes without image textures: a Lambertian's or a metal's att is its albedo, so
        // 1 / pr is a material constant the host formed in the same operations (rrt_host.cpp
        // rr_inv_pr, in the record's unused b.y); a dielectric's att is (1, 1, 1): pr = 0.95. (The
        // textured classes divide: the select costs C4's 80-VGPR class a spill.)
#ifndef RRT_PR_HOST
#define RRT_PR_HOST 1
#endif
        float inv_pr;
        if (RRT_PR_HOST && kBook2 == kBook1Untextured) inv_pr = kind == 2 ? 1.0f / 0.95f : __int_as_float(m.b.y);
        else inv_pr = recip_rn(pr);
        ps.T = muls(mul(ps.T, att), inv_pr);
    } else {
        ps.T = mul(ps.T, att);
    }
    ps.o = p;
    ps.d = dir;
    ps.k++;
    ps.skip = exit_skip(is_quad, is_medium, front, dir, nrm, prim);
    return false;
}

// ---- book 3 (the_rest_of_your_life): pdfs, light sampling, the MIS shading step ---------------
// Onb::new(n).transform(a) (onb.rs:8-33): w = unit(n), a helper axis, v = unit(w x axis), u = w x v.
__device__ __forceinline__ V3 onb_transform(V3 n, V3 a) {
    const V3 w = unit(n);
    const V3 ax = (__builtin_fabsf(w.x) > 0.9f) ? v3(0.0f, 1.0f, 0.0f) : v3(1.0f, 0.0f, 0.0f);
    const V3 v = unit(cross(w, ax));
    const V3 u = cross(w, v);
    return v3(a.x * u.x + a.y * v.x + a.z * w.x, a.x * u.y + a.y * v.y + a.z * w.y, a.x * u.z + a.y * v.z + a.z * w.z);
}

// Sphere::hit's root over (tmin, inf) for a static sphere (IEEE division: the light-pdf path).
__device__ __forceinline__ bool sphere_root(float4 c, V3 o, V3 d, float tmin) {
    const V3 oc = v3(c.x - o.x, c.y - o.y, c.z - o.z);
    const float a = dot(d, d);
    const float h = dot(d, oc);
    const float cc = dot(oc, oc) - c.w * c.w;
    const float disc = __builtin_fmaf(h, h, -(a * cc));
    if (disc < 0.0f) return false;
    const float sq = __builtin_sqrtf(disc);
    const float inf = __builtin_inff();
    float root = (h - sq) / a;
    if (!(tmin < root && root < inf)) {
        root = (h + sq) / a;
        if (!(tmin < root && root < inf)) return false;
    }
    return true;
}

// HittableList::pdf_value over the light list (hittable_list.rs:60-69): sum of (1/n) * pdf_i,
// Quad::pdf_value (quad.rs:93-102), Sphere::pdf_value (sphere.rs:102-115).
__device__ __forceinline__ float lights_pdf(const KParams &P, V3 o, V3 d) {
    const float weight = 1.0f / (float)P.n_lights;
    float sum = 0.0f;
    for (uint32_t l = 0; l < P.n_lights; ++l) {
        const GLight L = P.lights[l];
        float pdf = 0.0f;
        if (L.kind == 0u) {
            const GQuad g = P.quads[L.quad];
            float t;
            if (quad_hit(g, o, d, 0.001f, __builtin_inff(), t)) {
                const float len2 = dot(d, d);
                const float dist2 = t * t * len2;
                const float cosine = __builtin_fabsf(dot(d, v3(g.n.x, g.n.y, g.n.z))) / __builtin_sqrtf(len2);
                pdf = dist2 / (cosine * L.area);
            }
        } else if (sphere_root(L.sphere, o, d, 0.001f)) {
            const V3 oc = v3(L.sphere.x - o.x, L.sphere.y - o.y, L.sphere.z - o.z);
            const float cos_max = __builtin_sqrtf(1.0f - L.sphere.w * L.sphere.w / dot(oc, oc));
            pdf = 1.0f / ((2.0f * kPi) * (1.0f - cos_max));
        }
        sum = sum + weight * pdf;
    }
    return sum;
}

// HittableList::random (hittable_list.rs:71-75): random_int(0, n-1), then Quad::random
// (quad.rs:104-107) or Sphere::random + random_to_sphere (sphere.rs:55-66, 117-122).
__device__ __forceinline__ V3 lights_random(const KParams &P, V3 o, RngState &rng) {
    const int idx = (int)rnd_range(rng, 0.0f, (float)P.n_lights);
    const GLight L = P.lights[idx];
    if (L.kind == 0u) {
        const GQuad g = P.quads[L.quad];
        const float r1 = rnd(rng);
        const V3 a = v3(g.q.x + r1 * g.u.x, g.q.y + r1 * g.u.y, g.q.z + r1 * g.u.z);
        const float r2 = rnd(rng);
        const V3 p = v3(a.x + r2 * g.v.x, a.y + r2 * g.v.y, a.z + r2 * g.v.z);
        return sub(p, o);
    }
    const V3 dir = v3(L.sphere.x - o.x, L.sphere.y - o.y, L.sphere.z - o.z);
    const float d2 = dot(dir, dir);
    const float r1 = rnd(rng), r2 = rnd(rng);
    const float z = 1.0f + r2 * (__builtin_sqrtf(1.0f - L.sphere.w * L.sphere.w / d2) - 1.0f);
    const float phi = (2.0f * kPi) * r1;
    const float sxy = __builtin_sqrtf(1.0f - z * z);
    return onb_transform(dir, v3(rrt_cosf(phi) * sxy, rrt_sinf(phi) * sxy, z));
}

// the_rest_of_your_life/camera.rs:184-254 in throughput form. Metal / dielectric keep the
// book-2 scatter (skip_pdf); Lambertian (cosine pdf) and Isotropic (sphere pdf) sample the
// mixture 0.5 * lights + 0.5 * material and weight by scattering_pdf / (pdf * rr).
template <bool kNoise, typename C, class PR>
__device__ __forceinline__ bool shade_b3(const KParams &P, const PR &prims, const GMaterial *mtl, PathState &ps,
                                         float t, int prim, V3 &sum, C &cnt, float gnoise, bool gnoise_ok) {
    if (prim < 0) {
        sum = add(sum, mul(ps.T, v3(P.background[0], P.background[1], P.background[2])));
        return true;
    }
    float4 qn;  // a quad's (normal, D): its motion slot
    const float4 cr = prims.at(prim, qn);
    const V3 p = v3(__builtin_fmaf(ps.d.x, t, ps.o.x), __builtin_fmaf(ps.d.y, t, ps.o.y), __builtin_fmaf(ps.d.z, t, ps.o.z));  // Ray::at, fused
    V3 outward;
    bool is_quad = false, is_medium = false;
    if (cr.w < 0.0f) {
        const int j = (int)(-cr.w) - 1;
        if (j >= (int)prims.n_quads) {
            is_medium = true;
            outward = v3(1.0f, 0.0f, 0.0f);
        } else {
            is_quad = true;
            outward = v3(qn.x, qn.y, qn.z);
        }
    } else {
        const float inv_r = RRT_INVR_HOST ? qn.w : 1.0f / cr.w;  // 1 / r from the host (shade)
        outward = v3((p.x - cr.x) * inv_r, (p.y - cr.y) * inv_r, (p.z - cr.z) * inv_r);
    }
    const bool front = (cr.w < 0.0f && (int)(-cr.w) - 1 >= (int)prims.n_quads) ? true : dot(ps.d, outward) < 0.0f;
    const V3 nrm = front ? outward : v3(-outward.x, -outward.y, -outward.z);
    const GMaterial m = mtl[prim];
    const int kind = m.b.x;
    if (kind == 4) {  // DiffuseLight: one-sided (material.rs:155-160), scatter None
        if (front) sum = add(sum, mul(ps.T, v3(m.a.x, m.a.y, m.a.z)));
        return true;
    }
    V3 att, dir;
    if (kind == 1 || kind == 2) {  // skip_pdf: the book-2 metal / dielectric scatter + RR
        if (kind == 1) {
            const V3 r = random_unit_vector(ps.rng, cnt);
            const V3 refl = unit(reflect(ps.d, nrm));
            dir = add(refl, muls(r, m.a.w));
            att = v3(m.a.x, m.a.y, m.a.z);
            // book 3 has no absorption test: the skip_pdf ray is followed whatever its direction
        } else {
            float ri, r0;
            dielectric_ri_r0(m, front, ri, r0);
            const V3 ud = unit(ps.d);
            float c = -dot(ud, nrm);
            c = (c < 1.0f) ? c : 1.0f;
            const float sn = sqrt_rn_big(1.0f - c * c);  // 0 or >= 2^-24
            const bool cannot = ri * sn > 1.0f;
            if (cannot || reflectance_r0(c, r0) > rnd(ps.rng)) dir = reflect(ud, nrm);
            else dir = refract(ud, nrm, ri);
            att = v3(1.0f, 1.0f, 1.0f);
        }
        if (ps.k >= 5u) {
            float pr = att.x;
            if (att.y > pr) pr = att.y;
            if (att.z > pr) pr = att.z;
            if (pr < 0.05f) pr = 0.05f;
            if (pr > 0.95f) pr = 0.95f;
            if (rnd(ps.rng) > pr) return true;
            ps.T = muls(mul(ps.T, att), 1.0f / pr);
        } else {
            ps.T = mul(ps.T, att);
        }
        ps.o = p;
        ps.d = dir;
        ps.k++;
        ps.skip = exit_skip(is_quad, is_medium, front, dir, nrm, prim);
        return false;
    }
    // pdf path: the material's attenuation (texture value at the hit)
    if (kind == 3) {
        const float theta = rrt_acosf(-outward.y);
        const float phi = rrt_atan2f(-outward.z, outward.x) + kPi;
        att = texel(P, m.b.z, div_by_const(phi, 2.0f * kPi), div_by_const(theta, kPi));
    } else if (kind == 5) {
        att = checker_even(m.a.w, p) ? v3(m.a.x, m.a.y, m.a.z)
                                     : v3(__int_as_float(m.b.y), __int_as_float(m.b.z), __int_as_float(m.b.w));
    } else if (kNoise && kind == 6) {
        const float g = gnoise_ok ? gnoise : noise_at(P, prims.perlin, m.b.z, m.a.w, p);
        att = v3(g, g, g);
    } else {
        att = v3(m.a.x, m.a.y, m.a.z);
    }
    float rr = 1.0f;
    if (ps.k >= 5u) {
        rr = att.x;
        if (att.y > rr) rr = att.y;
        if (att.z > rr) rr = att.z;
        if (rr < 0.05f) rr = 0.05f;
        if (rr > 0.95f) rr = 0.95f;
        if (rr < 1.0f && rnd(ps.rng) > rr) return true;
    }
    const bool iso = kind == 7;
    const float inv4pi = 1.0f / (4.0f * kPi);
    if (rnd(ps.rng) < 0.5f) {  // MixturePdf::generate (pdf.rs:92-98): p0 = lights
        dir = lights_random(P, p, ps.rng);
    } else if (iso) {  // SpherePdf::generate
        dir = random_unit_vector(ps.rng, cnt);
    } else {  // CosinePdf::generate: Onb(normal).transform(random_cosine_direction()) (vec3.rs:212-222)
        const float r1 = rnd(ps.rng), r2 = rnd(ps.rng);
        const float phi = (2.0f * kPi) * r1;
        const float sr2 = __builtin_sqrtf(r2);
        dir = onb_transform(nrm, v3(rrt_cosf(phi) * sr2, rrt_sinf(phi) * sr2, __builtin_sqrtf(1.0f - r2)));
    }
    float mat_pdf;
    if (iso) {
        mat_pdf = inv4pi;
    } else {  // CosinePdf::value (pdf.rs:36-44)
        const float cosine = dot(unit(dir), unit(nrm));
        mat_pdf = cosine <= 0.0f ? 0.0f : cosine / kPi;
    }
    const float pdf = 0.5f * lights_pdf(P, p, dir) + 0.5f * mat_pdf;
    if (pdf <= 0.0f) return true;
    float spdf;
    if (iso) {
        spdf = inv4pi;
    } else {  // Lambertian::scattering_pdf (material.rs:56-63)
        const float cosine = dot(nrm, unit(dir));
        spdf = cosine < 0.0f ? 0.0f : cosine / kPi;
    }
    ps.T = mul(ps.T, muls(muls(att, spdf), 1.0f / (pdf * rr)));
    ps.o = p;
    ps.d = dir;
    ps.k++;
    ps.skip = exit_skip(is_quad, is_medium, front, dir, nrm, prim);
    return false;
}


#ifndef RRT_LEAN_8W
#define RRT_LEAN_8W 0
#endif
#ifndef RRT_PKEY_HOLD  // with RRT_LEAN_8W: 0 = the 8-wave class forms the pixel key per path
#define RRT_PKEY_HOLD 0
#endif
#ifndef RRT_SUM_LDS  // with RRT_LEAN_8W: 1 = the 8-wave class keeps its radiance sum in LDS
#define RRT_SUM_LDS 1
#endif
// This lane's radiance-sum slot in LDS (12-B stride: lanes fall on distinct banks).
template <int kBlk>
__device__ __forceinline__ V3 *sum_slot() {
    __shared__ V3 slots[kBlk];
    return &slots[threadIdx.x];
}

// The shading step of the scene class: book 3's MIS integrator or the book-1/2 one.
template <int kBook2, bool kNoise, typename C, class PR>
__device__ __forceinline__ bool shade_any(const KParams &P, const PR &prims, const GMaterial *mtl, PathState &ps,
                                          float t, int prim, V3 &sum, C &cnt, float gnoise, bool gnoise_ok) {
    if constexpr (kBook2 == 4) return shade_b3<kNoise>(P, prims, mtl, ps, t, prim, sum, cnt, gnoise, gnoise_ok);
    else return shade<kBook2, kNoise>(P, prims, mtl, ps, t, prim, sum, cnt, gnoise, gnoise_ok);
}

// Debug builds only (-DRRT_TRACE_X/Y/S): one path's segments, printed at shading.
__device__ __forceinline__ void trace_segment(uint32_t xy, uint32_t s, const PathState &ps, float t, int prim) {
#ifdef RRT_TRACE_X
    if ((xy & 0xffffu) == RRT_TRACE_X && (xy >> 16) == RRT_TRACE_Y && s == RRT_TRACE_S)
        printf("K k=%u o=(%a %a %a) d=(%a %a %a) t=%a prim=%d T=(%a %a %a) rng=%llx\n", ps.k, ps.o.x, ps.o.y, ps.o.z,
               ps.d.x, ps.d.y, ps.d.z, t, prim, ps.T.x, ps.T.y, ps.T.z, (unsigned long long)rng_key(ps.rng));
#endif
}

// kNoise: the scene has Perlin tables (noise textures); false compiles the noise path out (a noise
// material needs a table: the host checks the index).
template <bool kLds, bool kCount, typename StackT, bool kWide, int kBook2, int kBlk, bool kNoise>
__device__ __forceinline__ void render_body(const KParams &P) {
    extern __shared__ uint4 lds_dyn[];
    // LDS layout: [traversal stack: stack_depth x kBlk x StackT, 16-B aligned][nodes][primitives]
    StackT *lds_stack = reinterpret_cast<StackT *>(lds_dyn);
    // BVH2 nodes: sign-ordered 80-B GNode when staged in LDS, 32-B f16 GNodeH in global memory
    using Node = typename std::conditional<kWide, GNode4, typename std::conditional<kLds, GNode, GNodeH>::type>::type;
    const Node *nodes = reinterpret_cast<const Node *>(P.nodes);
    const float4 *prims = P.prim_cr;
    const GMaterial *mtl = P.prim_mtl;
    const float4 *motion = P.prim_motion;
    if constexpr (kLds) {
        // Stage the whole BVH + spheres + their materials (KB-sized) in LDS once per block.
        uint4 *dst = lds_dyn + (P.stack_depth * kBlk * sizeof(StackT) + 15u) / 16u;
        const uint4 *src_n = reinterpret_cast<const uint4 *>(P.nodes);
        const uint32_t nn = P.n_nodes * (uint32_t)(sizeof(Node) / 16);
        for (uint32_t i = threadIdx.x; i < nn; i += kBlk) dst[i] = src_n[i];
        const uint4 *src_p = reinterpret_cast<const uint4 *>(P.prim_cr);
        for (uint32_t i = threadIdx.x; i < P.n_prims; i += kBlk) dst[nn + i] = src_p[i];
        const uint4 *src_m = reinterpret_cast<const uint4 *>(P.prim_mtl);
        const uint32_t nm = P.n_prims * (uint32_t)(sizeof(GMaterial) / 16);
        for (uint32_t i = threadIdx.x; i < nm; i += kBlk) dst[nn + P.n_prims + i] = src_m[i];
        if constexpr (kBook2 > 0) {
            const uint4 *src_v = reinterpret_cast<const uint4 *>(P.prim_motion);
            for (uint32_t i = threadIdx.x; i < P.n_prims; i += kBlk) dst[nn + P.n_prims + nm + i] = src_v[i];
        }
        __syncthreads();
        nodes = reinterpret_cast<const Node *>(dst);
        prims = reinterpret_cast<const float4 *>(dst + nn);
        mtl = reinterpret_cast<const GMaterial *>(dst + nn + P.n_prims);
        if constexpr (kBook2 > 0) motion = reinterpret_cast<const float4 *>(dst + nn + P.n_prims + nm);
    }
    // Perlin tables (5 KB each) staged in LDS after the scene: a noise texture value reads 56
    // lattice corners, each a permutation lookup then a dependent gradient load, so from L2 its
    // 7 octaves are a chain of ~100 round trips.
    const GPerlin *perlin = P.perlin;
    if constexpr (kBook2 > 0) {
        if (P.perlin_in_lds) {
            size_t off16 = (P.stack_depth * kBlk * sizeof(StackT) + 15u) / 16u;
            if constexpr (kLds) off16 += P.n_nodes * (uint32_t)(sizeof(Node) / 16) + 3u * P.n_prims + P.n_prims;
            uint4 *dst = lds_dyn + off16;
            const uint4 *src = reinterpret_cast<const uint4 *>(P.perlin);
            const uint32_t n16 = P.n_perlin * (uint32_t)(sizeof(GPerlin) / 16);
            for (uint32_t i = threadIdx.x; i < n16; i += kBlk) dst[i] = src[i];
            __syncthreads();
            perlin = reinterpret_cast<const GPerlin *>(dst);
        }
    }
    LdsStack<StackT, kBlk> stack;
    stack.init(lds_stack, threadIdx.x);

    // Persistent waves over a global queue of work units. A unit is (pixel, chunk of
    // P.chunk samples); unit ids run tile-major — 64 consecutive ids are the 8x8 pixels of
    // one tile and one chunk, the chunks of a tile follow each other — so a wave's lanes
    // (and every refill) stay spatially coherent. Lanes whose unit is done claim new units
    // together: one atomic per refill, issued by the lowest idle lane.
    const uint32_t lane = threadIdx.x & 63u;
    Counters cnt = {0, 0, 0, 0, 0, 0};
    uint32_t w_rays = 0, w_paths = 0;  // wave-uniform (scalar) ray / path counts
    // Per-lane flags as 0/1 integers (VGPRs) rather than bools (SGPR lane masks), see tr.node.
    uint32_t has = 0;     // lane owns a unit
    bool q_open = true;   // wave-uniform: the queue may still hold units
    // lane's unit: global pixel (x | y << 16), next sample s, end of its sample chunk s_hi
    uint32_t xy = 0, s = 0, s_hi = 0;
    // The 8-wave class (C2's, 1024-thread blocks, 64 VGPRs) frees registers: its pixel key is formed
    // again at each path start instead of held, and its radiance sum lives in LDS (RRT_LEAN_8W).
    constexpr bool kLean = RRT_LEAN_8W && kLds && kBook2 == kBook1Untextured && kBlk >= 1024;
    uint64_t pkey = 0;  // the unit's pixel key (one splitmix64 per unit instead of per path)
    V3 sum_reg = v3(0.0f, 0.0f, 0.0f);
    V3 *sum_ptr;
    if constexpr (kLean && RRT_SUM_LDS) sum_ptr = sum_slot<kBlk>();
    else sum_ptr = &sum_reg;
    V3 &sum = *sum_ptr;
    sum = v3(0.0f, 0.0f, 0.0f);
    PathState ps;
    Trav tr;
    // A lane is in the tree while tr.node >= 0 (or, inside the BVH2 loop, while it holds postponed
    // leaf tests): lane state lives in VGPR integers, so updating it in divergent code is one
    // v_mov instead of the three exec-mask merges a bool held in an SGPR pair costs.
    tr.node = -1;
    uint32_t need_ray = 0;  // the lane must start the next segment of its path
    // wave-uniform: claimed, not yet assigned units; a wave's first claim goes to its block's queue
    uint32_t pool_base = (blockIdx.x & (kQueues - 1u)) * 64u, pool_left = 0;
    [[maybe_unused]] uint64_t ph0 = 0, ph1 = 0, ph2 = 0, tp = 0;
    for (;;) {
        if constexpr (RRT_PHASE_TIMING == 1) tp = __builtin_amdgcn_s_memtime();
        if constexpr (RRT_PHASE_TIMING == 2) ph2++;
        // Issue priority by phase (s_setprio; the SIMD's arbiter prefers the higher one, then the
        // older wave): refill and segment start 2, node steps 1, leaf batches 2, shading 0. A wave
        // that shades runs long divergent code; the others hold its successors' work and LDS
        // requests. Same-box against all-equal priorities: C2 +3.0 %, C4 +3.5 %, C5 +2.4 %.
        __builtin_amdgcn_s_setprio(RRT_PRIO_REFILL);
        uint64_t idle = __ballot(!has);
        if (idle != 0 && pool_left == 0 && q_open) {
            // kQueues interleaved queues with a counter each, 128 B apart: tile-chunk group g (64
            // units) is queue g % kQueues's (g / kQueues)-th claim. One counter took every wave's
            // claims: device-scope atomics on one address serialise, which cost cheap-ray, low-spp
            // frames a third of their time. A claim goes to the queue of pool_base's group: a
            // wave's first claim to queue blockIdx % kQueues (the grid has >= kQueues blocks,
            // launch_variant), and once a claimed group is used up pool_base points at the next
            // group, so the wave's claims rotate q, q + 1, ... through all the queues (the claims
            // are spread over the 8 counters; they do not stay on one XCD's queue). A partial last
            // group leaves pool_base in its queue, whose next claim then fails. Drain: a wave stops
            // claiming at its first failed claim, i.e. at an exhausted queue. Every successful claim
            // on queue q is followed by a claim on q + 1, and queue sizes fall by at most one group
            // from q to q + 1 (G_0 >= G_1 >= ... >= G_7 >= G_0 - 1, the groups dealt g % 8), while
            // queue 0 also takes the first claims of its own blocks' waves: so once any queue is
            // exhausted the next one is too, round the cycle, and every group is claimed
            // (tests/test_gpu_parity.py::test_uneven_queues_drain checks every pixel's count).
            const uint32_t xq = (pool_base >> 6) & (kQueues - 1u);
            uint32_t k = 0;
            if (lane == 0) k = atomicAdd(P.unit_counter + 32u * xq, 1u);
            const uint32_t base = ((uint32_t)__builtin_amdgcn_readlane((int)k, 0) * kQueues + xq) * 64u;
            if (base >= P.n_units) {
                q_open = false;
            } else {
                pool_base = base;
                pool_left = min(64u, P.n_units - base);
            }
        }
        if (idle != 0 && pool_left != 0) {
            const uint32_t n = min((uint32_t)__popcll(idle), pool_left);
            // idle lanes below this one (v_mbcnt: no 64-bit lane mask held across the loop)
            const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
            if (!has && r < n) {
                const uint32_t u = pool_base + r;
                {
                    const auto &Q = *kernarg_params();
                    const uint32_t lit = u & 63u;
                    const uint32_t tc = u >> 6;
                    // big chunks of every tile first, then the tail chunks (small units last)
                    uint32_t t, chunk;
                    if (u < Q.n_big_units) {
                        t = fast_div(tc, fdiv(Q.fd_pass_big));
                        chunk = Q.chunk_begin + (tc - t * Q.pass_big);
                    } else {
                        const uint32_t ns = Q.pass_n - Q.pass_big, tc2 = tc - (Q.n_big_units >> 6);
                        t = fast_div(tc2, fdiv(Q.fd_pass_tail));
                        chunk = Q.chunk_begin + Q.pass_big + (tc2 - t * ns);
                    }
                    const uint32_t ty = fast_div(t, fdiv(Q.fd_tiles_x));
                    const uint32_t x = (t - ty * Q.tiles_x) * kTileW + (lit % kTileW);
                    const uint32_t ly = ty * kTileH + (lit / kTileW);
                    if (x < Q.width && ly < Q.tile_rows) {
                        // tile-local row -> global image row (row bands dealt over ranks in serpentine order, RrtTile)
                        const uint32_t band = fast_div(ly, fdiv(Q.fd_band_rows));
                        const uint32_t slot = (band & 1u) ? Q.n_ranks - 1u - Q.rank : Q.rank;  // serpentine bands
                        const uint32_t y = (band * Q.n_ranks + slot) * Q.band_rows + (ly - band * Q.band_rows);
                        xy = x | (y << 16);
                        s = Q.sample_begin + chunk_first(Q, chunk);
                        s_hi = min(s + (chunk < Q.n_big ? Q.chunk : Q.chunk_small), Q.sample_end);
                        sum = v3(0.0f, 0.0f, 0.0f);
                        const uint64_t key = pixel_key(Q, x, y);
                        if constexpr (!(kLean && !RRT_PKEY_HOLD)) pkey = key;
                        ps.rng = path_rng_k(key, s);
                        camera_ray<kBook2 == 4>(P, x, y, s, ps, cnt);
                        need_ray = 1;
                        has = 1;
                    }
                }
            }
            pool_base += n;
            pool_left -= n;
        }
        if (__ballot(has) == 0) break;

        uint32_t seg_done = 0;  // the lane's path ended without a query (depth limit)
        uint32_t started = 0;   // the lane starts a closest-hit query this iteration
        if (has && need_ray) {
            if (ps.k >= P.max_depth) {  // ray_color: depth <= 0 -> 0 (no query)
                seg_done = 1;
            } else {
                trav_begin(tr);
                need_ray = 0;
                started = 1;
            }
        }
        w_rays += (uint32_t)__popcll(__ballot(started));
        // Traverse until too few lanes of the wave are still in the tree, then let the
        // finished lanes shade and fetch their next segment (wave-uniform ballot exit).
        const uint32_t live = (uint32_t)__popcll(__ballot(has));
        const uint32_t min_active = (live * P.trav_frac) >> 8;
        if constexpr (RRT_PHASE_TIMING == 1) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph0 += t - tp;
            tp = t;
        }
        RayK rk;
        // the ordered f16 slab for scenes read from global memory (C5, bouncing spheres); the media
        // class keeps the min/max slab (RRT_F16_ORDERED_MAX_CLASS)
        constexpr bool kOrd16 = RRT_F16_ORDERED && !kLds && !kWide && kBook2 <= RRT_F16_ORDERED_MAX_CLASS;
        constexpr bool kHoldRa = !(kOrd16 && kBook2 == 3);
        if (tr.node >= 0) rk = ray_consts<!kOrd16, kHoldRa>(ps.o, ps.d);
        const Prims<kBook2> pr{prims, motion, ps.time, P.quads, P.media, P.n_quads, rng_key(ps.rng) ^ ((uint64_t)ps.k << 32), perlin};
        if constexpr (kWide) {
            for (;;) {
                if constexpr (RRT_PHASE_TIMING == 2) {
                    ph0 += 64;
                    ph1 += (uint64_t)__popcll(__ballot(tr.node >= 0));
                }
                if (tr.node >= 0) trav_step4<kCount>(nodes, pr, stack, ps.o, ps.d, rk, ps.skip, tr, cnt);
                if ((uint32_t)__popcll(__ballot(tr.node >= 0)) <= min_active) break;
            }
        } else {
            // BVH2 with postponed leaves: a lane whose visit hit leaf children waits (no further
            // node visits) until the wave runs its leaf loop, which happens once more than
            // leaf_min lanes wait, or no lane can take another node step, or before leaving.
            const uint32_t leaf_min = (live * P.leaf_frac) >> 8;
            __builtin_amdgcn_s_setprio(RRT_PRIO_NODE);  // the node steps (phase priorities: see the loop head)
            Leaves lv = 0;  // the postponed leaf range (0 = none: a range has count >= 1)
            for (;;) {
                if constexpr (RRT_PHASE_TIMING == 2) {
                    ph0 += 64;
                    ph1 += (uint64_t)__popcll(__ballot(tr.node >= 0 && lv == 0));
                }
                if constexpr (RRT_PHASE_TIMING == 8) {  // node steps whose stepping lanes all visit one node
                    const bool stepping = tr.node >= 0 && lv == 0;
                    const uint64_t sm = __ballot(stepping);
                    const int n0 = __builtin_amdgcn_readfirstlane(stepping ? tr.node : 0x7fffffff);
                    const uint64_t same = __ballot(stepping && tr.node == n0);
                    if (sm != 0) {
                        ph0 += 64;
                        if (same == sm) {
                            ph1 += 64;
                            ph2 += (uint64_t)__popcll(sm);
                        }
                    }
                }
                if (tr.node >= 0 && lv == 0) {
                    Leaves l;
                    if (trav_node<kCount, kOrd16>(nodes, stack, rk, tr, l, cnt)) lv = l;
                }
                // wave-uniform decisions in scalar registers, without short-circuit branches:
                // pm = lanes waiting on leaf tests, tm = lanes still in the tree (pm is a subset)
                const uint64_t pm = __ballot(lv != 0);
                const uint64_t tm = __ballot(tr.node >= 0) | pm;
                const bool leave = (uint32_t)__popcll(tm) <= min_active;
                const bool batch = ((uint32_t)__popcll(pm) > leaf_min) | leave | (tm == pm);
                if ((pm != 0) & batch) {
                    __builtin_amdgcn_s_setprio(RRT_PRIO_LEAF);
                    if (lv != 0) {
                        trav_leaves<kCount, kHoldRa>(pr, lv, ps.o, ps.d, rk, ps.skip, tr, cnt);
                        lv = 0;
                    }
                    __builtin_amdgcn_s_setprio(RRT_PRIO_NODE);
                }
                if (leave) break;
            }
        }
        __builtin_amdgcn_s_setprio(RRT_PRIO_SHADE);
        if constexpr (RRT_PHASE_TIMING == 1) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph1 += t - tp;
            tp = t;
        }
        // Noise kernels evaluate the shading lanes' noise textures with the whole wave between the
        // closest-hit query and shade (RRT_NOISE_WAVE): the shading block splits around it. Every
        // lane is active there (the loop leaves on a wave-uniform ballot).
        constexpr bool kWaveNoise = kNoise && RRT_NOISE_WAVE;
        const bool shading = has && !need_ray && tr.node < 0;
        if (shading) {
            need_ray = 1;
            const Prims<kBook2> spr{prims, motion, ps.time, P.quads, P.media, P.n_quads, rng_key(ps.rng) ^ ((uint64_t)ps.k << 32), perlin};
            if constexpr (RRT_LAZY_ROOT && !kCount && Prims<kBook2>::kR2 && !kWide)
                lazy_finish(spr, ps.o, ps.d, rk, tr.lo, tr.closest, tr.hit_prim);  // rk: the lane was in the tree this iteration
            if constexpr (Prims<kBook2>::kHasMedia) {
                // The unbounded media (a fog around the whole scene; rrt_host.cpp unbounded_media):
                // not in the tree, tested here against the closest hit of the walk, every lane whose
                // query ended this iteration together. The same hit as testing them in the tree: the
                // free flight is clipped to the closest hit so far and the draw is fixed per
                // (path, segment, medium). rk is this iteration's: the lane was in the tree.
                if (!kHoldRa) rk.ra = refine_ra(rk.a);
                for (uint32_t u = P.n_prims - P.n_unbounded; u < P.n_prims; ++u) {
                    if (kCount) cnt.spheres++;
                    const int m = (int)(-prims[u].w) - 1 - (int)P.n_quads;
                    float tm;
                    if (medium_hit(spr, m, ps.o, ps.d, rk, tr.closest, tm)) {
                        tr.closest = tm;
                        tr.hit_prim = (int)u;
                    }
                }
            }
            if constexpr (!kWaveNoise) {
                trace_segment(xy, s, ps, tr.closest, tr.hit_prim);
                seg_done = shade_any<kBook2, kNoise>(P, spr, mtl, ps, tr.closest, tr.hit_prim, sum, cnt, 0.0f, false) ? 1u : 0u;
            }
        }
        if constexpr (kWaveNoise) {
            bool want = false;
            int tbl = 0;
            float scale = 0.0f;
            if (shading && tr.hit_prim >= 0) {
                const GMaterial &hm = mtl[tr.hit_prim];
                want = hm.b.x == 6;
                tbl = hm.b.z;
                scale = hm.a.w;
            }
            const V3 ph = v3(__builtin_fmaf(ps.d.x, tr.closest, ps.o.x), __builtin_fmaf(ps.d.y, tr.closest, ps.o.y),
                             __builtin_fmaf(ps.d.z, tr.closest, ps.o.z));  // shade's Ray::at
            // one wave pass for up to RRT_NOISE_WAVE_MAX noise lanes; more are evaluated per lane
            // in shade (perlin_spheres: ~35 per shading pass; final_scene: 3.3)
            const uint64_t nm = __ballot(want);
            const bool gnoise_ok = nm != 0 && (uint32_t)__popcll(nm) <= RRT_NOISE_WAVE_MAX;
            float gnoise = 0.0f;
            if (gnoise_ok) gnoise = wave_noise(P, perlin, nm, ph, tbl, scale);
            if (shading) {
                const Prims<kBook2> spr{prims, motion, ps.time, P.quads, P.media, P.n_quads, rng_key(ps.rng) ^ ((uint64_t)ps.k << 32), perlin};
                trace_segment(xy, s, ps, tr.closest, tr.hit_prim);
                seg_done = shade_any<kBook2, kNoise>(P, spr, mtl, ps, tr.closest, tr.hit_prim, sum, cnt, gnoise, gnoise_ok) ? 1u : 0u;
            }
        }
        w_paths += (uint32_t)__popcll(__ballot(seg_done));
        if (seg_done) {  // pixel_color += ray_color(..) (camera.rs:73-76): already in `sum`
            ++s;
            const uint32_t x = xy & 0xffffu, y = xy >> 16;
            if (s < s_hi) {
                if constexpr (kLean && !RRT_PKEY_HOLD) ps.rng = path_rng_k(pixel_key(*kernarg_params(), x, y), s);
                else ps.rng = path_rng_k(pkey, s);
                if constexpr (RRT_PHASE_TIMING == 7) {
                    cnt.d0 += wave_slot();
                    cnt.d1 += 1;
                }
                camera_ray<kBook2 == 4>(P, x, y, s, ps, cnt);
            } else {  // unit complete: the chunk's sum, in sample order
                const auto &Q = *kernarg_params();
                // chunk index and tile-local row, re-derived from (y, s_hi) once per unit
                const uint32_t rel = s_hi - 1u - Q.sample_begin;
                const uint32_t nbs = Q.n_big * Q.chunk;
                const uint32_t chunk =
                    rel < nbs ? fast_div(rel, fdiv(Q.fd_chunk)) : Q.n_big + fast_div(rel - nbs, fdiv(Q.fd_chunk_small));
                const uint32_t gb = fast_div(y, fdiv(Q.fd_band_rows));
                const uint32_t ly = fast_div(gb, fdiv(Q.fd_n_ranks)) * Q.band_rows + (y - gb * Q.band_rows);
                const size_t px = (size_t)ly * Q.width + x;
                const float4 out = make_float4(sum.x, sum.y, sum.z, (float)(s_hi - (Q.sample_begin + chunk_first(Q, chunk))));
                if (Q.n_chunks == 1) Q.accum[px] = out;
                else Q.partial[(size_t)(chunk - Q.chunk_begin) * ((size_t)Q.tile_rows * Q.width) + px] = F3{sum.x, sum.y, sum.z};
                has = 0;
            }
        }
        if constexpr (RRT_PHASE_TIMING == 1) ph2 += __builtin_amdgcn_s_memtime() - tp;
    }
    if constexpr (((RRT_PHASE_TIMING >= 3 && RRT_PHASE_TIMING <= 7) || RRT_PHASE_TIMING == 9) && !kCount) {
        ph0 = wave_sum_u32(cnt.d0);
        ph1 = wave_sum_u32(cnt.d1);
        ph2 = wave_sum_u32(cnt.d2);
    }
    if constexpr (RRT_PHASE_TIMING != 0 && !kCount) {
        if (lane == 0) {
            atomicAdd(&P.counters[2], (unsigned long long)ph0);
            atomicAdd(&P.counters[3], (unsigned long long)ph1);
            atomicAdd(&P.counters[4], (unsigned long long)ph2);
        }
    }
    // one atomic per wave per counter
    const uint32_t r = w_rays;
    const uint32_t pa = w_paths;
    uint32_t nv = 0, bt = 0, st = 0;
    if (kCount) {
        nv = wave_sum_u32(cnt.nodes);
        bt = wave_sum_u32(cnt.boxes);
        st = wave_sum_u32(cnt.spheres);
    }
    if (lane == 0) {
        if (r) atomicAdd(&P.counters[0], (unsigned long long)r);
        if (pa) atomicAdd(&P.counters[1], (unsigned long long)pa);
        if (kCount) {
            atomicAdd(&P.counters[2], (unsigned long long)nv);
            atomicAdd(&P.counters[3], (unsigned long long)bt);
            atomicAdd(&P.counters[4], (unsigned long long)st);
        }
    }
}

template <bool kLds, bool kCount, typename StackT, bool kWide, int kWaves, int kBook2, int kBlk, bool kNoise>
__global__ __launch_bounds__(kBlk, kWaves) void rrt_render(KParams P) {
    render_body<kLds, kCount, StackT, kWide, kBook2, kBlk, kNoise>(P);
}

// The pass's chunk sums into accum, continuing the left fold over chunks in order: the first
// pass starts from its chunk 0, later passes from the accum so far; w = the tile's sample count.
// partial is [pass chunk][pixel], so each chunk row is read coalesced.
__global__ __launch_bounds__(256) void rrt_combine_chunks(const F3 *__restrict__ partial, float4 *__restrict__ accum,
                                                          uint32_t n_pixels, uint32_t n_chunks, uint32_t first,
                                                          float count) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n_pixels) return;
    float4 acc;
    if (first) {
        const F3 v = partial[p];
        acc = make_float4(v.x, v.y, v.z, 0.0f);
    } else {
        acc = accum[p];
    }
    for (uint32_t c = first ? 1u : 0u; c < n_chunks; ++c) {
        const F3 v = partial[(size_t)c * n_pixels + p];
        acc.x = acc.x + v.x;
        acc.y = acc.y + v.y;
        acc.z = acc.z + v.z;
    }
    accum[p] = make_float4(acc.x, acc.y, acc.z, count);
}

// render_io.rs:3-31 quantiser on the device: x * (1/spp) in f32, non-finite -> 0,
// sqrt(max(0, x)) (correctly rounded), clamp [0, 0.999], (x * 256) as u8 — the same f32 ops
// as the host's quantize_channel, so the bytes are identical. One thread per 4 pixels
// (12 output bytes as 3 dwords when the row of pixels is whole).
__device__ __forceinline__ uint32_t quantize_channel(float x, float scale) {
    float r = x * scale;
    if (!__builtin_isfinite(r)) r = 0.0f;
    r = __builtin_sqrtf(r < 0.0f ? 0.0f : r);
    if (r < 0.0f) r = 0.0f;
    if (r > 0.999f) r = 0.999f;
    return (uint32_t)(int)(r * 256.0f) & 0xffu;
}

__global__ __launch_bounds__(256) void rrt_quantize(const float4 *__restrict__ accum, uint8_t *__restrict__ rgb8,
                                                     uint32_t n_pixels, float scale) {
    const uint32_t q = blockIdx.x * 256u + threadIdx.x;  // group of 4 pixels
    const uint32_t p0 = q * 4u;
    if (p0 >= n_pixels) return;
    if (p0 + 4u <= n_pixels) {
        uint32_t b[12];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 a = accum[p0 + k];
            b[3 * k + 0] = quantize_channel(a.x, scale);
            b[3 * k + 1] = quantize_channel(a.y, scale);
            b[3 * k + 2] = quantize_channel(a.z, scale);
        }
        uint32_t *dst = reinterpret_cast<uint32_t *>(rgb8 + (size_t)p0 * 3u);  // 12-B aligned
#pragma unroll
        for (int w = 0; w < 3; ++w)
            dst[w] = b[4 * w] | (b[4 * w + 1] << 8) | (b[4 * w + 2] << 16) | (b[4 * w + 3] << 24);
    } else {
        for (uint32_t p = p0; p < n_pixels; ++p) {
            const float4 a = accum[p];
            rgb8[p * 3u + 0] = (uint8_t)quantize_channel(a.x, scale);
            rgb8[p * 3u + 1] = (uint8_t)quantize_channel(a.y, scale);
            rgb8[p * 3u + 2] = (uint8_t)quantize_channel(a.z, scale);
        }
    }
}

template <bool kLds, typename StackT, bool kWide, int kBook2, int kWaves = 1, int kBlk = kBlock, int kWavesNF = kWaves>
hipError_t launch_variant(const KParams &p, bool count, hipStream_t stream) {
    // Book 2/3: a noise-free scene runs a kernel without the noise path (the counting twin and the
    // 32-bit-stack kernels keep it: one instantiation each serves both), at kWavesNF waves per SIMD.
    constexpr bool kNoiseFree = kBook2 > 0 && sizeof(StackT) == 2;
    if (p.n_units == 0) return hipSuccess;
    size_t lds = ((size_t)p.stack_depth * kBlk * sizeof(StackT) + 15u) / 16u * 16u;
    if (kLds)
        lds += (size_t)p.n_nodes * (kWide ? sizeof(GNode4) : sizeof(GNode)) +  // LDS BVH2 = GNode
               (size_t)p.n_prims * (kPrimBytes + (kBook2 > 0 ? kMotionBytes : 0));
    if (kBook2 > 0 && p.perlin_in_lds) lds += (size_t)p.n_perlin * sizeof(GPerlin);
    auto kernel = count                       ? rrt_render<kLds, true, StackT, kWide, kWaves, kBook2, kBlk, (kBook2 > 0)>
                  : !kNoiseFree || p.n_perlin ? rrt_render<kLds, false, StackT, kWide, kWaves, kBook2, kBlk, (kBook2 > 0)>
                                              : rrt_render<kLds, false, StackT, kWide, kWavesNF, kBook2, kBlk, false>;
    // Persistent grid: as many blocks as can be resident (occupancy at this LDS size), capped
    // by the work; the queue counter is zeroed on the stream before the launch.
    int per_cu = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlk, lds);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const uint32_t want = (p.n_units + kBlk - 1) / kBlk;
    // at least kQueues blocks, so every work queue has a block (spare blocks find no work and exit)
    const uint32_t blocks = std::max<uint32_t>(std::min<uint32_t>(want, (uint32_t)per_cu * p.n_cus), kQueues);
    e = hipMemsetAsync(p.unit_counter, 0, kQueues * 32u * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(kBlk), lds, stream, p);
    e = hipGetLastError();
    if (e != hipSuccess || p.n_chunks <= 1) return e;
    const uint32_t n_pixels = p.tile_rows * p.width;
    hipLaunchKernelGGL(rrt_combine_chunks, dim3((n_pixels + 255) / 256), dim3(256), 0, stream, p.partial, p.accum,
                       n_pixels, p.pass_n, p.chunk_begin == 0 ? 1u : 0u, (float)(p.sample_end - p.sample_begin));
    return hipGetLastError();
}

template <bool kWide, int kBook2>
hipError_t launch_width(const KParams &p, bool count, hipStream_t stream) {
    if (p.stack_depth > (uint32_t)kMaxStackDepth) return hipErrorInvalidValue;
    if (p.n_nodes > 65535u) return launch_variant<false, uint32_t, kWide, kBook2>(p, count, stream);
    if constexpr (kBook2 > 0) {
        // Book-2 variants (motion, textures, quads) need ~105 VGPRs unbounded. In round 1, with
        // 40-110 spilled SGPRs, a 6-wave bound cost 3-14 % and a 5-wave bound 0-8 %.
        // Book 2 (classes 1-3): 256-thread blocks at 5 waves/SIMD (96 VGPRs). Measured on the
        // 1/4-spp scene table against 512 threads unbounded (~105 VGPRs, 4 waves): +2 ... +16 %
        // on every book-2 scene once the parameter spills were gone (256 x 4: +-1 %, 256 x 6:
        // -21 ... +9 %). Book 3 (class 4, the light-list pdfs) keeps the unbounded 512: -8 % at 5.
        // Class 3 (media: final_scene, cornell_smoke) read from L2: RRT_B2_MEDIA_GLOBAL_WAVES.
        constexpr int kGW = (kBook2 == 3 && RRT_B2_MEDIA_GLOBAL_WAVES > 0) ? RRT_B2_MEDIA_GLOBAL_WAVES : kBook2Waves;
        // Classes 1-2 without noise textures need ~88 VGPRs and run at RRT_B2_NF_WAVES (6: bouncing
        // spheres +6.4 %, checkered spheres +4 %, quads +3.3 %, cornell_box +6.8 % same-box over 5;
        // the media class and the noise kernels lose 8-15 % at 6 and stay at 5).
        constexpr int kNF = kBook2 <= 2 ? RRT_B2_NF_WAVES : kBook2Waves;
        constexpr int kGNF = kBook2 <= 2 ? RRT_B2_NF_WAVES : kGW;
        if constexpr (kBook2 != 4 && kBook2Waves > 1)
            return p.scene_in_lds ? launch_variant<true, uint16_t, kWide, kBook2, kBook2Waves, kBook2Block, kNF>(p, count, stream)
                                  : launch_variant<false, uint16_t, kWide, kBook2, kGW, kBook2Block, kGNF>(p, count, stream);
        if constexpr (kBook2 == 4 && kBook3Waves > 1)
            return p.scene_in_lds ? launch_variant<true, uint16_t, kWide, kBook2, kBook3Waves, kBook2Block>(p, count, stream)
                                  : launch_variant<false, uint16_t, kWide, kBook2, kBook3Waves, kBook2Block>(p, count, stream);
        return p.scene_in_lds ? launch_variant<true, uint16_t, kWide, kBook2>(p, count, stream)
                              : launch_variant<false, uint16_t, kWide, kBook2>(p, count, stream);
    } else {
        // C2's class staged in LDS: RRT_B1U_WAVES > 6 runs RRT_B1U_BLOCK-thread blocks (fewer scene copies)
        if constexpr (kBook2 == kBook1Untextured && RRT_B1U_WAVES > 6)
            if (!kWide && p.scene_in_lds && p.min_waves >= 6)
                return launch_variant<true, uint16_t, kWide, kBook2, RRT_B1U_WAVES, RRT_B1U_BLOCK>(p, count, stream);
        // the diffuse-only class (C4) staged in LDS: RRT_B1D_WAVES > 6 runs 256-thread blocks
        if constexpr (kBook2 == kBook1Diffuse && RRT_B1D_WAVES > 6)
            if (!kWide && p.scene_in_lds && p.min_waves >= 6)
                return launch_variant<true, uint16_t, kWide, kBook2, RRT_B1D_WAVES, kGlobalBlock>(p, count, stream);
        if (!kWide && p.scene_in_lds && p.min_waves >= 6)
            return launch_variant<true, uint16_t, kWide, kBook2, kWavesPerSimd>(p, count, stream);
        // Scenes read from L2 (C5) hold only the stack in LDS: 256-thread blocks at 7 waves/SIMD
        // (72 VGPRs), which 512-thread blocks cannot reach (3.5 blocks); C5 +2.8 % same-box over
        // 512 x 6 (256 x 8, 64 VGPRs: -16 %, spills).
        if (!kWide && !p.scene_in_lds && p.global_waves >= 7)
            return launch_variant<false, uint16_t, kWide, kBook2, kGlobalWaves, kGlobalBlock>(p, count, stream);
        if (!kWide && !p.scene_in_lds && p.global_waves >= 6)
            return launch_variant<false, uint16_t, kWide, kBook2, kWavesPerSimd>(p, count, stream);
        return p.scene_in_lds ? launch_variant<true, uint16_t, kWide, kBook2>(p, count, stream)
                              : launch_variant<false, uint16_t, kWide, kBook2>(p, count, stream);
    }
}

}  // namespace

hipError_t launch_render_pass(const KParams &p, bool count, hipStream_t stream) {
    if (p.flags & kFlagF64) return launch_render_pass_f64(p, count, stream);  // the f64 books path
    // Variant choice: BVH width, smallest LDS stack that holds the traversal, and the scene
    // staged in LDS when the BVH + spheres fit the per-block budget (RTOW: ~20-26 KB).
    // Book-2 scenes (moving spheres, checker / noise textures): BVH2 only (the host builds a
    // binary tree for them); motion is always present (zero for static spheres).
    if (p.prim_motion) {  // book 2: the binary BVH only
        if (p.bvh_width != 2) return hipErrorInvalidValue;
        if (p.flags & 0x4u) return launch_width<false, 4>(p, count, stream);  // RRT_FLAG_BOOK3
        if (p.n_media) return launch_width<false, 3>(p, count, stream);
        return p.n_quads ? launch_width<false, 2>(p, count, stream) : launch_width<false, 1>(p, count, stream);
    }
    if (p.bvh_width == 4) return launch_width<true, 0>(p, count, stream);
    // Scenes without image textures run the kernel with the texture path compiled out: C2 +1.0 %;
    // for scenes read from L2 (C5) it removes the 7-wave kernel's 4 spilled VGPRs (20 B of scratch
    // per lane, written and read back through memory) at equal time.
    if (!p.specular && p.scene_in_lds) return launch_width<false, kBook1Diffuse>(p, count, stream);
    if (!p.image_tex) return launch_width<false, kBook1Untextured>(p, count, stream);
    return launch_width<false, 0>(p, count, stream);
}

// One launch (+ combine) per sample pass of at most p.pass_chunks chunks, in chunk order.
hipError_t launch_render_kernel(const KParams &p, bool count, hipStream_t stream) {
    if ((p.flags & kFlagF64) && p.seq) return launch_render_f64_seq(p, count, stream);
    if (p.n_chunks <= 1 || p.pass_chunks == 0 || p.pass_chunks >= p.n_chunks) {
        KParams q = p;
        q.chunk_begin = 0;
        q.pass_n = p.n_chunks;
        q.pass_big = p.n_big;
        q.n_big_units = p.n_work_tiles * q.pass_big * 64u;
        q.n_units = p.n_work_tiles * q.pass_n * 64u;
        q.fd_pass_big = make_fastdiv(q.pass_big);
        q.fd_pass_tail = make_fastdiv(q.pass_n - q.pass_big);
        return launch_render_pass(q, count, stream);
    }
    for (uint32_t cb = 0; cb < p.n_chunks; cb += p.pass_chunks) {
        KParams q = p;
        q.chunk_begin = cb;
        q.pass_n = std::min(p.pass_chunks, p.n_chunks - cb);
        q.pass_big = cb < p.n_big ? std::min(p.n_big - cb, q.pass_n) : 0u;
        q.n_big_units = p.n_work_tiles * q.pass_big * 64u;
        q.n_units = p.n_work_tiles * q.pass_n * 64u;
        q.fd_pass_big = make_fastdiv(q.pass_big);
        q.fd_pass_tail = make_fastdiv(q.pass_n - q.pass_big);
        const hipError_t e = launch_render_pass(q, count, stream);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_render(const KParams &p, hipStream_t stream) { return launch_render_kernel(p, false, stream); }

hipError_t launch_quantize(const float *d_accum, uint8_t *d_rgb8, uint32_t n_pixels, float scale, hipStream_t stream) {
    if (n_pixels == 0) return hipSuccess;
    const uint32_t groups = (n_pixels + 3u) / 4u;
    hipLaunchKernelGGL(rrt_quantize, dim3((groups + 255u) / 256u), dim3(256), 0, stream,
                       reinterpret_cast<const float4 *>(d_accum), d_rgb8, n_pixels, scale);
    return hipGetLastError();
}
hipError_t launch_render_counting(const KParams &p, hipStream_t stream) { return launch_render_kernel(p, true, stream); }

namespace {
// Every f32 bit pattern: out[0] counts s with |s| in [2^-126, 2^126), +-0, +-inf or NaN whose
// recip_rn(s) is not the IEEE 1.0f / s (NaN results compare equal); out[1] counts s with |s| <
// 2^126 or NaN whose clamped_slope(s) is not clamp_inv(1.0f / s); out[2] counts s = +0 or s >=
// 2^-96 (+inf and positive NaN patterns included) whose sqrt_rn_big(s) is not the IEEE sqrt.
__global__ __launch_bounds__(256) void rrt_recip_check(unsigned long long *out) {
    uint32_t bad0 = 0, bad1 = 0, bad2 = 0;
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < (1ull << 32); k += (uint64_t)gridDim.x * 256ull) {
        const uint32_t u = (uint32_t)k, a = u & 0x7fffffffu;
        const float s = __uint_as_float(u);
        auto same = [](float x, float y) { return __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y); };
        const bool normal = a >= 0x00800000u && a < 0x7e800000u;
        const bool special = a == 0u || a >= 0x7f800000u;
        if ((normal || special) && !same(recip_rn(s), 1.0f / s)) ++bad0;
        if ((a < 0x7e800000u || a > 0x7f800000u) && !same(clamped_slope(s), clamp_inv(1.0f / s))) ++bad1;
        // +-0 and every |s| >= 2^-96 of either sign (negatives: NaN like the IEEE root; -0: -0), +-inf, NaN
        if ((a == 0u || a >= 0x0f800000u) && !same(sqrt_rn_big(s), __builtin_sqrtf(s))) ++bad2;
    }
    if (bad0) atomicAdd(&out[0], (unsigned long long)bad0);
    if (bad1) atomicAdd(&out[1], (unsigned long long)bad1);
    if (bad2) atomicAdd(&out[2], (unsigned long long)bad2);
}
}  // namespace

hipError_t launch_recip_check(unsigned long long *d_out, hipStream_t stream) {
    hipLaunchKernelGGL(rrt_recip_check, dim3(16384), dim3(256), 0, stream, d_out);
    return hipGetLastError();
}

}  // namespace rrt
