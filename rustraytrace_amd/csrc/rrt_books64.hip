// rrt_books64.hip — gfx950 kernel of the f64 books path (RRT_FLAG_F64).
//
// The reference's CPU books path computes in f64 (books/in_one_weekend/vec3.rs:5-8) and the
// north star checks the GPU against it ("per-channel <= 1e-4 before u8 quantisation; bit-exact PPM
// after"). The f32 megakernel (rrt_kernel.hip, the reference GPU slot's precision) is bit-exact
// against the oracle's f32 restatement but only statistically close to f64: a rounding that
// flips a discrete decision (a grazing hit, a rejection-loop acceptance, a Russian-roulette draw)
// sends a path another way. This kernel runs the books path's own arithmetic instead:
//   camera ray       camera.rs:152-180 (+ the time draw of the_next_week/camera.rs:160)
//   closest hit      sphere.rs:24-51 over (0.001, inf): oc, a, h, c, h*h - a*c, both roots,
//                    unfused and in the reference's operation order (Rust never contracts)
//   hit record       sphere.rs:47-48 p = o + t*d, (p - center) / r; hittable.rs:20-32 front face
//   scatter          material.rs:28-40 / 53-64 / 83-102, vec3.rs:181-189 (1e-160 < |p|^2 <= 1),
//                    vec3.rs:201-210 reflect / refract, Schlick with powi(5) = x * ((x*x)*(x*x))
//   Russian roulette camera.rs:189-200 (this bounce's attenuation, clamp [.05, .95])
//   sky / background camera.rs:206-208 / the_next_week/camera.rs:179-181
//   emission, image  the_next_week/material.rs:41-53, 116-135; sphere.rs:46-52 get_sphere_uv with
//   texture          one f64 acos / atan2 (fdlibm's algorithms, restated op for op by the oracle's
//                    BOOKS mode), texture.rs:89-109, rtw_image.rs:46-55
// in f64 (-ffp-contract=off; IEEE division and square root), on the same per-path random stream as
// the f32 kernel (rrt_device.h: every draw is a 24-bit value, exact in f32 and f64). Every path
// decision — which sphere a ray hits, the rejection loops, the Russian-roulette draw against this
// bounce's attenuation — depends only on ray geometry, the draws and the attenuation, so the f64
// paths follow the books path's exactly; only the throughput product's association differs (the
// reference multiplies back to front through its recursion, this kernel front to back), which moves
// a pixel's f64 sum by a few ulps. No exit_skip: in f64 a ray leaving a surface never re-hits it.
//
// Scope: book-1 scenes (the BASELINE configs C1, C2, C4, C5: Lambertian, metal, dielectric,
// image-textured Lambertian, diffuse light; sky or constant background). The host rejects book-2/3
// scene data with RRT_FLAG_F64. Same work queue, chunked accumulation order and BVH (f32 boxes,
// rounded outward and grown by the f32 slab bound, tested in f64: conservative) as the f32 kernel.
#include "rrt_internal.h"

#include <atomic>
#include <cstdlib>
#include <type_traits>

namespace rrt {
namespace {

#include "rrt_device.h"
#include "rrt_box32.h"
#include "rrt_sphere32.h"

// issue priority by loop phase (as rrt_kernel.hip: refill 2, node steps 1, leaf batches 2, shading 0)
constexpr int kPrioRefill = 2, kPrioNode = 1, kPrioLeaf = 2, kPrioShade = 0;

// Debug builds only (-DRRT_F64_STATS=1..4 in F64_FLAGS, never the shipped library): per-wave
// statistics written into counter slots 2..4 by the non-counting kernel.
//   1: s_memtime cycles in refill + ray start / the traversal loop (nodes + leaves) / shading
//   2: leaf batches (wave): sum of the batch's largest lane range (f64 sphere-test iterations the
//      wave runs) / sum of the largest lane count of tests with disc >= 0 / number of batches
//   3: lane f64 sphere tests / those with disc >= 0 / those that update the closest hit
//   4: node-step wave-iterations / sum of stepping lanes / leaf-batch wave-iterations x 64
//   5: spheres the f32 pre-test keeps / their f64 disc >= 0 / lane sphere tests (ranges)
#ifndef RRT_F64_STATS
#define RRT_F64_STATS 0
#endif
// Debug builds only: random_unit_vector takes its first candidate (prices the rejection loop)
#ifndef RRT_DEBUG_NOREJECT
#define RRT_DEBUG_NOREJECT 0
#endif
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
    return v;
}

struct D3 {
    double x, y, z;
};
__device__ __forceinline__ D3 d3(double x, double y, double z) { return D3{x, y, z}; }
__device__ __forceinline__ D3 add(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ D3 sub(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ D3 mul(D3 a, D3 b) { return d3(a.x * b.x, a.y * b.y, a.z * b.z); }
// vec3.rs:118-132: Vec3 * f64 and f64 * Vec3 both compute e[i] * s
__device__ __forceinline__ D3 muls(D3 a, double s) { return d3(a.x * s, a.y * s, a.z * s); }
// vec3.rs:156-158 dot = u0*v0 + u1*v1 + u2*v2 (left to right, unfused)
__device__ __forceinline__ double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// 1 / x, the IEEE quotient, in 6 instructions instead of the expansion's 11 for x in [2^-64, 2^64]:
// there the expansion's v_div_scale steps are identities (numerator 1, quotient in [2^-64, 2^64]) and
// its v_div_fixup passes the v_div_fmas result through, so what remains is its own reciprocal
// (v_rcp_f64 + two Newton steps) and final step fma(fma(-x, r, 1), r, r) — the same operations the
// f64 root divisions use (recip_a64 / div_a64, below). Outside the range: the IEEE division. Off by
// default: same-box within noise (C2 +-0.5 %, C4 -1 %, `profiles/r5_f64_ab_batch5.log`).
#ifndef RRT_F64_FASTRCP
#define RRT_F64_FASTRCP 0
#endif
__device__ __forceinline__ double recip64(double x) {
    if (!RRT_F64_FASTRCP || !(x >= 0x1.0p-64 && x <= 0x1.0p64)) return 1.0 / x;
    double r = __builtin_amdgcn_rcp(x);
    double e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-x, r, 1.0);
    r = __builtin_fma(r, e, r);
    return __builtin_fma(__builtin_fma(-x, r, 1.0), r, r);
}
// sqrt(x), the IEEE root: LLVM's AMDGPU f64 expansion (v_rsq_f64, a Goldschmidt step, two remainder
// corrections, a class check for +-0 and +inf) without its scaling of small arguments. The expansion
// multiplies x by 2^256 when x < 2^-767 and the root by 2^-128 after; for every other x both
// v_ldexp_f64 take exponent 0 and are identities, so this sequence is the same operations on the same
// values (rrt_testing_sqrt64_check compares the two bit for bit on 2^28 arguments). sqrt64 takes it
// when no active lane of the wave holds a nonzero x below 2^-767 (a wave-uniform branch, the f32
// kernel's sqrt_rn); saves two v_ldexp_f64, a compare and two selects per root. Taken in the leaf
// loop's root only (at the shading sites the second inlined sequence costs more registers than it
// saves). RRT_F64_SQRT=0: the library sequence everywhere.
#ifndef RRT_F64_SQRT
#define RRT_F64_SQRT 1
#endif
__device__ __forceinline__ double sqrt64_big(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(g, r, g);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return __builtin_amdgcn_class(x, 0x260) ? x : g;  // +-0, +inf: x itself
}
__device__ __forceinline__ bool sqrt64_small(double x) { return x < 0x1.0p-767 && x != 0.0; }
__device__ __forceinline__ double sqrt64(double x) {
    if (!RRT_F64_SQRT) return __builtin_sqrt(x);
    if (__ballot(sqrt64_small(x)) == 0) return sqrt64_big(x);
    return __builtin_sqrt(x);
}
// vec3.rs:168-170 unit_vector = v / |v|, Div<f64> = (1/rhs) * v (vec3.rs:142-148)
__device__ __forceinline__ D3 unit_vector(D3 v) { return muls(v, recip64(__builtin_sqrt(dot(v, v)))); }
__device__ __forceinline__ D3 f2d(float x, float y, float z) { return d3((double)x, (double)y, (double)z); }
// f64::min: a NaN operand yields the other
__device__ __forceinline__ double rmin(double a, double b) { return a < b ? a : b; }

// random_double(): the 24-bit draw, exact in f64; random_double_range(-1, 1) = u * 2 + -1 (exact;
// the rejection loops below draw it as draw_centred)
__device__ __forceinline__ double rnd64(RngState &s) { return (double)(rng_next(s) >> 8) * 0x1.0p-24; }

// The rejection loops decide on integers. A coordinate drawn by random_double_range(-1, 1) is
// x = a 2^-23 - 1 = (a - 2^23) 2^-23 for the draw's 24-bit a, exactly, in f64, so |p|^2 = S 2^-46
// with the integer S = sum (a_i - 2^23)^2 <= 3 2^46. The reference's f64 sum of the (exact)
// squares rounds by less than 2^-51 while S 2^-46 moves in steps of 2^-46, so its comparison with 1
// decides exactly as S against 2^46, and |p|^2 > 1e-160 exactly when S > 0
// (tests/test_rejection_exact.py). The loops compute S in 64-bit integers from 24-bit signed
// multiplies (full-rate VALU) instead of the reference's f64 conversions, products and sums
// (half-rate): same draws, same decisions, same accepted point, which is converted once.
__device__ __forceinline__ int32_t draw_centred(RngState &s) { return (int32_t)(rng_next(s) >> 8) - 8388608; }
__device__ __forceinline__ uint64_t sq_i24(int32_t a) { return (uint64_t)((int64_t)a * (int64_t)a); }
// The same decisions from f32 arithmetic where it is provably decisive (RRT_F64_REJ32): the f32
// sum of squares of the exact coordinates a, b, c (|a| <= 2^23: exact in f32) is within 3u S
// (u = 2^-24: one rounding per term) of the integer S, so it decides `S <= 2^46` (`S < 2^46` for the
// disk) outside the band 2^46 (1 +- 2^-21) and `S > 0` exactly (it is 0 only for a = b = c = 0).
// A wave with a lane in the band (~7e-7 of the candidates) decides those lanes on the integers.
// Off by default: same-box C2 -5 %, C4 -5 %, C5 -4 % (`profiles/r5_f64_ab_batch5.log`) — the
// band's ballot and branch in every iteration cost the scalar unit more than the integer
// multiplies they replace (round 4 measured the same of an f32 test with an f64 fallback).
#ifndef RRT_F64_REJ32
#define RRT_F64_REJ32 0
#endif
constexpr float kRej32Lo = 0x1.fffffp45f;   // 2^46 (1 - 2^-21)
constexpr float kRej32Hi = 0x1.000008p46f;  // 2^46 (1 + 2^-21)
// 1: 0 < S <= 2^46 (or S < 2^46 with kDisk), 0: not
template <bool kDisk>
__device__ __forceinline__ bool in_ball(int32_t a, int32_t b, int32_t c) {
    if (!RRT_F64_REJ32) {
        const uint64_t S = sq_i24(a) + sq_i24(b) + sq_i24(c);
        return kDisk ? S < (1ull << 46) : S - 1u < (1ull << 46);
    }
    const float af = (float)a, bf = (float)b, cf = (float)c;
    const float s32 = __builtin_fmaf(cf, cf, __builtin_fmaf(bf, bf, af * af));
    bool in = (kDisk || s32 > 0.0f) && s32 <= kRej32Lo;
    const bool band = s32 > kRej32Lo && s32 <= kRej32Hi;
    if (__ballot(band) != 0 && band) {
        const uint64_t S = sq_i24(a) + sq_i24(b) + sq_i24(c);
        in = kDisk ? S < (1ull << 46) : S - 1u < (1ull << 46);
    }
    return in;
}
__device__ __forceinline__ double centred_to_pm1(int32_t a) { return (double)a * 0x1.0p-23; }  // exact

// vec3.rs:181-189 random_unit_vector (Vec3::random_range(-1, 1): x, y, z drawn in order)
__device__ __forceinline__ D3 random_unit_vector(RngState &s) {
    int32_t a, b, c;
    for (;;) {
        a = draw_centred(s);
        b = draw_centred(s);
        c = draw_centred(s);
        if (RRT_DEBUG_NOREJECT || in_ball<false>(a, b, c)) break;  // 0 < S <= 2^46
    }
    const double x = centred_to_pm1(a), y = centred_to_pm1(b), z = centred_to_pm1(c);
    const double lensq = x * x + y * y + z * z;
    return muls(d3(x, y, z), recip64(__builtin_sqrt(lensq)));
}

// vec3.rs:201-203 reflect = v - (2 * dot(v, n)) * n
__device__ __forceinline__ D3 reflect(D3 v, D3 n) { return sub(v, muls(n, 2.0 * dot(v, n))); }
// vec3.rs:205-210 refract
__device__ __forceinline__ D3 refract(D3 uv, D3 n, double e) {
    const double c = rmin(-dot(uv, n), 1.0);
    const D3 perp = muls(add(uv, muls(n, c)), e);
    const D3 par = muls(n, -__builtin_sqrt(__builtin_fabs(1.0 - dot(perp, perp))));
    return add(perp, par);
}
// material.rs:75-80 Schlick at r0 = ((1 - ri) / (1 + ri))^2; powi(5) = x * ((x*x) * (x*x)) (LLVM's
// repeated squaring)
__device__ __forceinline__ double reflectance_r0(double cosine, double r0) {
    const double x = 1.0 - cosine;
    const double x2 = x * x;
    return r0 + (1.0 - r0) * (x * (x2 * x2));
}

// ---- f64 acos / atan2 for get_sphere_uv (the_next_week/sphere.rs:46-52) ----------------------
// The reference calls Rust's f64::acos / atan2 (the platform libm). Both sides here restate one
// algorithm — fdlibm's e_acos.c / s_atan.c / e_atan2.c (Sun Microsystems, freely distributable):
// only + - * / sqrt and exponent-word tests, so the oracle's BOOKS mode reproduces every bit; within
// 1 ulp of glibc's libm (tests/test_oracle.py checks 2e5 arguments).
__device__ __forceinline__ uint32_t hi_word(double x) { return (uint32_t)((uint64_t)__double_as_longlong(x) >> 32); }
__device__ __forceinline__ double clear_lo_word(double x) {
    return __longlong_as_double((long long)((uint64_t)__double_as_longlong(x) & 0xffffffff00000000ull));
}
constexpr double kPio2Hi = 1.57079632679489655800e+00, kPio2Lo = 6.12323399573676603587e-17;
constexpr double kPiD = 3.14159265358979311600e+00, kPiLo = 1.2246467991473531772e-16;
__device__ __forceinline__ double acos_rat(double z) {  // R(z) = p(z) / q(z) of e_acos.c
    const double p = z * (1.66666666666666657415e-01 +
                          z * (-3.25565818622400915405e-01 +
                               z * (2.01212532134862925881e-01 +
                                    z * (-4.00555345006794114027e-02 +
                                         z * (7.91534994289814532176e-04 + z * 3.47933107596021167570e-05)))));
    const double q = 1.0 + z * (-2.40339491173441421878e+00 +
                                z * (2.02094576023350569471e+00 +
                                     z * (-6.88283971605453293030e-01 + z * 7.70381505559019352791e-02)));
    return p / q;
}
__device__ double rrt_acos64(double x) {
    const uint32_t hx = hi_word(x), ix = hx & 0x7fffffffu;
    if (ix >= 0x3ff00000u) {  // |x| >= 1
        const uint32_t lx = (uint32_t)__double_as_longlong(x);
        if (((ix - 0x3ff00000u) | lx) == 0) return (hx >> 31) ? kPiD + 2.0 * kPio2Lo : 0.0;
        return (x - x) / (x - x);  // NaN
    }
    if (ix < 0x3fe00000u) {  // |x| < 0.5
        if (ix <= 0x3c600000u) return kPio2Hi + kPio2Lo;
        const double r = acos_rat(x * x);
        return kPio2Hi - (x - (kPio2Lo - x * r));
    }
    if (hx >> 31) {  // x < -0.5
        const double z = (1.0 + x) * 0.5;
        const double s = __builtin_sqrt(z);
        const double w = acos_rat(z) * s - kPio2Lo;
        return kPiD - 2.0 * (s + w);
    }
    const double z = (1.0 - x) * 0.5;  // x > 0.5
    const double s = __builtin_sqrt(z);
    const double df = clear_lo_word(s);
    const double c = (z - df * df) / (s + df);
    const double w = acos_rat(z) * s + c;
    return 2.0 * (df + w);
}
__device__ double rrt_atan64(double x) {
    constexpr double hi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                              1.57079632679489655800e+00};
    constexpr double lo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                              6.12323399573676603587e-17};
    const uint32_t hx = hi_word(x), ix = hx & 0x7fffffffu;
    int id;
    if (ix >= 0x44100000u) {  // |x| >= 2^66
        if (ix > 0x7ff00000u || (ix == 0x7ff00000u && (uint32_t)__double_as_longlong(x) != 0)) return x + x;
        return (hx >> 31) ? -hi[3] - lo[3] : hi[3] + lo[3];
    }
    if (ix < 0x3fdc0000u) {  // |x| < 0.4375
        if (ix < 0x3e200000u) return x;
        id = -1;
    } else {
        x = __builtin_fabs(x);
        if (ix < 0x3ff30000u) {      // |x| < 1.1875
            if (ix < 0x3fe60000u) {  // 7/16 <= |x| < 11/16
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else {
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else if (ix < 0x40038000u) {  // |x| < 2.4375
            id = 2;
            x = (x - 1.5) / (1.0 + 1.5 * x);
        } else {
            id = 3;
            x = -1.0 / x;
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (3.33333333333329318027e-01 +
                           w * (1.42857142725034663711e-01 +
                                w * (9.09088713343650656196e-02 +
                                     w * (6.66107313738753120669e-02 +
                                          w * (4.97687799461593236017e-02 + w * 1.62858201153657823623e-02)))));
    const double s2 = w * (-1.99999999998764832476e-01 +
                           w * (-1.11111104054623557880e-01 +
                                w * (-7.69187620504482999495e-02 +
                                     w * (-5.83357013379057348645e-02 + w * -3.65315727442169155270e-02))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = hi[id] - ((x * (s1 + s2) - lo[id]) - x);
    return (hx >> 31) ? -r : r;
}
__device__ double rrt_atan2_64(double y, double x) {
    const uint64_t bx = (uint64_t)__double_as_longlong(x), by = (uint64_t)__double_as_longlong(y);
    const uint32_t hx = (uint32_t)(bx >> 32), lx = (uint32_t)bx, hy = (uint32_t)(by >> 32), ly = (uint32_t)by;
    const uint32_t ix = hx & 0x7fffffffu, iy = hy & 0x7fffffffu;
    if ((ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || (iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;  // NaN
    if (((hx - 0x3ff00000u) | lx) == 0) return rrt_atan64(y);  // x = 1
    const uint32_t m = ((hy >> 31) & 1u) | ((hx >> 30) & 2u);  // 2 * sign(x) + sign(y)
    if ((iy | ly) == 0) {  // y = +-0
        if (m < 2) return y;
        return m == 2 ? kPiD : -kPiD;
    }
    if ((ix | lx) == 0) return (hy >> 31) ? -kPio2Hi : kPio2Hi;  // x = +-0
    if (ix == 0x7ff00000u) {  // x = +-inf
        if (iy == 0x7ff00000u) {
            const double v[4] = {0.25 * kPiD, -0.25 * kPiD, 0.75 * kPiD, -0.75 * kPiD};
            return v[m];
        }
        const double v[4] = {0.0, -0.0, kPiD, -kPiD};
        return v[m];
    }
    if (iy == 0x7ff00000u) return (hy >> 31) ? -kPio2Hi : kPio2Hi;  // y = +-inf
    const int k = ((int)iy - (int)ix) >> 20;
    double z;
    if (k > 60) z = kPio2Hi + 0.5 * kPiLo;
    else if ((hx >> 31) && k < -60) z = 0.0;
    else z = rrt_atan64(__builtin_fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return kPiD - (z - kPiLo);
        default: return (z - kPiLo) - kPiD;
    }
}

// x / c for the constant divisors 2 pi and pi (rrt_kernel.hip div_by_const in f64): q = x RN(1/c)
// and Markstein's fma correction, the IEEE quotient away from underflow (8e8 random f64 arguments
// in [2^-60, 8) against the CPU's division, tests/test_div_const.py); phi and theta are 0 or
// far above it. RRT_DIV_CONST=0: the IEEE division.
#ifndef RRT_DIV_CONST
#define RRT_DIV_CONST 1
#endif
__device__ __forceinline__ double div_by_const64(double x, double c) {
    if (!RRT_DIV_CONST) return x / c;
    const double rc = 1.0 / c;  // folded: RN(1/c)
    const double q = x * rc;
    return __builtin_fma(__builtin_fma(-q, c, x), rc, q);
}

// ImageTexture::value (texture.rs:89-109) at get_sphere_uv(outward) (the_next_week/sphere.rs:46-52):
// theta = acos(-y), phi = atan2(-z, x) + pi, u = phi / (2 pi), v = theta / pi. The texel's bytes
// r | g << 8 | b << 16 (value = (1/255) byte, rtw_image.rs:46-55), or 0x1000000 for a texture with no
// data (the solid cyan (0, 1, 1) of texture.rs:91-93).
#ifndef RRT_DEBUG_F64_TEXEL_FIXED  // debug builds only: no acos / atan2 (prices them; wrong images)
#define RRT_DEBUG_F64_TEXEL_FIXED 0
#endif
__device__ __forceinline__ int as_i32_rs(double x) {  // Rust `as i32`: saturating, NaN -> 0
    if (!(x == x)) return 0;
    if (x <= -2147483648.0) return (int)0x80000000;
    if (x >= 2147483647.0) return 0x7fffffff;
    return (int)x;
}
// The texel column of phi and the row of theta (Interval::clamp, 1 - v, the image scale, `as i32`,
// rtw_image.rs:51-52, 70-78's clamp). Every step is monotone — a correctly rounded division or
// product by a positive constant, a clamp, 1 - v, a truncation — so the column is non-decreasing in
// phi and the row non-increasing in theta.
__device__ __forceinline__ int texel_col64(double phi, int w) {
    double u = div_by_const64(phi, 2.0 * kPiD);
    u = u < 0.0 ? 0.0 : (u > 1.0 ? 1.0 : u);
    const int i = as_i32_rs(u * (double)w);
    return i < 0 ? 0 : (i < w ? i : w - 1);
}
__device__ __forceinline__ int texel_row64(double theta, int h) {
    double v = div_by_const64(theta, kPiD);
    v = 1.0 - (v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v));
    const int j = as_i32_rs(v * (double)h);
    return j < 0 ? 0 : (j < h ? j : h - 1);
}

// The texel decided from f32 angles where that is provably the books path's texel: an enclosure
// c +- e of rrt_acos64(-y) (of rrt_atan2_64(-z, x) + pi) from the device's f32 acosf (atanf) with
// bounded error, and the texel coordinate s = u w (v' h) of the f64 pipeline at c. The f64 angle's s
// lies within e w / (2 pi) (e h / pi) of it, plus the pipeline's own roundings (< 2^-30 here), so
// when no integer and no image edge lies that close to s, the f64 angle truncates to the same index
// (and no clamp applies). Else, and for arguments outside the enclosures' domains, the f64 fdlibm
// angle itself (a few lookups in ten thousand on C4). The error bounds are at least twice the largest
// error of acosf over every f32 in [-1, 1] and of atanf over every f32 in [0, 1] against the device's
// f64 acos / atan (rrt_testing_trig32_check, tests/test_gpu_trig32.py); kLibm64Err covers fdlibm's
// f64 error (< 1 ulp, < 2^-51 for these angles) many times over. RRT_F64_TEXEL_FAST=0: the fdlibm
// angles always. Without image data no angle is needed (texture.rs:91-93).
#ifndef RRT_F64_TEXEL_FAST
#define RRT_F64_TEXEL_FAST 1
#endif
constexpr double kAcos32Err = 0x1.0p-20;
constexpr double kAtan32Err = 0x1.0p-21;
constexpr double kLibm64Err = 0x1.0p-40;
__device__ __forceinline__ float next_up32(float x) {
    const uint32_t b = __float_as_uint(x);
    if ((b & 0x7fffffffu) == 0u) return __uint_as_float(1u);  // +-0 -> the smallest subnormal
    return __uint_as_float((b >> 31) ? b - 1u : b + 1u);
}
__device__ __forceinline__ float next_down32(float x) { return -next_up32(-x); }
// acos(y) for y in [yd, yu] (the f32 neighbours around fl32(y)) lies in [acos(yu), acos(yd)] (acos is
// decreasing); the f32 ends' sum and difference are exact in f64
__device__ __forceinline__ bool acos_enclosure64(double y, double &c, double &e) {
    const float y32 = (float)y;
    const float yd = next_down32(y32), yu = next_up32(y32);
    if (!(yd >= -1.0f && yu <= 1.0f)) return false;  // |y| at or beyond 1 in f32, or NaN
    const double lo = (double)acosf(yu), hi = (double)acosf(yd);
    c = 0.5 * (lo + hi);
    e = 0.5 * (hi - lo) + (kAcos32Err + kLibm64Err + 0x1.0p-49);
    return true;
}
// atan2(yy, xx) + pi from atanf of the f32 ratio t = min / max of |yy|, |xx| (<= 1): the inputs' and
// the quotient's roundings move t by at most 3 2^-24 t <= 2^-22 and atan is 1-Lipschitz; the octant
// arithmetic, pi's rounding and the + pi in f64 add < 2^-48 (the f64 path's own + pi included).
// Zero, tiny, huge or NaN components take fdlibm.
__device__ __forceinline__ bool phi_enclosure64(double yy, double xx, double &c, double &e) {
    const double ay = __builtin_fabs(yy), ax = __builtin_fabs(xx);
    const double mn = ay < ax ? ay : ax, mx = ay < ax ? ax : ay;
    if (!(mn >= 0x1.0p-60 && mx <= 0x1.0p60)) return false;
    const float t = (float)mn / (float)mx;
    const double base = (double)atanf(t);
    double a = ay > ax ? 0.5 * kPiD - base : base;  // the angle in [0, pi/2]
    if (xx < 0.0) a = kPiD - a;
    if (yy < 0.0) a = -a;
    c = a + kPiD;
    e = kAtan32Err + 0x1.0p-22 + kLibm64Err + 0x1.0p-48;
    return true;
}
// The column / row at the centre when the whole enclosure truncates to it: s_c = fl(fl(c / k) n) for
// the image size n <= 2^20 and k = 2 pi (pi with the flip 1 - v); 1 / (2 pi) < 0.16, 1 / pi < 0.32.
__device__ __forceinline__ bool texel_col_decided(double c, double e, int w, int &i) {
    if (w > (1 << 20)) return false;
    const double s = div_by_const64(c, 2.0 * kPiD) * (double)w;
    const double hw = e * (double)w * 0.16 + 0x1.0p-30;
    const double lo = s - hw, hi = s + hw;
    if (!(lo > 0.0 && hi < (double)w)) return false;  // an image edge within reach (or NaN)
    const double f = __builtin_floor(lo);
    if (!(hi < f + 1.0)) return false;  // a column edge within reach
    i = (int)f;
    return true;
}
__device__ __forceinline__ bool texel_row_decided(double c, double e, int h, int &j) {
    if (h > (1 << 20)) return false;
    const double s = (1.0 - div_by_const64(c, kPiD)) * (double)h;
    const double hw = e * (double)h * 0.32 + 0x1.0p-30;
    const double lo = s - hw, hi = s + hw;
    if (!(lo > 0.0 && hi < (double)h)) return false;
    const double f = __builtin_floor(lo);
    if (!(hi < f + 1.0)) return false;
    j = (int)f;
    return true;
}
__device__ __forceinline__ uint32_t texel_bytes64(const KParams &P, int tex, D3 outward) {
    const GTexture t = P.texs[tex];
    if (t.height <= 0) return 0x1000000u;  // texture.rs:91-93: (0, 1, 1)
    int i = 0, j = 0;
    if (RRT_DEBUG_F64_TEXEL_FIXED) {
        i = texel_col64(2.0 + outward.x * 0x1.0p-60, t.width);
        j = texel_row64(1.0 + outward.y * 0x1.0p-60, t.height);
    } else {
        double c = 0.0, e = 0.0;
        if (!(RRT_F64_TEXEL_FAST && phi_enclosure64(-outward.z, outward.x, c, e) && texel_col_decided(c, e, t.width, i)))
            i = texel_col64(rrt_atan2_64(-outward.z, outward.x) + kPiD, t.width);
        if (!(RRT_F64_TEXEL_FAST && acos_enclosure64(-outward.y, c, e) && texel_row_decided(c, e, t.height, j)))
            j = texel_row64(rrt_acos64(-outward.y), t.height);
    }
    const uint8_t *px = P.tex_pool + t.offset + ((size_t)j * t.width + i) * 3;
    return (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
}
__device__ __forceinline__ double texel_channel64(uint32_t byte) {
    const double cs = 1.0 / 255.0;
    return cs * (double)byte;
}
__device__ __forceinline__ D3 texel_value64(uint32_t bytes) {
    if (bytes == 0x1000000u) return d3(0.0, 1.0, 1.0);
    return d3(texel_channel64(bytes & 0xffu), texel_channel64((bytes >> 8) & 0xffu), texel_channel64(bytes >> 16));
}

// ---- the throughput product back to front (camera.rs:182-209's recursion) -----------------------
// BOOKS returns attenuation * ray_color(scattered) [/ p] up its recursion, so a path's radiance is
// L_k = (att_k (.) L_{k+1}) [* (1/p_k) for k >= 5] from the end of the path back to the camera ray:
// each scatter's attenuation is kept in the lane's history (global memory, [bounce][lane slot], 12 B:
// an attenuation is an f32 albedo, (1, 1, 1), or a texel's bytes — each byte b stored as the f32 bit
// pattern kTexelTag + b, a signalling NaN no albedo can hold: the host canonicalises NaN albedos to
// the quiet NaN, rrt_host.cpp canonical_albedo) and the product is formed back to front when a path ends with radiance (sky, background or
// a light). The same roundings as the recursion, in the same order: the kernel's per-sample radiance
// equals BOOKS' bit for bit. RRT_F64_B2F=0: the throughput carried front to back (a few ulps off).
#ifndef RRT_F64_B2F
#define RRT_F64_B2F 1
#endif
// the record's words are f32 bit patterns, kept as integers so that no move can quieten a tag
struct Att32 {
    uint32_t x, y, z;
};
// texel byte b <-> the signalling-NaN bit pattern kTexelTag + b (payloads 1..256). Any albedo,
// negative or -0 included, decodes as itself (round 5 tagged texels by the sign bit, which read a
// negative albedo back as a texel byte).
constexpr uint32_t kTexelTag = 0x7F800001u;
__device__ __forceinline__ double att_decode(uint32_t f) {
    return f - kTexelTag < 256u ? texel_channel64(f - kTexelTag) : (double)__uint_as_float(f);
}
// RRT_F64_REC4 = 1: a 4-B record instead — the primitive index (its material's albedo), kRecOne for a
// dielectric's (1, 1, 1), or kRecTexel | the texel's bytes (kRecTexel | 0x1000000: the no-data
// texture's (0, 1, 1)); the fold reads the albedo back from the material record.
#ifndef RRT_F64_REC4
#define RRT_F64_REC4 0
#endif
[[maybe_unused]] constexpr uint32_t kRecOne = 0xFFFFFFFEu, kRecTexel = 0x80000000u;
#if RRT_F64_REC4
using HRec = uint32_t;
#else
using HRec = Att32;
#endif
__device__ __forceinline__ HRec rec_albedo(int prim, const GMaterial &m) {
#if RRT_F64_REC4
    (void)m;
    return (uint32_t)prim;
#else
    (void)prim;
    return Att32{__float_as_uint(m.a.x), __float_as_uint(m.a.y), __float_as_uint(m.a.z)};
#endif
}
__device__ __forceinline__ HRec rec_one() {
#if RRT_F64_REC4
    return kRecOne;
#else
    return Att32{0x3F800000u, 0x3F800000u, 0x3F800000u};
#endif
}
__device__ __forceinline__ HRec rec_texel(uint32_t b) {
#if RRT_F64_REC4
    return kRecTexel | b;
#else
    if (b == 0x1000000u) return Att32{0u, 0x3F800000u, 0x3F800000u};
    return Att32{kTexelTag + (b & 0xffu), kTexelTag + ((b >> 8) & 0xffu), kTexelTag + (b >> 16)};
#endif
}
// the attenuation a record stands for (kTex: the class has image textures)
template <bool kTex>
__device__ __forceinline__ D3 rec_att(const HRec &r, const GMaterial *__restrict__ mtl) {
#if RRT_F64_REC4
    if (r == kRecOne) return d3(1.0, 1.0, 1.0);
    if (kTex && (r & kRecTexel)) return texel_value64(r & 0x1ffffffu);
    const float4 a = mtl[r].a;
    return f2d(a.x, a.y, a.z);
#else
    (void)mtl;
    return kTex ? d3(att_decode(r.x), att_decode(r.y), att_decode(r.z))
                : f2d(__uint_as_float(r.x), __uint_as_float(r.y), __uint_as_float(r.z));
#endif
}
// camera.rs:191-195: max of the attenuation's components, clamped to [0.05, 0.95]
__device__ __forceinline__ double rr_probability64(D3 att) {
    double pr = att.x;
    if (att.y > pr) pr = att.y;
    if (att.z > pr) pr = att.z;
    if (pr < 0.05) pr = 0.05;
    if (pr > 0.95) pr = 0.95;
    return pr;
}
// The first RRT_F64_LDS_HIST records of a lane's history live in an LDS ring beside the traversal
// stack ([bounce][thread], 12 B), the rest in global memory ([bounce][lane slot]): most paths are
// short (C2: 2.6 rays per path), so their records never leave the CU.
#ifndef RRT_F64_LDS_HIST
#define RRT_F64_LDS_HIST 0
#endif
struct Hist64 {
    HRec *ring;      // LDS: RRT_F64_LDS_HIST x block threads
    HRec *global;    // P.hist
    uint32_t lanes;  // P.hist_lanes
    uint32_t slot;   // the lane's global slot
    uint32_t tid;    // threadIdx.x
    uint32_t blk;    // block threads
    __device__ __forceinline__ void store(uint32_t k, const HRec &r) const {
        if (RRT_F64_LDS_HIST > 0 && k < (uint32_t)RRT_F64_LDS_HIST) ring[k * blk + tid] = r;
        else global[(size_t)k * lanes + slot] = r;
    }
    __device__ __forceinline__ HRec load(uint32_t k) const {
        if (RRT_F64_LDS_HIST > 0 && k < (uint32_t)RRT_F64_LDS_HIST) return ring[k * blk + tid];
        return global[(size_t)k * lanes + slot];
    }
};

// Debug builds only (RRT_F64_B2F_MODE): 1 = the records stored but the radiance carried front to
// back (prices the stores), 2 = the fold without its loads (prices the loads); wrong images.
#ifndef RRT_F64_B2F_MODE
#define RRT_F64_B2F_MODE 0
#endif
// Back to front in groups of RRT_F64_FOLD_GROUP records: a group's loads issue together, then its
// products in order.
#ifndef RRT_F64_FOLD_GROUP
#define RRT_F64_FOLD_GROUP 4
#endif
template <bool kTex>
__device__ __forceinline__ D3 fold_back64(const Hist64 &hist, const GMaterial *__restrict__ mtl, uint32_t n, D3 L) {
    constexpr uint32_t G = RRT_F64_FOLD_GROUP;
    uint32_t k = n;
    while (k > 0u) {
        const uint32_t m = k < G ? k : G;
        HRec a[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j)
            if (j < m) a[j] = RRT_F64_B2F_MODE == 2 ? rec_one() : hist.load(k - 1u - j);
        D3 at[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j)
            if (j < m) at[j] = rec_att<kTex>(a[j], mtl);
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) {
            if (j < m) {
                const D3 att = at[j];
                L = mul(att, L);
                if (k - 1u - j >= 5u) L = muls(L, recip64(rr_probability64(att)));  // Div<f64>: (1/p) * v (vec3.rs:142-148)
            }
        }
        k -= m;
    }
    return L;
}

// Per-ray constants of the box test (rrt_box32.h: f32 arithmetic on the f32 / f16 planes, widened
// so that it never rejects a box the f64 ray meets).
struct RayK64 {
    RayBox32 b;
    // byte offsets of the ray's (entry, exit) plane pairs of each axis in an LDS Node112
    uint32_t ox, oy, oz;
    // the 32-B f16 node (GNodeH, global memory) holds lo | hi << 16 per axis: rotating the word by
    // 16 bits when 1/d_a < 0 puts the (entry, exit) pair in (lo, hi) order
    uint32_t rx, ry, rz;
};
__device__ __forceinline__ RayK64 ray_consts64(D3 o, D3 d) {
    RayK64 r;
    r.b = box32_ray(o.x, o.y, o.z, d.x, d.y, d.z);
    // the ray's (entry, exit) offsets in a Node112 axis: both children's (lo, hi) at 32a, (hi, lo)
    // at 32a + 16
    r.ox = r.b.ix < 0.0f ? 16u : 0u;
    r.oy = r.b.iy < 0.0f ? 48u : 32u;
    r.oz = r.b.iz < 0.0f ? 80u : 64u;
    r.rx = r.b.ix < 0.0f ? 16u : 0u;
    r.ry = r.b.iy < 0.0f ? 16u : 0u;
    r.rz = r.b.iz < 0.0f ? 16u : 0u;
    return r;
}

struct Trav64 {
    double closest;   // the best hit's root, or (lazy roots) an upper bound of it
    double lo;        // lazy roots: a lower bound of the best hit's root (== closest when exact)
    float closest32;  // fl32(closest): the box test's exit bound (rrt_box32.h)
    int hit_prim;
    int node;
    int sp;
};

// One BVH2 node visit (rrt_kernel.hip trav_node's schedule): both child boxes against the closest
// hit so far, hit leaf children postponed as one primitive range, the nearer internal child next
// and the farther one pushed. The visiting order only prunes: the closest hit is the smallest
// accepted root whatever the order (exact ties aside), as with BvhNode::hit's left-first walk.
template <bool kCount, typename Node, typename Stack>
__device__ __forceinline__ bool trav_node64(const Node *__restrict__ nodes, Stack &stack, const RayK64 &rk,
                                            Trav64 &t, Leaves &lv, Counters &cnt) {
    if (kCount) { cnt.nodes++; cnt.boxes += 2; }
    bool h0, h1;
    uint32_t l0, l1;
    float tn0 = 0.0f, tn1 = 0.0f;
    if constexpr (std::is_same<Node, GNode>::value) {  // LDS: the Node112 layout (render64_body)
        const char *bx = reinterpret_cast<const char *>(nodes) + __umul24((uint32_t)t.node, 112u);
        auto quad = [&](uint32_t byte_off) { return *reinterpret_cast<const float4 *>(bx + byte_off); };
        const float4 x = quad(rk.ox), y = quad(rk.oy), z = quad(rk.oz);
        h0 = box32_hit(x.x, x.y, y.x, y.y, z.x, z.y, rk.b, t.closest32, tn0);
        h1 = box32_hit(x.z, x.w, y.z, y.w, z.z, z.w, rk.b, t.closest32, tn1);
        const uint2 lk = *reinterpret_cast<const uint2 *>(bx + 96);
        l0 = lk.x;
        l1 = lk.y;
    } else {  // global memory: the 32-B f16 node (GNodeH), each axis's halves in (entry, exit) order
        const uint4 *q = reinterpret_cast<const uint4 *>(nodes + t.node);
        const uint4 a = q[0], b = q[1];
        auto ord = [](uint32_t w, uint32_t r) { return __builtin_amdgcn_alignbit(w, w, r); };
        const uint32_t x0 = ord(a.x, rk.rx), y0 = ord(a.y, rk.ry), z0 = ord(a.z, rk.rz);
        const uint32_t x1 = ord(a.w, rk.rx), y1 = ord(b.x, rk.ry), z1 = ord(b.y, rk.rz);
        h0 = box32_hit(lo16(x0), hi16(x0), lo16(y0), hi16(y0), lo16(z0), hi16(z0), rk.b, t.closest32, tn0);
        h1 = box32_hit(lo16(x1), hi16(x1), lo16(y1), hi16(y1), lo16(z1), hi16(z1), rk.b, t.closest32, tn1);
        l0 = b.z;
        l1 = b.w;
    }
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

// Sphere::hit (sphere.rs:24-51) over the leaf range: oc = center - o, a = |d|^2, h = d.oc,
// c = |oc|^2 - r*r, disc = h*h - a*c, roots (h -+ sqrt(disc)) / a in the open (0.001, closest).
// (h + sq) / a >= (h - sq) / a, so the far root is tried only when the near one is <= 0.001 (or
// NaN), exactly the roots the reference's surrounds() tests accept.
#ifndef RRT_F64_DIVA
#define RRT_F64_DIVA 1
#endif
// Per-ray reciprocal of a = |d|^2 for the root divisions: the reciprocal steps of the compiler's
// IEEE f64 division expansion (v_rcp_f64 + two Newton steps) once per ray instead of per division.
// For a in [2^-64, 2^64] v_div_scale is an identity on a, and on any numerator whose quotient is
// not far below 0.001 (the acceptance bound), so quotient = fma(n - a q, r, q) with q = n r is the
// expansion's own v_div_fmas result; 0 marks a ray outside that range (plain division).
__device__ __forceinline__ double recip_a64(double a) {
    if (!(a >= 0x1.0p-64 && a <= 0x1.0p64)) return 0.0;
    double r = __builtin_amdgcn_rcp(a);
    double e = __builtin_fma(-a, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-a, r, 1.0);
    return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double div_a64(double n, double a, double ra) {
    if (!RRT_F64_DIVA || ra == 0.0) return n / a;
    const double q = n * ra;
    return __builtin_fma(__builtin_fma(-a, q, n), ra, q);
}

// A sphere record widened to f64 while the block stages the scene in LDS (kF64LdsWide): center and
// r * r formed once instead of four f32 -> f64 conversions and a product per sphere test. The f32
// radius squared is exact in f64 (48 significant bits), so r2 is the reference's r * r, and
// sqrt(r2) its r again (a correctly rounded root of an exact square).
#ifndef RRT_F64_R2
#define RRT_F64_R2 1
#endif
struct alignas(16) Sphere64 {
    double cx, cy, cz, r2;  // r2 = r * r (RRT_F64_R2) or r
};
__device__ __forceinline__ D3 center_of(const float4 &c) { return f2d(c.x, c.y, c.z); }
__device__ __forceinline__ D3 center_of(const Sphere64 &c) { return d3(c.cx, c.cy, c.cz); }
__device__ __forceinline__ double radius_of(const float4 &c) { return (double)c.w; }
__device__ __forceinline__ double radius_of(const Sphere64 &c) { return RRT_F64_R2 ? __builtin_sqrt(c.r2) : c.r2; }
__device__ __forceinline__ double radius_sq_of(const float4 &c) { return (double)c.w * (double)c.w; }
__device__ __forceinline__ double radius_sq_of(const Sphere64 &c) { return RRT_F64_R2 ? c.r2 : c.r2 * c.r2; }

// The f32 pre-test (rrt_sphere32.h) over the lane's range first: it marks the spheres whose f64
// discriminant may be >= 0, and the f64 test runs over the marked ones only, in index order (the
// unmarked ones would `continue` in it). The wave runs the f64 body max-over-lanes of the marked
// counts instead of the range lengths (C2: 1.17 against 2.21 iterations per leaf batch, measured by
// RRT_F64_STATS=2). Off by default (RRT_F64_SPHERE32=1 builds it): same-box it did not pay — C2
// -0..-3.5 %, C5 -2.4 % — the f64 sphere tests are not where the f64 kernel's time goes (C2: 54 % of
// the tests reach disc >= 0 and the traversal loop, node steps included, is half the wave cycles).
#ifndef RRT_F64_SPHERE32
#define RRT_F64_SPHERE32 0
#endif
#ifndef RRT_F64_S32_HOLD
#define RRT_F64_S32_HOLD 0
#endif
// ---- lazy exact roots (rrt_kernel.hip's RRT_LAZY_ROOT, for the f64 roots) ----------------------------
// Each root is bracketed from the f32 square root of fl32(disc) and the per-ray reciprocal: the best
// candidate is kept as an interval [lo, closest], a candidate wholly below lo replaces it, one wholly at
// or above closest is rejected (both the exact loop's decisions: strictly less, the first of equal
// roots wins), and an overlap — or a root near tmin, a ray inside the sphere, disc outside
// [2^-96, 2^126], a NaN — is decided on the exact roots. The winner's exact root is formed once, when
// the query ends (lazy_finish64). The box tests prune with the upper bound, a superset of the exact
// walk in the same order. So every decision and every t equal the exact loop's (tests/test_gpu_books64.py
// green with it on). Measured and left off (round 6, same-box, profiles/r6_f64_sqrt_lazy_ab.log): C2
// -8 %, C5 -5.5 %, C4 -10 % — the winner's exact root at each query's end, the held interval (a
// double more: 4 VGPRs spilled at the 128-VGPR bound) and the bookkeeping cost more than the sparse
// exact roots did. RRT_F64_LAZY=1 turns it on.
#ifndef RRT_F64_LAZY
#define RRT_F64_LAZY 0
#endif
// The exact root leaves64 forms for primitive i: the near root if above tmin, else the far.
template <typename Rec>
__device__ __forceinline__ double exact_root64(const Rec *__restrict__ prims, int i, D3 o, D3 d, double a, double ra) {
    const Rec cr = prims[i];
    const D3 oc = sub(center_of(cr), o);
    const double h = dot(d, oc);
    const double c = dot(oc, oc) - radius_sq_of(cr);
    const double disc = h * h - a * c;
    const double sq = sqrt64(disc);
    double root = div_a64(h - sq, a, ra);
    if (!(0.001 < root)) root = div_a64(h + sq, a, ra);
    return root;
}
template <typename Rec>
__device__ __forceinline__ void lazy_resolve64(const Rec *__restrict__ prims, int i, D3 o, D3 d, double a, double ra,
                                               Trav64 &t) {
    const double rc = exact_root64(prims, i, o, d, a, ra);
    if (0.001 < rc && rc < t.closest) {  // else rc >= closest >= the best's root: rejected
        const double rb = (t.hit_prim >= 0 && t.lo != t.closest) ? exact_root64(prims, t.hit_prim, o, d, a, ra) : t.closest;
        if (rc < rb) t.hit_prim = i;
        t.lo = t.closest = rc < rb ? rc : rb;
        t.closest32 = (float)t.closest;
    }
}
template <typename Rec>
__device__ __forceinline__ void lazy_finish64(const Rec *__restrict__ prims, D3 o, D3 d, Trav64 &t) {
    if (t.hit_prim >= 0 && t.lo != t.closest) {
        const double a = dot(d, d);
        t.lo = t.closest = exact_root64(prims, t.hit_prim, o, d, a, RRT_F64_DIVA ? recip_a64(a) : 0.0);
    }
}

template <bool kCount, typename Rec>
__device__ __forceinline__ void leaves64(const Rec *__restrict__ prims, const float4 *__restrict__ recs32, Leaves lv,
                                         D3 o, D3 d, double a, const RaySphere32 &r32, bool pre, Trav64 &t,
                                         Counters &cnt) {
    const double ra = RRT_F64_DIVA ? recip_a64(a) : 0.0;
    const int first = (int)(lv & kLinkFirstMask), count = (int)(lv >> kLinkCountShift);
    uint32_t todo = (1u << count) - 1u;
    if (RRT_F64_SPHERE32 && pre) {
        // the ray's f32 constants: held from the ray start, or formed here per batch (fewer VGPRs
        // live across the node steps)
        const RaySphere32 rs = RRT_F64_S32_HOLD ? r32 : sphere32_ray(o.x, o.y, o.z, d.x, d.y, d.z);
        todo = 0;
        for (int j = 0; j < count; ++j) {
            const float4 c = recs32[first + j];
            if (!sphere32_miss(rs, c.x, c.y, c.z, c.w)) todo |= 1u << j;
        }
    }
    if (kCount) cnt.spheres += (uint32_t)count;
    if (RRT_F64_STATS == 5) {
        cnt.d2 += (uint32_t)count;
        cnt.d0 += (uint32_t)__popc(todo);
    }
    while (todo != 0) {
        const int i = first + __builtin_ctz(todo);
        todo &= todo - 1u;
        const Rec cr = prims[i];
        const D3 oc = sub(center_of(cr), o);
        const double h = dot(d, oc);
        const double c = dot(oc, oc) - radius_sq_of(cr);
        const double disc = h * h - a * c;
        if (RRT_F64_STATS == 3) cnt.d0++;
        if (disc < 0.0) continue;
        if (RRT_F64_STATS == 2 || RRT_F64_STATS == 3 || RRT_F64_STATS == 5) cnt.d1++;
        if constexpr (RRT_F64_LAZY && !kCount && RRT_F64_DIVA) {
            // |sv - sqrt(disc)| <= 2^-22.2 sqrt(disc): fl32(disc) moves the root by 2^-25 relative, and
            // v_sqrt_f32 is within 1.5 ulp (the f32 kernel's exhaustive device check); so
            // |q - r0| <= 2^-21.9 sv ra + 2^-50 (|h| + sv) ra, and e = 2^-20 (sv + |h|) ra bounds it
            // with 3.7x to spare (the f64 roundings of e and of q -+ e are ~2^-52 relative)
            const float df = (float)disc;
            const double sv = (double)__builtin_amdgcn_sqrtf(df);
            const double q = (h - sv) * ra;
            const double e = (sv + __builtin_fabs(h)) * (ra * 0x1.0p-20);
            const double l = q - e, u = q + e;
            const bool valid = (df >= 0x1.0p-96f) & (df <= 0x1.0p126f) & (l > 0.001);
            const bool acc = valid & (u < t.lo);
            const bool rej = valid & (l >= t.closest);
            t.lo = acc ? l : t.lo;
            t.closest = acc ? u : t.closest;
            t.closest32 = acc ? (float)u : t.closest32;
            t.hit_prim = acc ? i : t.hit_prim;
            if (!(acc | rej)) lazy_resolve64(prims, i, o, d, a, ra, t);
        } else {
            const double sq = sqrt64(disc);
            double root = div_a64(h - sq, a, ra);
            if (!(0.001 < root)) root = div_a64(h + sq, a, ra);
            if (0.001 < root && root < t.closest) {
                if (RRT_F64_STATS == 3) cnt.d2++;
                t.closest = root;
                t.lo = root;
                t.closest32 = (float)root;
                t.hit_prim = i;
            }
        }
    }
}

struct Path64 {
    D3 o, d;
#if !RRT_F64_B2F || RRT_F64_B2F_MODE == 1
    D3 T;
#endif
    RngState rng;
    uint32_t k;  // bounce index (camera ray = 0)
};

// Camera::get_ray (camera.rs:152-180) in f64 from the camera block the host widened to f64
// (KParams.cam64: the f32 ABI values cast as gpu/mod.rs:278-298 casts them; defocus_disk_u/v =
// u/v * radius formed in f64, camera.rs:136-138).
__device__ __forceinline__ void camera_ray64(uint32_t x, uint32_t y, Path64 &ps) {
    const auto &C = *kernarg_params();
    const double ox = rnd64(ps.rng) - 0.5, oy = rnd64(ps.rng) - 0.5;  // sample_square
    const double fi = (double)x + ox, fj = (double)y + oy;
#ifndef RRT_F64_CAM64
#define RRT_F64_CAM64 1
#endif
#if !RRT_F64_CAM64
    const D3 sample = d3(((double)C.p00[0] + (double)C.du[0] * fi) + (double)C.dv[0] * fj,
                         ((double)C.p00[1] + (double)C.du[1] * fi) + (double)C.dv[1] * fj,
                         ((double)C.p00[2] + (double)C.du[2] * fi) + (double)C.dv[2] * fj);
    D3 origin = f2d(C.center[0], C.center[1], C.center[2]);
#else
    const D3 sample = d3((C.cam64[0][0] + C.cam64[1][0] * fi) + C.cam64[2][0] * fj,
                         (C.cam64[0][1] + C.cam64[1][1] * fi) + C.cam64[2][1] * fj,
                         (C.cam64[0][2] + C.cam64[1][2] * fi) + C.cam64[2][2] * fj);
    D3 origin = d3(C.cam64[3][0], C.cam64[3][1], C.cam64[3][2]);
#endif
    if (C.defocus_radius > 0.0f) {
        int32_t a, b;
        for (;;) {  // vec3.rs:172-179 random_in_unit_disk, decided on integers (random_unit_vector)
            a = draw_centred(ps.rng);
            b = draw_centred(ps.rng);
            if (in_ball<true>(a, b, 0)) break;  // S < 2^46
        }
        const double px = centred_to_pm1(a), py = centred_to_pm1(b);
        const D3 du = d3(C.cam64[4][0], C.cam64[4][1], C.cam64[4][2]);
        const D3 dv = d3(C.cam64[5][0], C.cam64[5][1], C.cam64[5][2]);
        origin = add(add(origin, muls(du, px)), muls(dv, py));
    }
    if (C.flags & 0x1u) (void)rnd64(ps.rng);  // RRT_FLAG_RAY_TIME: the time draw (the_next_week/camera.rs:160)
    ps.o = origin;
    ps.d = sub(sample, origin);
#if !RRT_F64_B2F || RRT_F64_B2F_MODE == 1
    ps.T = d3(1.0, 1.0, 1.0);
#endif
    ps.k = 0;
}

// After the closest-hit query: sky / background, or emission / scatter / RR (camera.rs:182-209).
// Returns true when the path has ended; `Le` then holds the radiance at its end (sky, background,
// emission; 0 when absorbed, killed by Russian roulette or — in the caller — cut at max_depth),
// which the caller carries back to the camera ray (fold_back64). A scatter stores its attenuation at
// bounce k of the lane's history.
// kClass: kF64Full (every book-1 material kind), kF64Untextured (no image texture: the f64 acos /
// atan2 / texel path compiled out), kF64Diffuse (Lambertian and emissive only: metal and dielectric
// compiled out), chosen per scene by launch_render_pass_f64 like the f32 kernel's classes.
constexpr int kF64Full = 0, kF64Untextured = 1, kF64Diffuse = 2;
// RRT_F64_DEFER = n > 0: a Lambertian scatter's rejection loop (random_unit_vector) draws at most n
// candidates per pass of the work loop; a lane whose candidates all fail stays at its hit (ps.o = the
// hit point, ps.d = the normal, `prec` = the attenuation record, `pend` = 1), takes no closest-hit
// query, and draws on in the next pass. The same draws in the same order (candidates, then Russian
// roulette's), so the same path: only the wave's schedule changes. The wave no longer runs the
// loop until its unluckiest lane accepts (~5.6 wave-iterations for ~1.9 candidates per lane).
#ifndef RRT_F64_DEFER
#define RRT_F64_DEFER 0
#endif
template <int kClass, typename Rec>
__device__ __forceinline__ bool shade64(const KParams &P, const Rec *prims, const GMaterial *mtl, const double *inv_r,
                                        Path64 &ps, double t, int prim, D3 &Le, const Hist64 &hist, uint32_t &pend,
                                        HRec &prec) {
    Le = d3(0.0, 0.0, 0.0);
    if (prim < 0) {
        D3 bg;
        if (P.bg_mode == 1u) {
            bg = f2d(P.background[0], P.background[1], P.background[2]);
        } else {  // (1 - a) * (1, 1, 1) + a * (0.5, 0.7, 1)
            const D3 ud = unit_vector(ps.d);
            const double a = 0.5 * (ud.y + 1.0);
            bg = d3((1.0 - a) * 1.0 + a * 0.5, (1.0 - a) * 1.0 + a * 0.7, (1.0 - a) * 1.0 + a * 1.0);
        }
#if RRT_F64_B2F && RRT_F64_B2F_MODE != 1
        Le = bg;
#else
        Le = mul(ps.T, bg);
#endif
        return true;
    }
    const Rec cr = prims[prim];
    const D3 p = add(ps.o, muls(ps.d, t));  // Ray::at = orig + t * dir
#ifndef RRT_F64_HOST_INVR
#define RRT_F64_HOST_INVR 1
#endif
    // (p - center) / r = (1/r) * v (vec3.rs:142-148)
    const D3 outward = muls(sub(p, center_of(cr)), RRT_F64_HOST_INVR ? inv_r[prim] : 1.0 / radius_of(cr));
    const bool front = dot(ps.d, outward) < 0.0;
    const D3 nrm = front ? outward : d3(-outward.x, -outward.y, -outward.z);
    const GMaterial m = mtl[prim];
    const int kind = m.b.x;
    const D3 albedo = f2d(m.a.x, m.a.y, m.a.z);
    if (kind == 4) {  // DiffuseLight: emitted, scatter None
#if RRT_F64_B2F && RRT_F64_B2F_MODE != 1
        Le = albedo;
#else
        Le = mul(ps.T, albedo);
#endif
        return true;
    }
    D3 att, dir;
    HRec rec = rec_albedo(prim, m);  // the attenuation's history record
    if (kClass != kF64Diffuse && kind == 1) {  // Metal (material.rs:53-64): unit(reflect) + fuzz * random_unit_vector
        const D3 refl = unit_vector(reflect(ps.d, nrm));
        dir = add(refl, muls(random_unit_vector(ps.rng), (double)m.a.w));
        if (!(dot(dir, nrm) > 0.0)) return true;  // absorbed
        att = albedo;
    } else if (kClass != kF64Diffuse && kind == 2) {  // Dielectric (material.rs:83-102)
        const double eta = (double)__int_as_float(m.b.y);
#ifndef RRT_F64_DIEL_HOST
#define RRT_F64_DIEL_HOST 1
#endif
        double ri, r0;
        if (RRT_F64_DIEL_HOST) {  // 1 / eta and both r0 formed on the host (rrt_host.cpp dielectric_consts64)
            const double4 k = P.prim_diel64[prim];
            ri = front ? k.x : eta;
            r0 = front ? k.y : k.z;
        } else {
            ri = front ? 1.0 / eta : eta;
            r0 = (1.0 - ri) / (1.0 + ri);
            r0 = r0 * r0;
        }
        const D3 ud = unit_vector(ps.d);
        const double c = rmin(-dot(ud, nrm), 1.0);
        const double sn = __builtin_sqrt(1.0 - c * c);
        const bool cannot = ri * sn > 1.0;
        if (cannot || reflectance_r0(c, r0) > rnd64(ps.rng)) dir = reflect(ud, nrm);
        else dir = refract(ud, nrm, ri);
        att = d3(1.0, 1.0, 1.0);
        rec = rec_one();
    } else {  // Lambertian, plain or image-textured (material.rs:28-40; the_next_week/material.rs:41-53)
        att = albedo;
        if (kClass != kF64Untextured && kind == 3) {
            const uint32_t b = texel_bytes64(P, m.b.z, outward);
            att = texel_value64(b);
            rec = rec_texel(b);
        }
        if (RRT_F64_DEFER) {  // the scatter direction is drawn by the work loop (lambert_draw64)
            ps.o = p;
            ps.d = nrm;
            prec = rec;
            pend = 1;
            return false;
        }
        dir = add(nrm, random_unit_vector(ps.rng));
        if (__builtin_fabs(dir.x) < 1e-8 && __builtin_fabs(dir.y) < 1e-8 && __builtin_fabs(dir.z) < 1e-8) dir = nrm;
    }
    if (ps.k >= 5u) {  // camera.rs:189-200
        const double pr = rr_probability64(att);
        if (rnd64(ps.rng) > pr) return true;
#if !RRT_F64_B2F || RRT_F64_B2F_MODE == 1
        ps.T = muls(mul(ps.T, att), recip64(pr));
    } else {
        ps.T = mul(ps.T, att);
#endif
    }
#if RRT_F64_B2F
    hist.store(ps.k, rec);
#else
    (void)rec;
    (void)hist;
#endif
    ps.o = p;
    ps.d = dir;
    ps.k++;
    return false;
}

// A pending Lambertian scatter (RRT_F64_DEFER): up to RRT_F64_DEFER candidates of random_unit_vector
// (vec3.rs:181-189, decided on integers); on acceptance the scatter completes as in shade64 —
// direction nrm + unit, near_zero (material.rs:33-35), Russian roulette (camera.rs:189-200) and the
// history record. Returns 1 when the path ended (Russian roulette), 0 otherwise; pend = 0 once done.
template <int kClass>
__device__ __forceinline__ uint32_t lambert_draw64(const KParams &P, Path64 &ps, const Hist64 &hist, uint32_t &pend,
                                                   const HRec &prec, const GMaterial *mtl) {
    int32_t a = 0, b = 0, c = 0;
    bool ok = false;
    for (int it = 0; it < (RRT_F64_DEFER > 0 ? RRT_F64_DEFER : 1) && !ok; ++it) {
        a = draw_centred(ps.rng);
        b = draw_centred(ps.rng);
        c = draw_centred(ps.rng);
        ok = in_ball<false>(a, b, c);  // 0 < S <= 2^46
    }
    if (!ok) return 0u;
    pend = 0;
    const double x = centred_to_pm1(a), y = centred_to_pm1(b), z = centred_to_pm1(c);
    const double lensq = x * x + y * y + z * z;
    const D3 nrm = ps.d;
    D3 dir = add(nrm, muls(d3(x, y, z), recip64(__builtin_sqrt(lensq))));
    if (__builtin_fabs(dir.x) < 1e-8 && __builtin_fabs(dir.y) < 1e-8 && __builtin_fabs(dir.z) < 1e-8) dir = nrm;
    if (ps.k >= 5u) {
        const D3 att = rec_att<kClass != kF64Untextured>(prec, mtl);
        if (rnd64(ps.rng) > rr_probability64(att)) return 1u;
    }
    hist.store(ps.k, prec);
    ps.d = dir;
    ps.k++;
    return 0u;
}

// The persistent work loop of rrt_kernel.hip's render_body (same queue, units, chunk order,
// postponed leaves and wave-uniform exits) over Path64 state.
// kMode: kF64Global (f16 nodes and records read from global memory), kF64Lds (the f32 nodes as
// Node112 and the spheres staged in LDS), kF64LdsWide (the same with the sphere records widened to
// f64, Sphere64, when the block stays within 64 KB). The 1/r table joins an LDS scene when it fits.
constexpr int kF64Global = 0, kF64Lds = 1, kF64LdsWide = 2;
template <int kMode, bool kCount, int kBlk, int kClass>
__device__ __forceinline__ void render64_body(const KParams &P) {
    constexpr bool kLds = kMode != kF64Global;
    using Rec = typename std::conditional<kMode == kF64LdsWide, Sphere64, float4>::type;
    extern __shared__ uint4 lds_dyn[];
    uint16_t *lds_stack = reinterpret_cast<uint16_t *>(lds_dyn);
    using Node = typename std::conditional<kLds, GNode, GNodeH>::type;
    const Node *nodes = reinterpret_cast<const Node *>(P.nodes);
    const Rec *prims = reinterpret_cast<const Rec *>(P.prim_cr);
    const GMaterial *mtl = P.prim_mtl;
    const double *inv_r = P.prim_inv_r64;
    const float4 *recs32 = P.prim_cr;  // the pre-test's f32 records (center, r)
    const uint32_t stack16 = (P.stack_depth * kBlk * sizeof(uint16_t) + 15u) / 16u;
    constexpr uint32_t kRing16 = (uint32_t)RRT_F64_LDS_HIST * kBlk * (uint32_t)sizeof(HRec) / 16u;  // kBlk: a multiple of 64
    if constexpr (kLds) {  // stage nodes + spheres (+ 1/r) once per block
        uint4 *dst = lds_dyn + stack16 + kRing16;
        // Node112: each 80-B GNode re-laid as 112 B whose axis a holds both children's (lo, hi), then
        // both (hi, lo), and the links at 96 — one ds_read_b128 per axis at the ray's sign offset
        // reads both children's (entry, exit) pairs (4 LDS cycles, against 8 for two ds_read2_b32):
        // C2 +0.5 %, C4 +0.6 % same-box. The materials stay in global memory (one 32-B read per hit)
        // so the block keeps within the 64 KB it may declare.
        uint32_t nn;
        {
            const GNode *sn = reinterpret_cast<const GNode *>(P.nodes);
            for (uint32_t i = threadIdx.x; i < P.n_nodes; i += kBlk) {
                const GNode g = sn[i];
                uint4 *o = dst + 7u * i;
                for (int ax = 0; ax < 3; ++ax) {
                    const uint32_t lo0 = __float_as_uint(g.box[0][3 * ax]), hi0 = __float_as_uint(g.box[0][3 * ax + 1]);
                    const uint32_t lo1 = __float_as_uint(g.box[1][3 * ax]), hi1 = __float_as_uint(g.box[1][3 * ax + 1]);
                    o[2 * ax] = make_uint4(lo0, hi0, lo1, hi1);
                    o[2 * ax + 1] = make_uint4(hi0, lo0, hi1, lo1);
                }
                o[6] = make_uint4(g.link[0], g.link[1], 0u, 0u);
            }
            nn = 7u * P.n_nodes;
        }
        constexpr uint32_t kRec16 = (uint32_t)(sizeof(Rec) / 16);
        for (uint32_t i = threadIdx.x; i < P.n_prims; i += kBlk) {
            const float4 c = P.prim_cr[i];
            if constexpr (kMode == kF64LdsWide)
                reinterpret_cast<Sphere64 *>(dst + nn)[i] = Sphere64{(double)c.x, (double)c.y, (double)c.z,
                                                                         RRT_F64_R2 ? (double)c.w * (double)c.w : (double)c.w};
            else
                reinterpret_cast<float4 *>(dst + nn)[i] = c;
        }
        const uint32_t np = P.n_prims * kRec16;
        double *dr = reinterpret_cast<double *>(dst + nn + np);
        if (P.inv_r_in_lds)
            for (uint32_t i = threadIdx.x; i < P.n_prims; i += kBlk) dr[i] = P.prim_inv_r64[i];
        // the f32 records of the pre-test, after the 1/r table (widened layout only; otherwise the
        // staged records are the f32 ones)
        float4 *d32 = reinterpret_cast<float4 *>(dst + nn + np + (P.inv_r_in_lds ? (P.n_prims + 1u) / 2u : 0u));
        if (kMode == kF64LdsWide && P.rec32_in_lds)
            for (uint32_t i = threadIdx.x; i < P.n_prims; i += kBlk) d32[i] = P.prim_cr[i];
        __syncthreads();
        nodes = reinterpret_cast<const Node *>(dst);
        prims = reinterpret_cast<const Rec *>(dst + nn);
        if (P.inv_r_in_lds) inv_r = dr;
        if constexpr (kMode == kF64LdsWide) {
            if (P.rec32_in_lds) recs32 = d32;
        } else {
            recs32 = reinterpret_cast<const float4 *>(prims);
        }
    }
    LdsStack<uint16_t, kBlk> stack;
    stack.init(lds_stack, threadIdx.x);

    const uint32_t lane = threadIdx.x & 63u;
    Counters cnt = {0, 0, 0, 0, 0, 0};
    uint32_t w_rays = 0, w_paths = 0;
    uint32_t has = 0, need_ray = 0;
    bool q_open = true;
    uint32_t xy = 0, s = 0, s_hi = 0;
    uint32_t px = 0;         // the unit's tile-local pixel index
    uint32_t tail = 0;       // the unit is a tail chunk: its samples' radiances go to seq64 one by one
    uint32_t tcidx = 0;      // a tail unit's chunk index within the pass
    uint32_t tmask = 0;      // a tail unit's samples with nonzero radiance (bit = sample - its first)
    uint32_t pend = 0;       // RRT_F64_DEFER: a Lambertian scatter waits for an accepted candidate
    HRec prec{};
    const Hist64 hist{reinterpret_cast<HRec *>(lds_dyn + stack16), reinterpret_cast<HRec *>(P.hist), P.hist_lanes,
                      blockIdx.x * (uint32_t)kBlk + threadIdx.x, threadIdx.x, (uint32_t)kBlk};
    uint64_t pkey = 0;
    D3 sum = d3(0.0, 0.0, 0.0);
    Path64 ps;
    Trav64 tr;
    tr.node = -1;
    [[maybe_unused]] uint64_t ph0 = 0, ph1 = 0, ph2 = 0, tp = 0;
    uint32_t pool_base = (blockIdx.x & (kQueues - 1u)) * 64u, pool_left = 0;  // queue claims: rrt_kernel.hip
    for (;;) {
        if constexpr (RRT_F64_STATS == 1) tp = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_s_setprio(kPrioRefill);
        const uint64_t idle = __ballot(!has);
        if (idle != 0 && pool_left == 0 && q_open) {
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
                const auto &Q = *kernarg_params();
                const uint32_t u = pool_base + r;
                const uint32_t lit = u & 63u, tc = u >> 6;
                uint32_t t, chunk;  // big chunks of every tile first, then the tail chunks
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
                    const uint32_t band = fast_div(ly, fdiv(Q.fd_band_rows));
                    const uint32_t slot = (band & 1u) ? Q.n_ranks - 1u - Q.rank : Q.rank;  // serpentine bands
                    const uint32_t y = (band * Q.n_ranks + slot) * Q.band_rows + (ly - band * Q.band_rows);
                    xy = x | (y << 16);
                    s = Q.sample_begin + chunk_first(Q, chunk);
                    s_hi = min(s + (chunk < Q.n_big ? Q.chunk : Q.chunk_small), Q.sample_end);
                    px = ly * Q.width + x;
                    tail = Q.seq && chunk >= Q.n_big ? 1u : 0u;
                    tcidx = tail ? fast_div(s - Q.sample_begin - Q.seq_first, fdiv(Q.fd_chunk_small)) : 0u;
                    tmask = 0u;
                    sum = d3(0.0, 0.0, 0.0);
                    pkey = pixel_key(Q, x, y);
                    ps.rng = path_rng_k(pkey, s);
                    camera_ray64(x, y, ps);
                    need_ray = 1;
                    has = 1;
                }
            }
            pool_base += n;
            pool_left -= n;
        }
        if (__ballot(has) == 0) break;

        uint32_t seg_done = 0, started = 0;
        if (has && need_ray) {
            if (ps.k >= P.max_depth) {  // ray_color: depth <= 0 -> 0 (no query)
                seg_done = 1;
            } else {
                tr.closest = __builtin_inf();  // Interval(0.001, INFINITY)
                tr.lo = __builtin_inf();
                tr.closest32 = __builtin_inff();
                tr.hit_prim = -1;
                tr.node = 0;
                tr.sp = 0;
                need_ray = 0;
                started = 1;
            }
        }
        w_rays += (uint32_t)__popcll(__ballot(started));
        const uint32_t live = (uint32_t)__popcll(__ballot(has));
        const uint32_t min_active = (live * P.trav_frac) >> 8;
        const uint32_t leaf_min = (live * P.leaf_frac) >> 8;
        if constexpr (RRT_F64_STATS == 1) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph0 += t - tp;
            tp = t;
        }
        RayK64 rk;
        RaySphere32 r32;
        double a = 0.0;
        if (tr.node >= 0) {
            rk = ray_consts64(ps.o, ps.d);
            if (RRT_F64_SPHERE32 && RRT_F64_S32_HOLD) r32 = sphere32_ray(ps.o.x, ps.o.y, ps.o.z, ps.d.x, ps.d.y, ps.d.z);
            a = dot(ps.d, ps.d);  // sphere.rs:27 r.direction().length_squared()
        }
        __builtin_amdgcn_s_setprio(kPrioNode);
        Leaves lv = 0;
        for (;;) {
            if constexpr (RRT_F64_STATS == 4) {
                const uint64_t sm = __ballot(tr.node >= 0 && lv == 0);
                if (sm != 0) {
                    ph0 += 1;
                    ph1 += (uint64_t)__popcll(sm);
                }
            }
            if (tr.node >= 0 && lv == 0) {
                Leaves l;
                if (trav_node64<kCount>(nodes, stack, rk, tr, l, cnt)) lv = l;
            }
            const uint64_t pm = __ballot(lv != 0);
            const uint64_t tm = __ballot(tr.node >= 0) | pm;
            const bool leave = (uint32_t)__popcll(tm) <= min_active;
            const bool batch = ((uint32_t)__popcll(pm) > leaf_min) | leave | (tm == pm);
            if ((pm != 0) & batch) {
                __builtin_amdgcn_s_setprio(kPrioLeaf);
                [[maybe_unused]] const uint32_t n_l = lv >> kLinkCountShift, s_l = cnt.d1;
                if (lv != 0) {
                    leaves64<kCount>(prims, recs32, lv, ps.o, ps.d, a, r32, P.sphere32 != 0u, tr, cnt);
                    lv = 0;
                }
                if constexpr (RRT_F64_STATS == 2) {
                    ph0 += wave_max_u32(n_l);
                    ph1 += wave_max_u32(cnt.d1 - s_l);
                    ph2 += 1;
                }
                if constexpr (RRT_F64_STATS == 4) ph2 += 64;
                __builtin_amdgcn_s_setprio(kPrioNode);
            }
            if (leave) break;
        }
        if constexpr (RRT_F64_STATS == 1) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            ph1 += t - tp;
            tp = t;
        }
        __builtin_amdgcn_s_setprio(kPrioShade);
        D3 Le = d3(0.0, 0.0, 0.0);
        if (has && !need_ray && tr.node < 0 && !pend) {
            need_ray = 1;
            if constexpr (RRT_F64_LAZY && !kCount && RRT_F64_DIVA) lazy_finish64(prims, ps.o, ps.d, tr);
            seg_done = shade64<kClass>(P, prims, mtl, inv_r, ps, tr.closest, tr.hit_prim, Le, hist, pend, prec) ? 1u : 0u;
        }
        if (RRT_F64_DEFER && pend) {
            seg_done = lambert_draw64<kClass>(P, ps, hist, pend, prec, mtl);
            need_ray = pend ? 0u : 1u;
        }
        w_paths += (uint32_t)__popcll(__ballot(seg_done));
        if (seg_done) {  // pixel_color += ray_color(..) (camera.rs:72-76)
#if RRT_F64_B2F && RRT_F64_B2F_MODE != 1
            // the radiance at the path's end carried back through its scatters; a path that ended
            // with none (absorbed, Russian roulette, max_depth) adds an exact 0
            if (Le.x != 0.0 || Le.y != 0.0 || Le.z != 0.0)
                Le = fold_back64<kClass != kF64Untextured>(hist, mtl, ps.k, Le);
#endif
            const auto &Q = *kernarg_params();
            if (tail) {  // a tail sample: its radiance, folded into the pixel's sum in order later
                // only nonzero radiances are kept (an exact 0 leaves BOOKS' sum unchanged), packed in
                // sample order, with the unit's mask of which samples they are
                if (Le.x != 0.0 || Le.y != 0.0 || Le.z != 0.0) {
                    const size_t npx = (size_t)Q.tile_rows * Q.width;
                    const uint32_t j = (uint32_t)__popc(tmask);
                    double *o = Q.seq64 + 3u * (((size_t)tcidx * Q.chunk_small + j) * npx + px);
#ifndef RRT_F64_SEQ_NT
#define RRT_F64_SEQ_NT 1
#endif
                    if (RRT_F64_SEQ_NT) {  // streamed (read once, by the fold after the pass): kept
                        __builtin_nontemporal_store(Le.x, o);  // from evicting the history's lines in L2
                        __builtin_nontemporal_store(Le.y, o + 1);
                        __builtin_nontemporal_store(Le.z, o + 2);
                    } else {
                        o[0] = Le.x;
                        o[1] = Le.y;
                        o[2] = Le.z;
                    }
                    tmask |= 1u << (s - Q.sample_begin - Q.seq_first - tcidx * Q.chunk_small);
                }
            } else {
                sum = add(sum, Le);
            }
            ++s;
            const uint32_t x = xy & 0xffffu, y = xy >> 16;
            if (s < s_hi) {
                ps.rng = path_rng_k(pkey, s);
                camera_ray64(x, y, ps);
            } else {  // unit complete: the chunk's f64 sum, in sample order
                const uint32_t rel = s_hi - 1u - Q.sample_begin;
                const uint32_t nbs = Q.n_big * Q.chunk;
                const uint32_t chunk =
                    rel < nbs ? fast_div(rel, fdiv(Q.fd_chunk)) : Q.n_big + fast_div(rel - nbs, fdiv(Q.fd_chunk_small));
                const D4 out{sum.x, sum.y, sum.z, (double)(s_hi - (Q.sample_begin + chunk_first(Q, chunk)))};
                if (Q.n_chunks == 1 || (Q.seq && !tail)) Q.accum64[px] = out;  // the whole pixel, or its prefix
                else if (!tail) Q.partial64[(size_t)(chunk - Q.chunk_begin) * ((size_t)Q.tile_rows * Q.width) + px] = out;
                else Q.seqmask[(size_t)tcidx * ((size_t)Q.tile_rows * Q.width) + px] = tmask;
                has = 0;
            }
        }
        if constexpr (RRT_F64_STATS == 1) ph2 += __builtin_amdgcn_s_memtime() - tp;
    }
    if constexpr ((RRT_F64_STATS == 3 || RRT_F64_STATS == 5) && !kCount) {
        ph0 = wave_sum_u32(cnt.d0);
        ph1 = wave_sum_u32(cnt.d1);
        ph2 = wave_sum_u32(cnt.d2);
    }
    if constexpr (RRT_F64_STATS != 0 && !kCount) {
        if (lane == 0) {
            atomicAdd(&P.counters[2], (unsigned long long)ph0);
            atomicAdd(&P.counters[3], (unsigned long long)ph1);
            atomicAdd(&P.counters[4], (unsigned long long)ph2);
        }
    }
    uint32_t nv = 0, bt = 0, st = 0;
    if (kCount) {
        nv = wave_sum_u32(cnt.nodes);
        bt = wave_sum_u32(cnt.boxes);
        st = wave_sum_u32(cnt.spheres);
    }
    if (lane == 0) {
        if (w_rays) atomicAdd(&P.counters[0], (unsigned long long)w_rays);
        if (w_paths) atomicAdd(&P.counters[1], (unsigned long long)w_paths);
        if (kCount) {
            atomicAdd(&P.counters[2], (unsigned long long)nv);
            atomicAdd(&P.counters[3], (unsigned long long)bt);
            atomicAdd(&P.counters[4], (unsigned long long)st);
        }
    }
}

#ifndef RRT_F64_BLOCK
#define RRT_F64_BLOCK 512
#endif
#ifndef RRT_F64_WAVES
#define RRT_F64_WAVES 4  // waves/SIMD bound of the untextured and diffuse classes (<= 128 VGPRs, no spills)
#endif
constexpr int kBlock64 = RRT_F64_BLOCK;  // threads per block of the f64 kernel
// The full class (texture + specular) needs more than 128 VGPRs (3 waves/SIMD): 512-thread blocks,
// since a block of 1024 needs 4 waves per SIMD.
__host__ __device__ constexpr int blk64(int cls) { return cls == 0 ? 512 : kBlock64; }
// LDS one block may declare: 160 KiB on gfx950 (MI355X_MICROARCH.md occupancy section) when the
// block is the CU's only one (1024 threads at 4 waves/SIMD), else the 64 KiB that keeps two
// 512-thread blocks per CU
#ifndef RRT_F64_LDS512_KB
#define RRT_F64_LDS512_KB 64
#endif
__host__ __device__ constexpr size_t lds_budget64(int blk) {
    return blk >= 1024 ? 160u * 1024u : (size_t)RRT_F64_LDS512_KB * 1024u;
}

template <int kMode, bool kCount, int kClass>
__global__ __launch_bounds__(blk64(kClass), kClass == kF64Full ? 1 : RRT_F64_WAVES) void rrt_render64(KParams P) {
    render64_body<kMode, kCount, blk64(kClass), kClass>(P);
}

// The pass's f64 chunk sums into accum64, continuing the left fold over chunks in order (as
// rrt_combine_chunks); w = the tile's sample count.
__global__ __launch_bounds__(256) void rrt_combine_chunks64(const D4 *__restrict__ partial, D4 *__restrict__ accum,
                                                            uint32_t n_pixels, uint32_t n_chunks, uint32_t first,
                                                            double count) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n_pixels) return;
    D4 acc = first ? partial[p] : accum[p];
    for (uint32_t c = first ? 1u : 0u; c < n_chunks; ++c) {
        const D4 v = partial[(size_t)c * n_pixels + p];
        acc.x = acc.x + v.x;
        acc.y = acc.y + v.y;
        acc.z = acc.z + v.z;
    }
    accum[p] = D4{acc.x, acc.y, acc.z, count};
}

// Sequential-sum mode: the pass's tail-sample radiances added to each pixel's sum in sample order
// (pixel_color += ray_color(..), camera.rs:72-76), continuing from the prefix chunk's sum (or the
// previous pass's); w = the samples summed so far.
// The tail units kept each chunk's nonzero radiances packed in sample order plus a mask; the zero
// ones add nothing (s + 0 = s for the nonnegative sums), so the fold skips them.
__global__ __launch_bounds__(256) void rrt_fold_samples64(const double *__restrict__ seq,
                                                          const uint32_t *__restrict__ masks, D4 *__restrict__ accum,
                                                          uint32_t n_pixels, uint32_t n_chunks, uint32_t chunk_small,
                                                          double count) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n_pixels) return;
    D4 acc = accum[p];
    for (uint32_t c = 0; c < n_chunks; ++c) {
        const uint32_t n = (uint32_t)__popc(masks[(size_t)c * n_pixels + p]);
        for (uint32_t j = 0; j < n; ++j) {
            const double *v = seq + 3u * (((size_t)c * chunk_small + j) * n_pixels + p);
            acc.x = acc.x + v[0];
            acc.y = acc.y + v[1];
            acc.z = acc.z + v[2];
        }
    }
    accum[p] = D4{acc.x, acc.y, acc.z, count};
}

// f64 sums rounded to the ABI's f32 RGBA accum (round to nearest: the closest f32 to each sum).
__global__ __launch_bounds__(256) void rrt_accum64_to_f32(const D4 *__restrict__ a64, float4 *__restrict__ a32,
                                                          uint32_t n_pixels) {
    const uint32_t p = blockIdx.x * 256u + threadIdx.x;
    if (p >= n_pixels) return;
    const D4 v = a64[p];
    a32[p] = make_float4((float)v.x, (float)v.y, (float)v.z, (float)v.w);
}

// LDS of the f64 kernel's block in each mode (stack, then the staged scene; the 1/r table when
// p.inv_r_in_lds)
// Test support (rrt_testing_trig32_check): the largest |acosf(x) - acos(x)| over every f32 x in
// [-1, 1] and |atanf(t) - atan(t)| over every f32 t in [0, 1], against the device's f64 functions,
// as f64 bit patterns (non-negative doubles order as their bits) in out[0], out[1].
__global__ __launch_bounds__(256) void rrt_trig32_check(unsigned long long *out) {
    double e_acos = 0.0, e_atan = 0.0;
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k <= 0x3f800000ull; k += (uint64_t)gridDim.x * 256ull) {
        const float x = __uint_as_float((uint32_t)k);  // every f32 in [0, 1]
        const double dx = (double)x;
        double d = __builtin_fabs((double)acosf(x) - acos(dx));
        e_acos = d > e_acos ? d : e_acos;
        d = __builtin_fabs((double)acosf(-x) - acos(-dx));
        e_acos = d > e_acos ? d : e_acos;
        d = __builtin_fabs((double)atanf(x) - atan(dx));
        e_atan = d > e_atan ? d : e_atan;
    }
    for (int off = 32; off > 0; off >>= 1) {
        e_acos = fmax(e_acos, __shfl_xor(e_acos, off, 64));
        e_atan = fmax(e_atan, __shfl_xor(e_atan, off, 64));
    }
    if ((threadIdx.x & 63u) == 0u) {
        atomicMax(&out[0], (unsigned long long)__double_as_longlong(e_acos));
        atomicMax(&out[1], (unsigned long long)__double_as_longlong(e_atan));
    }
}

// Test support (rrt_testing_sqrt64_check): sqrt64_big against the library root, bit for bit, on
// 2^28 arguments: every exponent from 2^-767 up to the largest finite, each with a random and a
// nearly-square mantissa (k^2 and its neighbours, where the rounding is decided by the corrections),
// plus +-0 and +inf. out[0] counts differing results, out[1] the arguments checked.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void rrt_sqrt64_check(unsigned long long *out) {
    uint32_t bad = 0, n = 0;
    for (uint64_t k = blockIdx.x * 256ull + threadIdx.x; k < (1ull << 28); k += (uint64_t)gridDim.x * 256ull) {
        const uint64_t r = mix64(k);
        const uint64_t e = 256u + (r >> 52) % (2046u - 256u);  // biased exponents of [2^-767, 2^1023)
        uint64_t bits;
        if (k & 1u) {
            bits = (e << 52) | (r & 0xFFFFFFFFFFFFFull);
        } else {  // a square of a 26-bit integer (exact), scaled, then moved by a few ulps
            const double q = (double)(((r >> 8) & 0x3FFFFFFu) | 1u);
            const double sq = q * q;
            const uint64_t b = (uint64_t)__double_as_longlong(sq);
            bits = ((b & 0xFFFFFFFFFFFFFull) | (((e & ~1ull) | 0x1ull) << 52)) + ((r >> 3) & 7u) - 3u;
        }
        if (k < 4) bits = k == 0 ? 0ull : k == 1 ? 0x8000000000000000ull : k == 2 ? 0x7FF0000000000000ull : 0x0010000000000000ull;
        const double x = __longlong_as_double((long long)bits);
        if (sqrt64_small(x)) continue;
        ++n;
        if (__double_as_longlong(sqrt64_big(x)) != __double_as_longlong(__builtin_sqrt(x))) ++bad;
    }
    atomicAdd(&out[0], (unsigned long long)bad);
    atomicAdd(&out[1], (unsigned long long)n);
}

size_t lds64_bytes(const KParams &p, int mode, int blk = kBlock64) {
    size_t lds = ((size_t)p.stack_depth * blk * sizeof(uint16_t) + 15u) / 16u * 16u;
    lds += (size_t)RRT_F64_LDS_HIST * blk * sizeof(HRec);  // the history ring
    if (mode != kF64Global)
        lds += (size_t)p.n_nodes * 112u +
               (size_t)p.n_prims * ((mode == kF64LdsWide ? sizeof(Sphere64) : sizeof(float4)) +
                                    (p.inv_r_in_lds ? sizeof(double) : 0u) +
                                    (mode == kF64LdsWide && p.rec32_in_lds ? sizeof(float4) : 0u)) +
               (p.inv_r_in_lds ? 8u : 0u);  // the f32 records start 16-B aligned
    return lds;
}

}  // namespace

size_t f64_lds_min_bytes(uint32_t n_nodes, uint32_t n_prims, uint32_t stack_depth) {
    KParams p{};
    p.n_nodes = n_nodes;
    p.n_prims = n_prims;
    p.stack_depth = stack_depth;
    p.inv_r_in_lds = 0u;
    p.rec32_in_lds = 0u;
    // the host's staging rule (rrt_host.cpp scene_bvh): the 512-thread block's layout without the
    // history ring within 64 KB, whatever block the classes launch
    return lds64_bytes(p, kF64Lds, 512) - (size_t)RRT_F64_LDS_HIST * 512u * sizeof(HRec);
}

namespace {

template <int kMode, int kClass>
hipError_t launch64(const KParams &p, bool count, hipStream_t stream) {
    constexpr int B = blk64(kClass);
    const size_t lds = lds64_bytes(p, kMode, B);
    if (lds > lds_budget64(B)) return hipErrorInvalidValue;
    auto kernel = count ? rrt_render64<kMode, true, kClass> : rrt_render64<kMode, false, kClass>;
    hipError_t e;
    if (lds > 64u * 1024u) {  // beyond the default dynamic-LDS limit (gfx950 allows 160 KiB per block)
        e = hipFuncSetAttribute(reinterpret_cast<const void *>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
        if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, B, lds);
    if (e != hipSuccess) return e;
    if (per_cu < 1) per_cu = 1;
    const uint32_t want = (p.n_units + B - 1) / B;
    uint32_t blocks = std::max<uint32_t>(std::min<uint32_t>(want, (uint32_t)per_cu * p.n_cus), kQueues);
    if (RRT_F64_B2F) {  // every lane needs a history slot
        if (!p.hist || p.hist_lanes < kQueues * (uint32_t)B) return hipErrorInvalidValue;
        blocks = std::min<uint32_t>(blocks, p.hist_lanes / (uint32_t)B);
    }
    e = hipMemsetAsync(p.unit_counter, 0, kQueues * 32u * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(B), lds, stream, p);
    return hipGetLastError();
}

// The scene placement: the f32 nodes, spheres and materials in LDS when they fit (C1, C2, C4), else
// the f16 nodes and records from global memory (C5).
#ifndef RRT_F64_WIDE_SPHERES
#define RRT_F64_WIDE_SPHERES 1
#endif
// rrt_testing_f64_layout: a forced LDS layout (bit 0: widened Sphere64 records, bit 1: the 1/r table,
// bit 2: the f32 pre-test records beside widened ones), or -1 for the automatic choice below
std::atomic<int> g_f64_layout{-1};

template <int kClass>
hipError_t launch64_placed(const KParams &p, bool count, hipStream_t stream) {
    if (!p.scene_in_lds) return launch64<kF64Global, kClass>(p, count, stream);
    if (const int lay = g_f64_layout.load(); lay >= 0) {
        KParams q = p;
        const bool wide = (lay & 1) != 0;
        q.inv_r_in_lds = (lay & 2) ? 1u : 0u;
        q.rec32_in_lds = wide && (lay & 4) ? 1u : 0u;
        if (lds64_bytes(q, wide ? kF64LdsWide : kF64Lds, blk64(kClass)) > lds_budget64(blk64(kClass)))
            return hipErrorInvalidValue;
        return wide ? launch64<kF64LdsWide, kClass>(q, count, stream) : launch64<kF64Lds, kClass>(q, count, stream);
    }
    // the widened sphere records and the 1/r table join the staged scene while the block stays
    // within the 64 KB it may declare
    // (widened records before the 1/r table: a sphere test reads a record, a hit reads 1/r)
    KParams q = p;
    q.rec32_in_lds = 0u;
#ifndef RRT_F64_PREFER_F32REC
#define RRT_F64_PREFER_F32REC 0
#endif
    if (RRT_F64_WIDE_SPHERES && !(RRT_F64_PREFER_F32REC && p.sphere32)) {
        // with the pre-test: the f32 records staged too, or read from global memory (L1 / L2)
        for (const uint32_t rec32 : {p.sphere32 && RRT_F64_SPHERE32 ? 1u : 0u, 0u}) {
            q.rec32_in_lds = rec32;
            for (const uint32_t inv_r : {1u, 0u}) {
                q.inv_r_in_lds = inv_r;
                if (lds64_bytes(q, kF64LdsWide, blk64(kClass)) <= lds_budget64(blk64(kClass)))
                    return launch64<kF64LdsWide, kClass>(q, count, stream);
            }
        }
    }
    q.rec32_in_lds = 0u;
    q.inv_r_in_lds = 1u;
    if (lds64_bytes(q, kF64Lds, blk64(kClass)) > lds_budget64(blk64(kClass))) q.inv_r_in_lds = 0u;
    return launch64<kF64Lds, kClass>(q, count, stream);
}

}  // namespace

hipError_t launch_render_pass_f64(const KParams &p, bool count, hipStream_t stream) {
    if (p.n_units == 0) return hipSuccess;
    if (p.bvh_width != 2 || p.prim_motion || p.stack_depth > (uint32_t)kMaxStackDepth || p.n_nodes > 65535u)
        return hipErrorInvalidValue;  // the host builds a 16-bit-stack BVH2 for book-1 scenes
#ifndef RRT_F64_CLASSES
#define RRT_F64_CLASSES 1
#endif
    hipError_t e;
    if (RRT_F64_CLASSES && !p.specular) e = launch64_placed<kF64Diffuse>(p, count, stream);
    else if (RRT_F64_CLASSES && !p.image_tex) e = launch64_placed<kF64Untextured>(p, count, stream);
    else e = launch64_placed<kF64Full>(p, count, stream);
    if (e != hipSuccess || p.n_chunks <= 1 || p.seq) return e;
    const uint32_t n_pixels = p.tile_rows * p.width;
    hipLaunchKernelGGL(rrt_combine_chunks64, dim3((n_pixels + 255) / 256), dim3(256), 0, stream, p.partial64,
                       p.accum64, n_pixels, p.pass_n, p.chunk_begin == 0 ? 1u : 0u,
                       (double)(p.sample_end - p.sample_begin));
    return hipGetLastError();
}

void set_f64_layout(int layout) { g_f64_layout.store(layout < 0 ? -1 : layout & 7); }

// Passes of the sequential-sum schedule: the first holds the prefix chunk (chunk 0) and up to
// pass_chunks tail chunks, each later one up to pass_chunks tail chunks; after a pass its tail samples
// are folded into accum64 in order.
hipError_t launch_sqrt64_check(unsigned long long *d_out, hipStream_t stream) {
    hipLaunchKernelGGL(rrt_sqrt64_check, dim3(8192), dim3(256), 0, stream, d_out);
    return hipGetLastError();
}

hipError_t launch_trig32_check(unsigned long long *d_out, double *bounds, hipStream_t stream) {
    bounds[0] = kAcos32Err;
    bounds[1] = kAtan32Err;
    hipLaunchKernelGGL(rrt_trig32_check, dim3(4096), dim3(256), 0, stream, d_out);
    return hipGetLastError();
}

hipError_t launch_render_f64_seq(const KParams &p, bool count, hipStream_t stream) {
    const uint32_t n_tail = p.n_chunks > 0 ? p.n_chunks - 1u : 0u, m = std::max(1u, p.pass_chunks);
    const uint32_t n_pixels = p.tile_rows * p.width;
    const uint32_t S = p.sample_end - p.sample_begin;
    uint32_t cb = 0;
    while (cb < p.n_chunks) {
        KParams q = p;
        q.chunk_begin = cb;
        q.pass_big = cb == 0 ? std::min(1u, p.n_big) : 0u;
        q.pass_n = cb == 0 ? 1u + std::min(m, n_tail) : std::min(m, p.n_chunks - cb);
        if (p.n_big == 0) q.pass_n = p.n_chunks;  // one chunk: the whole pixel
        q.n_big_units = p.n_work_tiles * q.pass_big * 64u;
        q.n_units = p.n_work_tiles * q.pass_n * 64u;
        q.fd_pass_big = make_fastdiv(q.pass_big);
        q.fd_pass_tail = make_fastdiv(q.pass_n - q.pass_big);
        const uint32_t end = cb + q.pass_n;
        const uint32_t tail0 = std::max(cb, p.n_big);  // the pass's first tail chunk
        q.seq_first = tail0 < end ? chunk_first(p, tail0) : 0u;
        hipError_t e = launch_render_pass_f64(q, count, stream);
        if (e != hipSuccess) return e;
        if (tail0 < end) {
            const uint32_t done = std::min(S, chunk_first(p, end));
            hipLaunchKernelGGL(rrt_fold_samples64, dim3((n_pixels + 255) / 256), dim3(256), 0, stream, p.seq64,
                               p.seqmask, p.accum64, n_pixels, end - tail0, p.chunk_small, (double)done);
            e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
        cb = end;
    }
    return hipSuccess;
}

hipError_t launch_accum64_to_f32(const D4 *d_accum64, float4 *d_accum, uint32_t n_pixels, hipStream_t stream) {
    if (n_pixels == 0) return hipSuccess;
    hipLaunchKernelGGL(rrt_accum64_to_f32, dim3((n_pixels + 255) / 256), dim3(256), 0, stream, d_accum64, d_accum,
                       n_pixels);
    return hipGetLastError();
}

}  // namespace rrt
