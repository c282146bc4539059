// rrt_oracle.cpp — CPU restatement of the reference's "books" path. TEST INFRASTRUCTURE ONLY:
// only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
// library, and only as the checker / CPU baseline — never as the thing measured or shipped.
//
// The reference (jwheo12/RustRayTrace) is Rust and cannot be built here (no cargo/rustc,
// no crates offline: SURVEY §8c). This file restates its CPU path as text, function by
// function (citations are relative to /root/reference/src):
//
//   Vec3 / dot / unit_vector / reflect / refract / random_*   books/in_one_weekend/vec3.rs
//   Interval::surrounds / clamp                               books/in_one_weekend/interval.rs:30-42
//   Aabb::new / from_points / from_boxes / hit / pad          books/in_one_weekend/aabb.rs:23-115
//   BvhNode::build (binned SAH, 12 buckets) / hit             books/in_one_weekend/bvh.rs:16-172
//   Sphere::new / hit, HitRecord::new                          books/in_one_weekend/sphere.rs:16-51, hittable.rs:20-32
//   Lambertian / Metal / Dielectric scatter, reflectance      books/in_one_weekend/material.rs:28-102
//   Camera::get_ray / sample_square / defocus_disk_sample     books/in_one_weekend/camera.rs:152-180
//   Camera::ray_color (recursive, RR from bounce 5)           books/in_one_weekend/camera.rs:182-209
//   book-2 ray_color (emission, background), time draw        books/the_next_week/camera.rs:148-201
//   get_sphere_uv, ImageTexture::value, RtwImage::pixel_data  the_next_week/sphere.rs:46-52, texture.rs:89-109,
//                                                             rtw_image.rs:46-78
//   DiffuseLight::emitted                                     the_next_week/material.rs:116-135
//   Sphere::new_moving / hit at ray time                      the_next_week/sphere.rs:24-45
//   CheckerTexture / NoiseTexture::value                      the_next_week/texture.rs:39-77, 111-126
//   Perlin::noise / turb / perlin_interp                      the_next_week/perlin.rs:25-98
//   write_color (f64 quantiser)                               books/in_one_weekend/color.rs:6-32
//   write_ppm_from_accum (f32 quantiser)                      render_io.rs:3-31
//   build_in_one_weekend_scene (seeded SmallRng scene)        gpu/mod.rs:124-301
//
// Two modes over the same scene and the same per-path random stream:
//   BOOKS (mode 1): T = double, the reference's recursion (ray_color calls itself, the
//          throughput multiplies back-to-front), the reference's BVH tree walked left-first
//          exactly as BvhNode::hit. The books-faithful CPU baseline.
//   TWIN  (mode 0): T = float, every operation in the reference's order, throughput carried
//          front-to-back like the HIP kernel. Its per-pixel f32 sums are the bit-parity target
//          for the GPU (no FP contraction: built with -ffp-contract=off).
// Deliberate restatement choices:
//   * RNG: the reference's thread-local SmallRng::from_entropy (rtweekend.rs:9-11) is not
//     reproducible; both sides use a xoshiro128+ stream per (seed, pixel, sample) instead, and
//     random_double() = (u32 >> 8) * 2^-24 (exact in f32 and f64).
//   * f32 twin: 1e-160 (vec3.rs:185) underflows to 0; transcendentals of sphere UV and the
//     noise texture's sin use the Cephes f32 polynomials the kernel uses (books mode: libm sin;
//     the sphere UV's acos / atan2 are fdlibm's algorithms restated, <= 1 ulp from libm and
//     shared bit for bit with the f64 kernel).
#include "../include/rrt_hip.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <thread>
#include <type_traits>
#include <vector>

namespace {

template <class T>
constexpr T lit(double d, float f) {
    if constexpr (std::is_same_v<T, float>) return f;
    else return (T)d;
}
#define L(x) lit<T>(x, x##f)

// ---- vec3.rs ----------------------------------------------------------------------------
template <class T>
struct Vec3 {
    T e[3];
    T x() const { return e[0]; }
    T y() const { return e[1]; }
    T z() const { return e[2]; }
    T operator[](int i) const { return e[i]; }
};
template <class T> Vec3<T> mk(T a, T b, T c) { return Vec3<T>{{a, b, c}}; }
template <class T> Vec3<T> operator+(Vec3<T> a, Vec3<T> b) { return mk(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
template <class T> Vec3<T> operator-(Vec3<T> a, Vec3<T> b) { return mk(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
template <class T> Vec3<T> operator-(Vec3<T> a) { return mk(-a.e[0], -a.e[1], -a.e[2]); }
template <class T> Vec3<T> operator*(Vec3<T> a, Vec3<T> b) { return mk(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
// vec3.rs:118-132: Vec3 * f64 and f64 * Vec3 both compute e[i] * s
template <class T> Vec3<T> operator*(Vec3<T> a, T s) { return mk(a.e[0] * s, a.e[1] * s, a.e[2] * s); }
template <class T> Vec3<T> operator*(T s, Vec3<T> a) { return a * s; }
// vec3.rs:142-148: Div<f64> is (1.0 / rhs) * self
template <class T> Vec3<T> operator/(Vec3<T> a, T s) { return (T(1) / s) * a; }
// f32 modes (TWIN, KBVH) evaluate dot products and sums of squares the way the kernel does:
// u0*v0, then two fused multiply-adds (one rounding per term instead of two; rrt_kernel.hip dot).
// BOOKS (f64) keeps the reference's unfused (u0*v0 + u1*v1) + u2*v2 (vec3.rs:156-158, Rust
// never contracts).
template <class T> T dot3(T a0, T b0, T a1, T b1, T a2, T b2) {
    if constexpr (std::is_same_v<T, float>) return std::fma(a2, b2, std::fma(a1, b1, a0 * b0));
    else return a0 * b0 + a1 * b1 + a2 * b2;
}
template <class T> T length_squared(Vec3<T> v) { return dot3(v.e[0], v.e[0], v.e[1], v.e[1], v.e[2], v.e[2]); }
template <class T> T length(Vec3<T> v) { return std::sqrt(length_squared(v)); }
template <class T> T dot(Vec3<T> u, Vec3<T> v) { return dot3(u.e[0], v.e[0], u.e[1], v.e[1], u.e[2], v.e[2]); }
// Sphere::hit's discriminant h*h - a*c (sphere.rs:30); f32 modes fuse it like the kernel:
// fma(h, h, -(a*c)).
template <class T> T sphere_disc(T h, T a, T c) {
    if constexpr (std::is_same_v<T, float>) return std::fma(h, h, -(a * c));
    else return h * h - a * c;
}
// Ray::at (ray.rs: orig + t*dir) for the hit record; f32 modes fuse it like the kernel's shading.
template <class T> Vec3<T> ray_at(Vec3<T> o, Vec3<T> d, T t) {
    if constexpr (std::is_same_v<T, float>)
        return mk(std::fma(t, d.e[0], o.e[0]), std::fma(t, d.e[1], o.e[1]), std::fma(t, d.e[2], o.e[2]));
    else return o + t * d;
}
template <class T> Vec3<T> unit_vector(Vec3<T> v) { return v / length(v); }
template <class T> bool near_zero(Vec3<T> v) {  // vec3.rs:38-41
    const T s = L(1e-8);
    return std::fabs(v.e[0]) < s && std::fabs(v.e[1]) < s && std::fabs(v.e[2]) < s;
}
template <class T> Vec3<T> cross(Vec3<T> u, Vec3<T> v) {  // vec3.rs cross
    return mk(u.e[1] * v.e[2] - u.e[2] * v.e[1], u.e[2] * v.e[0] - u.e[0] * v.e[2], u.e[0] * v.e[1] - u.e[1] * v.e[0]);
}
template <class T> Vec3<T> reflect(Vec3<T> v, Vec3<T> n) { return v - T(2) * dot(v, n) * n; }  // vec3.rs:201-203
template <class T> T rmin(T a, T b) { return a < b ? a : b; }  // f64::min with a possibly NaN: returns b
template <class T> Vec3<T> refract(Vec3<T> uv, Vec3<T> n, T etai_over_etat) {  // vec3.rs:205-210
    const T cos_theta = rmin(-dot(uv, n), T(1));
    const Vec3<T> r_out_perp = etai_over_etat * (uv + cos_theta * n);
    const Vec3<T> r_out_parallel = -std::sqrt(std::fabs(T(1) - length_squared(r_out_perp))) * n;
    return r_out_perp + r_out_parallel;
}

// ---- RNG (restatement choice, see header) ---------------------------------------------------
uint64_t splitmix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
struct PathRng {  // xoshiro128+ (the kernel's rng_next, rrt_kernel.hip)
    uint32_t a, b, c, d;
    PathRng(uint64_t z, uint64_t key)
        : a((uint32_t)z), b((uint32_t)(z >> 32)), c((uint32_t)key), d((uint32_t)(key >> 32) | 1u) {}
    uint64_t key() const { return (uint64_t)a | ((uint64_t)b << 32); }
    uint32_t next() {
        const uint32_t r = a + d;
        const uint32_t t = b << 9;
        c ^= a;
        d ^= b;
        b ^= c;
        a ^= d;
        c ^= t;
        d = (d << 11) | (d >> 21);
        return r;
    }
    template <class T> T random_double() { return (T)(next() >> 8) * lit<T>(0x1.0p-24, 0x1.0p-24f); }
    template <class T> T random_double_range(T lo, T hi) { return random_double<T>() * (hi - lo) + lo; }
};

template <class T> Vec3<T> random_unit_vector(PathRng &rng) {  // vec3.rs:181-189
    for (;;) {
        const T a = rng.random_double_range<T>(T(-1), T(1));
        const T b = rng.random_double_range<T>(T(-1), T(1));
        const T c = rng.random_double_range<T>(T(-1), T(1));
        const Vec3<T> p = mk(a, b, c);
        const T lensq = length_squared(p);
        if (L(1e-160) < lensq && lensq <= T(1)) return p / std::sqrt(lensq);
    }
}
template <class T> Vec3<T> random_in_unit_disk(PathRng &rng) {  // vec3.rs:172-179
    for (;;) {
        const T a = rng.random_double_range<T>(T(-1), T(1));
        const T b = rng.random_double_range<T>(T(-1), T(1));
        const Vec3<T> p = mk(a, b, T(0));
        if (length_squared(p) < T(1)) return p;
    }
}

// ---- Cephes f32 acos / atan2 (twin) or fdlibm (books, below) -------------------------------
float asin_core(float x) {
    const float z = x * x;
    return ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z +
            1.6666752422e-1f) * z * x + x;
}
const float kPiF = 3.14159265358979323846f;
float cephes_acosf(float x) {
    if (x < -0.5f) return kPiF - 2.0f * asin_core(std::sqrt(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * asin_core(std::sqrt(0.5f * (1.0f - x)));
    return 1.57079632679489661923f - asin_core(x);
}
float cephes_atanf(float x) {
    float sgn = 1.0f;
    if (x < 0.0f) { sgn = -1.0f; x = -x; }
    float y = 0.0f;
    if (x > 2.414213562373095f) { y = 1.57079632679489661923f; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y = 0.78539816339744830962f; x = (x - 1.0f) / (x + 1.0f); }
    const float z = x * x;
    y = y + ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z * x + x);
    return sgn * y;
}
float cephes_atan2f(float y, float x) {
    if (x == 0.0f) {
        if (y > 0.0f) return 1.57079632679489661923f;
        if (y < 0.0f) return -1.57079632679489661923f;
        return 0.0f;
    }
    float z = cephes_atanf(y / x);
    if (x < 0.0f) z = (y < 0.0f) ? z - kPiF : z + kPiF;
    return z;
}
// ---- f64 acos / atan2 (books): fdlibm's e_acos.c, s_atan.c, e_atan2.c restated ----------------
// The reference's f64::acos / atan2 call the platform libm, whose last-ulp choices this container
// cannot pin against the Rust build. BOOKS uses fdlibm's published algorithms instead (only + - * /
// sqrt and exponent-word tests), the same ones the f64 kernel (rrt_books64.hip) restates, so the two
// agree bit for bit; tests/test_oracle.py bounds the restatement against glibc's libm (<= 1 ulp).
uint32_t fd_hi(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (uint32_t)(b >> 32);
}
uint32_t fd_lo(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    return (uint32_t)b;
}
double fd_with_lo_zero(double x) {
    uint64_t b;
    std::memcpy(&b, &x, 8);
    b &= 0xffffffff00000000ull;
    std::memcpy(&x, &b, 8);
    return x;
}
const double fd_pio2_hi = 1.57079632679489655800e+00, fd_pio2_lo = 6.12323399573676603587e-17;
const double fd_pi = 3.14159265358979311600e+00, fd_pi_lo = 1.2246467991473531772e-16;
double fd_acos_r(double z) {  // p(z) / q(z)
    const double pS0 = 1.66666666666666657415e-01, pS1 = -3.25565818622400915405e-01,
                 pS2 = 2.01212532134862925881e-01, pS3 = -4.00555345006794114027e-02,
                 pS4 = 7.91534994289814532176e-04, pS5 = 3.47933107596021167570e-05;
    const double qS1 = -2.40339491173441421878e+00, qS2 = 2.02094576023350569471e+00,
                 qS3 = -6.88283971605453293030e-01, qS4 = 7.70381505559019352791e-02;
    const double p = z * (pS0 + z * (pS1 + z * (pS2 + z * (pS3 + z * (pS4 + z * pS5)))));
    const double q = 1.0 + z * (qS1 + z * (qS2 + z * (qS3 + z * qS4)));
    return p / q;
}
double fdlibm_acos(double x) {
    const int32_t hx = (int32_t)fd_hi(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x3ff00000) {
        if (((ix - 0x3ff00000) | (int32_t)fd_lo(x)) == 0) return hx > 0 ? 0.0 : fd_pi + 2.0 * fd_pio2_lo;
        return (x - x) / (x - x);
    }
    if (ix < 0x3fe00000) {
        if (ix <= 0x3c600000) return fd_pio2_hi + fd_pio2_lo;
        const double z = x * x;
        const double r = fd_acos_r(z);
        return fd_pio2_hi - (x - (fd_pio2_lo - x * r));
    } else if (hx < 0) {
        const double z = (1.0 + x) * 0.5;
        const double s = std::sqrt(z);
        const double r = fd_acos_r(z);
        const double w = r * s - fd_pio2_lo;
        return fd_pi - 2.0 * (s + w);
    } else {
        const double z = (1.0 - x) * 0.5;
        const double s = std::sqrt(z);
        const double df = fd_with_lo_zero(s);
        const double c = (z - df * df) / (s + df);
        const double r = fd_acos_r(z);
        const double w = r * s + c;
        return 2.0 * (df + w);
    }
}
double fdlibm_atan(double x) {
    static const double atanhi[] = {4.63647609000806093515e-01, 7.85398163397448278999e-01,
                                    9.82793723247329054082e-01, 1.57079632679489655800e+00};
    static const double atanlo[] = {2.26987774529616870924e-17, 3.06161699786838301793e-17,
                                    1.39033110312309984516e-17, 6.12323399573676603587e-17};
    static const double aT[] = {3.33333333333329318027e-01, -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                                -1.11111104054623557880e-01, 9.09088713343650656196e-02, -7.69187620504482999495e-02,
                                6.66107313738753120669e-02, -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                                -3.65315727442169155270e-02, 1.62858201153657823623e-02};
    const int32_t hx = (int32_t)fd_hi(x);
    const int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x44100000) {
        if (ix > 0x7ff00000 || (ix == 0x7ff00000 && fd_lo(x) != 0)) return x + x;
        return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
    }
    if (ix < 0x3fdc0000) {
        if (ix < 0x3e200000) return x;
        id = -1;
    } else {
        x = std::fabs(x);
        if (ix < 0x3ff30000) {
            if (ix < 0x3fe60000) {
                id = 0;
                x = (2.0 * x - 1.0) / (2.0 + x);
            } else {
                id = 1;
                x = (x - 1.0) / (x + 1.0);
            }
        } else {
            if (ix < 0x40038000) {
                id = 2;
                x = (x - 1.5) / (1.0 + 1.5 * x);
            } else {
                id = 3;
                x = -1.0 / x;
            }
        }
    }
    const double z = x * x;
    const double w = z * z;
    const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
    const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
    if (id < 0) return x - x * (s1 + s2);
    const double r = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
    return hx < 0 ? -r : r;
}
double fdlibm_atan2(double y, double x) {
    const int32_t hx = (int32_t)fd_hi(x), hy = (int32_t)fd_hi(y);
    const uint32_t lx = fd_lo(x), ly = fd_lo(y);
    const int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (((uint32_t)ix | ((lx | (0u - lx)) >> 31)) > 0x7ff00000u || ((uint32_t)iy | ((ly | (0u - ly)) >> 31)) > 0x7ff00000u)
        return x + y;
    if ((((uint32_t)hx - 0x3ff00000u) | lx) == 0) return fdlibm_atan(y);
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if ((iy | (int32_t)ly) == 0) {
        switch (m) {
            case 0:
            case 1: return y;
            case 2: return fd_pi;
            default: return -fd_pi;
        }
    }
    if ((ix | (int32_t)lx) == 0) return hy < 0 ? -fd_pio2_hi : fd_pio2_hi;
    if (ix == 0x7ff00000) {
        const double pi_o_4 = 7.8539816339744827900e-01;
        if (iy == 0x7ff00000) {
            const double v[4] = {pi_o_4, -pi_o_4, 3.0 * pi_o_4, -3.0 * pi_o_4};
            return v[m];
        }
        const double v[4] = {0.0, -0.0, fd_pi, -fd_pi};
        return v[m];
    }
    if (iy == 0x7ff00000) return hy < 0 ? -fd_pio2_hi : fd_pio2_hi;
    const int k = (iy - ix) >> 20;
    double z;
    if (k > 60) z = fd_pio2_hi + 0.5 * fd_pi_lo;
    else if (hx < 0 && k < -60) z = 0.0;
    else z = fdlibm_atan(std::fabs(y / x));
    switch (m) {
        case 0: return z;
        case 1: return -z;
        case 2: return fd_pi - (z - fd_pi_lo);
        default: return (z - fd_pi_lo) - fd_pi;
    }
}
template <class T> T t_acos(T x) { if constexpr (std::is_same_v<T, float>) return cephes_acosf(x); else return fdlibm_acos(x); }
template <class T> T t_atan2(T y, T x) { if constexpr (std::is_same_v<T, float>) return cephes_atan2f(y, x); else return fdlibm_atan2(y, x); }
template <class T> T t_pi() { return lit<T>(3.14159265358979323846, 3.14159265358979323846f); }

// ---- interval.rs / aabb.rs -----------------------------------------------------------------
template <class T> struct Interval {
    T min, max;
    T size() const { return max - min; }
    bool surrounds(T x) const { return min < x && x < max; }
    bool contains(T x) const { return min <= x && x <= max; }
    T clamp(T x) const { return x < min ? min : (x > max ? max : x); }
    Interval expand(T delta) const { const T p = delta / T(2); return Interval{min - p, max + p}; }
};
template <class T> Interval<T> iv_union(Interval<T> a, Interval<T> b) {
    return Interval<T>{a.min <= b.min ? a.min : b.min, a.max >= b.max ? a.max : b.max};
}
template <class T> struct Aabb {
    Interval<T> ax[3];
};
template <class T> Aabb<T> pad(Aabb<T> b) {  // aabb.rs:104-115
    const T delta = L(0.0001);
    for (int i = 0; i < 3; ++i)
        if (b.ax[i].size() < delta) b.ax[i] = b.ax[i].expand(delta);
    return b;
}
template <class T> Aabb<T> empty_box() {
    const T inf = std::numeric_limits<T>::infinity();
    return Aabb<T>{{{inf, -inf}, {inf, -inf}, {inf, -inf}}};
}
template <class T> Aabb<T> from_boxes(const Aabb<T> &a, const Aabb<T> &b) {
    return pad(Aabb<T>{{iv_union(a.ax[0], b.ax[0]), iv_union(a.ax[1], b.ax[1]), iv_union(a.ax[2], b.ax[2])}});
}
template <class T> Aabb<T> from_points(Vec3<T> a, Vec3<T> b) {  // aabb.rs:29-34
    Aabb<T> r;
    for (int i = 0; i < 3; ++i) r.ax[i] = a[i] <= b[i] ? Interval<T>{a[i], b[i]} : Interval<T>{b[i], a[i]};
    return pad(r);
}
template <class T> int longest_axis(const Aabb<T> &b) {
    if (b.ax[0].size() > b.ax[1].size()) return b.ax[0].size() > b.ax[2].size() ? 0 : 2;
    return b.ax[1].size() > b.ax[2].size() ? 1 : 2;
}
template <class T> T surface_area(const Aabb<T> &b) {
    const T a = b.ax[0].size(), c = b.ax[1].size(), d = b.ax[2].size();
    return T(2) * (a * c + a * d + c * d);
}
// The slab arithmetic runs in f64 for both arithmetics: a box test only prunes, and in f32 the
// reference's (min - o) * (1/d) loses the 1e-4 padding of a flat box at |o| ~ 1e3 (the Cornell
// walls: 554.99994 + 800 rounds to 1355), rejecting rays that hit the face.
template <class T> bool aabb_hit(const Aabb<T> &box, Vec3<T> o, Vec3<T> d, Interval<T> ray_in) {  // aabb.rs:52-85
    Interval<double> ray_t{(double)ray_in.min, (double)ray_in.max};
    for (int axis = 0; axis < 3; ++axis) {
        const Interval<double> ax{(double)box.ax[axis].min, (double)box.ax[axis].max};
        const double adinv = 1.0 / (double)d[axis];
        const double t0 = (ax.min - (double)o[axis]) * adinv;
        const double t1 = (ax.max - (double)o[axis]) * adinv;
        if (t0 < t1) {
            if (t0 > ray_t.min) ray_t.min = t0;
            if (t1 < ray_t.max) ray_t.max = t1;
        } else {
            if (t1 > ray_t.min) ray_t.min = t1;
            if (t0 < ray_t.max) ray_t.max = t0;
        }
        if (ray_t.max <= ray_t.min) return false;
    }
    return true;
}

// Cephes logf: the kernel's rrt_logf op for op (x > 0 finite or 0).
float cephes_logf(float x) {
    if (x == 0.0f) return -std::numeric_limits<float>::infinity();
    uint32_t b;
    std::memcpy(&b, &x, 4);
    int e = (int)((b >> 23) & 255u) - 126;
    const uint32_t mb = (b & 0x807fffffu) | 0x3f000000u;
    float m;
    std::memcpy(&m, &mb, 4);
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
// Cephes cosf: the kernel's rrt_cosf op for op.
float cephes_cosf(float xx) {
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
float cephes_sinf(float xx);
template <class T> T t_log(T x) { if constexpr (std::is_same_v<T, float>) return cephes_logf(x); else return std::log(x); }

// ---- scene in T ---------------------------------------------------------------------------------
template <class T> struct Sphere {
    Vec3<T> center;  // center1 (Ray origin of the_next_week/sphere.rs:38)
    T radius;
    uint32_t mat;
    Aabb<T> bbox;
    Vec3<T> motion;  // center2 - center1 (zero: static)
    Vec3<T> at(T time) const { return center + time * motion; }  // Ray::at (ray.rs: orig + t*dir)
};
// Quad::new (the_next_week/quad.rs:21-45). The derived plane (normal, D, w) is computed in f64
// from the stored f32 corner and edges and rounded to T, as rrt_host.cpp does for the kernel.
template <class T> struct QuadT {
    Vec3<T> q, u, v, normal, w;
    T D;
    uint32_t mat;
    Aabb<T> bbox;
};
template <class T> QuadT<T> make_quad(const RrtQuad &rq) {
    const Vec3<double> q = mk<double>(rq.q[0], rq.q[1], rq.q[2]), u = mk<double>(rq.u[0], rq.u[1], rq.u[2]),
                       v = mk<double>(rq.v[0], rq.v[1], rq.v[2]);
    const Vec3<double> nv = cross(u, v);
    const Vec3<double> normal = unit_vector(nv);
    const double dd = dot(normal, q);
    const Vec3<double> wv = nv / dot(nv, nv);
    auto cast = [](Vec3<double> a) { return mk<T>((T)a[0], (T)a[1], (T)a[2]); };
    QuadT<T> qd;
    qd.q = cast(q);
    qd.u = cast(u);
    qd.v = cast(v);
    qd.normal = cast(normal);
    qd.w = cast(wv);
    qd.D = (T)dd;
    qd.mat = rq.material_index;
    // set_bounding_box (quad.rs:40-45)
    qd.bbox = from_boxes(from_points(qd.q, qd.q + qd.u + qd.v), from_points(qd.q + qd.u, qd.q + qd.v));
    return qd;
}
// ConstantMedium (the_next_week/constant_medium.rs) over a boundary sphere or boundary quads.
template <class T> struct MediumT {
    uint32_t kind;  // 0 sphere, 1 quads [first, first + count) of World::bquads
    Vec3<T> center;
    T radius;
    uint32_t first, count;
    T neg_inv_density;  // -1/density in f64, rounded to T (constant_medium.rs:24)
    uint32_t mat;
    Aabb<T> bbox;
};
template <class T> struct Material {
    uint32_t kind;
    Vec3<T> albedo;
    T fuzz;   // metal fuzz (clamped <= 1)
    T w;      // albedo_fuzz[3] raw: checker inv_scale, noise scale
    T ref_idx;
    uint32_t tex;
    Vec3<T> odd;  // checker odd colour
};
template <class T> struct PerlinT {  // perlin.rs:4-9
    Vec3<T> randvec[256];
    uint32_t perm_x[256], perm_y[256], perm_z[256];
};
struct Texture {
    const uint8_t *data;
    int32_t width, height;
};

template <class T> struct Hit {
    T t;
    int32_t sphere;
};

// BvhNode per bvh.rs: children are either spheres (>= 0 as ~index? no: tagged) or nodes.
struct ChildRef {
    bool is_sphere;
    int32_t index;
};
template <class T> struct BvhNode {
    ChildRef left, right;
    Aabb<T> bbox;
};

template <class T> struct World {
    std::vector<Sphere<T>> spheres;
    std::vector<QuadT<T>> quads;  // primitive n_spheres + j
    std::vector<MediumT<T>> media;  // primitive n_spheres + n_quads + m
    std::vector<QuadT<T>> bquads;  // media boundaries
    struct LightT {  // book-3 MIS light (RrtLight)
        uint32_t kind;
        Vec3<T> center;
        T radius;
        QuadT<T> quad;
        T area;
    };
    std::vector<LightT> lights;
    std::vector<Material<T>> mats;
    std::vector<Texture> texs;
    std::vector<PerlinT<T>> perlin;
    bool book2 = false;  // moving spheres or checker / noise materials (kernel: kBook2)
    // diagnostic mode bit 0x800 (BOOKS only): the sphere UV's acos / atan2 from this host's libm, as
    // the reference's f64::acos / atan2 compute them, instead of the fdlibm restatement the f64
    // kernel shares (tests/test_gpu_books64.py counts what the difference changes)
    bool libm_trig = false;
    std::vector<BvhNode<T>> nodes;
    ChildRef root{false, -1};
    // f32 modes: the unbounded media's primitive ids, tested after the tree walk (not in the tree;
    // unbounded_media). BOOKS keeps every primitive in its tree (bvh.rs).
    std::vector<int32_t> unbounded;

    ChildRef build(std::vector<int32_t> &objs, size_t lo, size_t hi) {  // bvh.rs:21-156
        const size_t span = hi - lo;
        Aabb<T> bbox = empty_box<T>();
        for (size_t i = lo; i < hi; ++i) bbox = from_boxes(bbox, prim_box(objs[i]));
        const int32_t me = (int32_t)nodes.size();
        nodes.push_back(BvhNode<T>{});
        ChildRef left, right;
        if (span == 1) {
            left = right = ChildRef{true, objs[lo]};
        } else if (span == 2) {
            left = ChildRef{true, objs[lo]};
            right = ChildRef{true, objs[lo + 1]};
        } else {
            const int kBuckets = 12;
            const int axis = longest_axis(bbox);
            auto cmp = [&](int32_t a, int32_t b) { return prim_box(a).ax[axis].min < prim_box(b).ax[axis].min; };
            auto centroid = [&](int32_t o) {
                const Interval<T> iv = prim_box(o).ax[axis];
                return T(0.5) * (iv.min + iv.max);
            };
            T cmin = std::numeric_limits<T>::infinity(), cmax = -std::numeric_limits<T>::infinity();
            for (size_t i = lo; i < hi; ++i) {
                const T c = centroid(objs[i]);
                if (c < cmin) cmin = c;
                if (c > cmax) cmax = c;
            }
            size_t mid;
            bool median = false;
            if (std::fabs(cmax - cmin) < L(1e-12)) {
                median = true;
            } else {
                auto bucket = [&](int32_t o) {
                    size_t idx = (size_t)((centroid(o) - cmin) / (cmax - cmin) * (T)kBuckets);
                    return idx >= (size_t)kBuckets ? (size_t)kBuckets - 1 : idx;
                };
                size_t count[12] = {0};
                Aabb<T> bb[12];
                for (int i = 0; i < kBuckets; ++i) bb[i] = empty_box<T>();
                for (size_t i = lo; i < hi; ++i) {
                    const size_t b = bucket(objs[i]);
                    count[b]++;
                    bb[b] = from_boxes(bb[b], prim_box(objs[i]));
                }
                Aabb<T> rbox[12];
                size_t rcnt[12];
                Aabb<T> acc = empty_box<T>();
                size_t accn = 0;
                for (int i = kBuckets - 1; i >= 0; --i) {
                    accn += count[i];
                    acc = from_boxes(acc, bb[i]);
                    rbox[i] = acc;
                    rcnt[i] = accn;
                }
                Aabb<T> lbox = empty_box<T>();
                size_t lcnt = 0;
                T best = std::numeric_limits<T>::infinity();
                size_t best_split = 0;
                for (int i = 0; i < kBuckets - 1; ++i) {
                    lcnt += count[i];
                    lbox = from_boxes(lbox, bb[i]);
                    if (lcnt == 0 || rcnt[i + 1] == 0) continue;
                    const T cost = surface_area(lbox) * (T)lcnt + surface_area(rbox[i + 1]) * (T)rcnt[i + 1];
                    if (cost < best) {
                        best = cost;
                        best_split = (size_t)i;
                    }
                }
                if (!std::isfinite(best)) {
                    median = true;
                } else {
                    size_t m = 0;
                    for (size_t i = 0; i < span; ++i)
                        if (bucket(objs[lo + i]) <= best_split) std::swap(objs[lo + i], objs[lo + m++]);
                    if (m == 0 || m == span) median = true;
                    else mid = lo + m;
                }
            }
            if (median) {
                std::stable_sort(objs.begin() + lo, objs.begin() + hi, cmp);
                mid = lo + span / 2;
            }
            left = build(objs, lo, mid);
            right = build(objs, mid, hi);
        }
        nodes[me] = BvhNode<T>{left, right, bbox};
        return ChildRef{false, me};
    }

    const Aabb<T> &prim_box(int32_t p) const {
        if ((size_t)p < spheres.size()) return spheres[p].bbox;
        if ((size_t)p < spheres.size() + quads.size()) return quads[p - spheres.size()].bbox;
        return media[p - spheres.size() - quads.size()].bbox;
    }

    // Quad::hit (the_next_week/quad.rs:61-87): t in the closed interval, (alpha, beta) in [0,1]^2.
    bool hit_quad(int32_t j, Vec3<T> o, Vec3<T> d, Interval<T> ray_t, T &t_out, uint64_t *tests) const {
        if (tests) ++*tests;
        return quad_hit(quads[j], o, d, ray_t, t_out);
    }
    static bool quad_hit(const QuadT<T> &qd, Vec3<T> o, Vec3<T> d, Interval<T> ray_t, T &t_out) {
        const T denom = dot(qd.normal, d);
        if (std::fabs(denom) < L(1e-8)) return false;
        const T t = (qd.D - dot(qd.normal, o)) / denom;
        if (!ray_t.contains(t)) return false;
        const Vec3<T> intersection = o + t * d;
        const Vec3<T> planar = intersection - qd.q;
        const T alpha = dot(qd.w, cross(planar, qd.v));
        const T beta = dot(qd.w, cross(qd.u, planar));
        const Interval<T> unit{T(0), T(1)};
        if (!unit.contains(alpha) || !unit.contains(beta)) return false;
        t_out = t;
        return true;
    }

    bool hit_prim(int32_t p, Vec3<T> o, Vec3<T> d, T time, Interval<T> ray_t, T &t_out, uint64_t *tests,
                  uint64_t seg, int32_t skip = -1) const {
        if (p == skip) {  // the primitive the ray is leaving (ray_color_twin): tested, never hit
            if (tests) ++*tests;
            return false;
        }
        if ((size_t)p < spheres.size()) return hit_sphere(p, o, d, time, ray_t, t_out, tests);
        const size_t j = p - spheres.size();
        if (j < quads.size()) return hit_quad((int32_t)j, o, d, ray_t, t_out, tests);
        if (tests) ++*tests;
        return hit_medium((uint32_t)(j - quads.size()), o, d, ray_t, t_out, seg);
    }

    // ConstantMedium::hit (constant_medium.rs:40-84). The boundary's hits over (-inf, inf) and
    // after t1 + 0.0001; the free-flight uniform is the per-(path, segment, medium) draw of
    // include/rrt_hip.h (seg = path RNG state ^ bounce << 32), ln by Cephes logf in f32.
    bool hit_medium(uint32_t m, Vec3<T> o, Vec3<T> d, Interval<T> ray_t, T &t_out, uint64_t seg) const {
        const MediumT<T> &md = media[m];
        const T inf = std::numeric_limits<T>::infinity();
        T t1, t2;
        if (md.kind == RRT_BOUNDARY_SPHERE) {
            if (!sphere_root(md.center, md.radius, o, d, Interval<T>{-inf, inf}, t1)) return false;
            if (!sphere_root(md.center, md.radius, o, d, Interval<T>{t1 + L(0.0001), inf}, t2)) return false;
        } else {
            auto list_hit = [&](Interval<T> iv, T &t_hit) {  // HittableList::hit over the boundary
                bool any = false;
                for (uint32_t k = 0; k < md.count; ++k) {
                    T t;
                    if (quad_hit(bquads[md.first + k], o, d, iv, t)) {
                        any = true;
                        iv.max = t;
                        t_hit = t;
                    }
                }
                return any;
            };
            if (!list_hit(Interval<T>{-inf, inf}, t1)) return false;
            if (!list_hit(Interval<T>{t1 + L(0.0001), inf}, t2)) return false;
        }
        if (t1 < ray_t.min) t1 = ray_t.min;
        if (t2 > ray_t.max) t2 = ray_t.max;
        if (t1 >= t2) return false;
        if (t1 < T(0)) t1 = T(0);
        const T ray_length = length(d);
        const T inside = (t2 - t1) * ray_length;
        const T u = (T)(uint32_t)(splitmix64(seg ^ (uint64_t)m) >> 40) * lit<T>(0x1.0p-24, 0x1.0p-24f);
        const T hit_distance = md.neg_inv_density * t_log<T>(u);
        if (hit_distance > inside) return false;
        t_out = t1 + hit_distance / ray_length;
        return true;
    }

    // Sphere::hit's root selection for a static sphere and an interval.
    static bool sphere_root(Vec3<T> center, T radius, Vec3<T> o, Vec3<T> d, Interval<T> ray_t, T &t_out) {
        const Vec3<T> oc = center - o;
        const T a = length_squared(d);
        const T h = dot(d, oc);
        const T c = length_squared(oc) - radius * radius;
        const T disc = sphere_disc(h, a, c);
        if (disc < T(0)) return false;
        const T sqrtd = std::sqrt(disc);
        T root = (h - sqrtd) / a;
        if (!ray_t.surrounds(root)) {
            root = (h + sqrtd) / a;
            if (!ray_t.surrounds(root)) return false;
        }
        t_out = root;
        return true;
    }

    // Sphere::hit (sphere.rs:24-51): Some(t) iff a root lies in the open interval.
    bool hit_sphere(int32_t i, Vec3<T> o, Vec3<T> d, T time, Interval<T> ray_t, T &t_out, uint64_t *tests) const {
        if (tests) ++*tests;
        const Sphere<T> &s = spheres[i];
        const Vec3<T> oc = (book2 ? s.at(time) : s.center) - o;  // current_center (the_next_week/sphere.rs:44)
        const T a = length_squared(d);
        const T h = dot(d, oc);
        const T c = length_squared(oc) - s.radius * s.radius;
        const T disc = sphere_disc(h, a, c);
        if (disc < T(0)) return false;
        const T sqrtd = std::sqrt(disc);
        T root = (h - sqrtd) / a;
        if (!ray_t.surrounds(root)) {
            root = (h + sqrtd) / a;
            if (!ray_t.surrounds(root)) return false;
        }
        t_out = root;
        return true;
    }

    // HittableObject::hit dispatch + BvhNode::hit (bvh.rs:159-172), left first, right with
    // max = left.t, result = right.or(left).
    bool hit(ChildRef ref, Vec3<T> o, Vec3<T> d, T time, Interval<T> ray_t, Hit<T> &rec, uint64_t *tests,
             uint64_t seg, int32_t skip = -1) const {
        if (ref.is_sphere) {
            T t;
            if (!hit_prim(ref.index, o, d, time, ray_t, t, tests, seg, skip)) return false;
            rec = Hit<T>{t, ref.index};
            return true;
        }
        const BvhNode<T> &n = nodes[ref.index];
        if (!aabb_hit(n.bbox, o, d, ray_t)) return false;
        Hit<T> hl, hr;
        const bool l = hit(n.left, o, d, time, ray_t, hl, tests, seg, skip);
        const bool r = hit(n.right, o, d, time, Interval<T>{ray_t.min, l ? hl.t : ray_t.max}, hr, tests, seg, skip);
        if (r) { rec = hr; return true; }
        if (l) { rec = hl; return true; }
        return false;
    }
};

// ---- KBVH mode: the kernel's own flattened BVH walked in the kernel's order ----------------
// (rustraytrace_amd/csrc/rrt_kernel.hip trav_step / trav_step4; layouts in rrt_internal.h).
// Only IEEE-exact operations (div, fma, min, max) decide the traversal, so the CPU reproduces
// every pruning and ordering decision of the GPU: with it, whole frames are bit-comparable even
// where the closest-hit winner depends on BVH topology (near-ties and grazing rays).
struct KTree {
    uint32_t width = 0;
    uint32_t stride = 0;  // bytes per node: 80 or 32 (BVH2), 128 (BVH4)
    const uint8_t *nodes = nullptr;
    uint32_t n_nodes = 0;
    const uint32_t *order = nullptr;  // leaf-order primitive -> original sphere index
    // the unbounded media (RrtBvhInfo.n_unbounded): the last entries of the leaf order, not in the
    // tree, tested after the walk
    const uint32_t *unbounded = nullptr;
    uint32_t n_unbounded = 0;
};

// 1/d clamped to +-2^64: a zero direction component gives a huge finite slope instead of inf,
// so (P - o) * inv keeps its sign (inf * P - inf * o would be NaN or -inf at a straddling slab)
inline float kclamp_inv(float v) { return std::fmax(std::fmin(v, 0x1.0p64f), -0x1.0p64f); }
struct KRay {
    float ix, iy, iz, oix, oiy, oiz;
};

// IEEE-754 minNum/maxNum (the GPU's v_min_f32 / v_max_f32): a NaN operand yields the other.
// Inline (libm fminf/fmaxf are calls on x86); zero signs may differ but every use compares
// against tmin = 0.001 or orders strictly, so they cannot change a decision.
static inline float min_num(float a, float b) { return (b != b) ? a : ((a != a) ? b : (a < b ? a : b)); }
static inline float max_num(float a, float b) { return (b != b) ? a : ((a != a) ? b : (a > b ? a : b)); }

// IEEE binary16 bits -> float (exact)
static inline float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t b;
    if (e == 0) {
        const float v = std::ldexp((float)m, -24);  // zero or subnormal
        return s ? -v : v;
    }
    b = e == 31 ? (s | 0x7f800000u | (m << 13)) : (s | ((e + 112u) << 23) | (m << 13));
    float out;
    std::memcpy(&out, &b, 4);
    return out;
}

// Kernel slab test (rrt_kernel.hip box_hit). A macro so the FMAs are emitted inside each
// target clone of kbvh_hit (as vfmadd where the host has FMA3, else the libm call).
#define KBOX(lx, hx, ly, hy, lz, hz, r, tmin, tmax, tnear, out)                                                  \
    do {                                                                                                           \
        const float x0_ = __builtin_fmaf(lx, r.ix, -r.oix), x1_ = __builtin_fmaf(hx, r.ix, -r.oix);              \
        const float y0_ = __builtin_fmaf(ly, r.iy, -r.oiy), y1_ = __builtin_fmaf(hy, r.iy, -r.oiy);              \
        const float z0_ = __builtin_fmaf(lz, r.iz, -r.oiz), z1_ = __builtin_fmaf(hz, r.iz, -r.oiz);              \
        const float nr_ = max_num(max_num(min_num(x0_, x1_), min_num(y0_, y1_)),                                 \
                                  max_num(min_num(z0_, z1_), tmin));                                               \
        const float fr_ = min_num(min_num(max_num(x0_, x1_), max_num(y0_, y1_)),                                 \
                                  min_num(max_num(z0_, z1_), tmax));                                               \
        tnear = nr_;                                                                                               \
        out = nr_ < fr_;                                                                                           \
    } while (0)

// std::fmaf is a slow libm call without -mfma: clone the traversal for FMA-capable hosts
// (results are identical either way: fmaf is correctly rounded in both).
__attribute__((target_clones("fma", "default")))
bool kbvh_hit(const World<float> &w, const KTree &kt, Vec3<float> o, Vec3<float> d, float time, Hit<float> &rec,
              uint64_t *tests, uint64_t seg, int32_t skip) {
    KRay r;
    r.ix = kclamp_inv(1.0f / d[0]);  // the kernel's ray_consts
    r.iy = kclamp_inv(1.0f / d[1]);
    r.iz = kclamp_inv(1.0f / d[2]);
    r.oix = o[0] * r.ix;
    r.oiy = o[1] * r.iy;
    r.oiz = o[2] * r.iz;
    const float kTmin = 0.001f;
    float closest = std::numeric_limits<float>::infinity();
    int32_t hit = -1;
    auto leaf = [&](int32_t first, int32_t count) {
        for (int32_t i = first; i < first + count; ++i) {
            float t;
            if (w.hit_prim((int32_t)kt.order[i], o, d, time, Interval<float>{kTmin, closest}, t, tests, seg, skip)) {
                closest = t;
                hit = i;
            }
        }
    };
    int32_t stack[128];
    int sp = 0;
    int32_t node = 0;
    for (;;) {
        if (kt.width == 2) {
            // BVH2 nodes (rrt_internal.h), links = node index, or first | count << 28:
            //   80 B (LDS): per child lo, hi, lo for x, y, z (9 floats), then the two links; the
            //        kernel reads each axis' (entry, exit) pair by the sign of 1/d, which takes
            //        the same decisions as min/max over (lo, hi) here;
            //   32 B (global): per child and axis lo | hi << 16 as f16 bits, then the links
            //        (rrt_internal.h GNodeH); decoded exactly, as the kernel's v_fma_mix_f32 reads them.
            const uint8_t *nb = kt.nodes + (size_t)node * kt.stride;
            const float *f = reinterpret_cast<const float *>(nb);
            const bool ordered = kt.stride == 80;
            float hf[12];
            if (!ordered) {
                const uint32_t *w = reinterpret_cast<const uint32_t *>(nb);
                for (int k = 0; k < 6; ++k) {
                    hf[2 * k] = half_to_float((uint16_t)(w[k] & 0xffffu));
                    hf[2 * k + 1] = half_to_float((uint16_t)(w[k] >> 16));
                }
                f = hf;
            }
            const uint32_t *lk = reinterpret_cast<const uint32_t *>(nb + (ordered ? 72 : 24));
            const int32_t l[4] = {(int32_t)(lk[0] & 0x0fffffffu), (int32_t)(lk[1] & 0x0fffffffu), (int32_t)(lk[0] >> 28),
                                  (int32_t)(lk[1] >> 28)};
            float tn0 = 0.0f, tn1 = 0.0f;
            bool h0, h1;
            if (ordered) {
                KBOX(f[0], f[1], f[3], f[4], f[6], f[7], r, kTmin, closest, tn0, h0);
                KBOX(f[9], f[10], f[12], f[13], f[15], f[16], r, kTmin, closest, tn1, h1);
            } else {  // f16 planes, decoded: c0 lo.x hi.x lo.y hi.y lo.z hi.z, c1 the same
                KBOX(f[0], f[1], f[2], f[3], f[4], f[5], r, kTmin, closest, tn0, h0);
                KBOX(f[6], f[7], f[8], f[9], f[10], f[11], r, kTmin, closest, tn1, h1);
            }
            if (h0 && l[2] > 0) { leaf(l[0], l[2]); h0 = false; }
            if (h1 && l[3] > 0) { leaf(l[1], l[3]); h1 = false; }
            if (h0 && h1) {
                const bool first1 = tn1 < tn0;
                stack[sp++] = first1 ? l[0] : l[1];
                node = first1 ? l[1] : l[0];
                continue;
            }
            if (h0) { node = l[0]; continue; }
            if (h1) { node = l[1]; continue; }
        } else {
            const float *f = reinterpret_cast<const float *>(kt.nodes + (size_t)node * 128);
            const int32_t *child = reinterpret_cast<const int32_t *>(kt.nodes + (size_t)node * 128 + 96);
            const int32_t *count = child + 4;
            const float inf = std::numeric_limits<float>::infinity();
            float key[4];
            int32_t idx[4];
            for (int c = 0; c < 4; ++c) {
                float tn = 0.0f;
                bool h;
                KBOX(f[c], f[4 + c], f[8 + c], f[12 + c], f[16 + c], f[20 + c], r, kTmin, closest, tn, h);
                key[c] = h ? tn : inf;
                idx[c] = child[c];
            }
            for (int c = 0; c < 4; ++c)
                if (count[c] > 0) {
                    if (key[c] < inf) leaf(child[c], count[c]);
                    key[c] = inf;
                }
            for (int c = 0; c < 4; ++c) key[c] = key[c] < closest ? key[c] : inf;
            auto cswap = [&](int i, int j) {
                if (key[j] < key[i]) { std::swap(key[i], key[j]); std::swap(idx[i], idx[j]); }
            };
            cswap(0, 1);
            cswap(2, 3);
            cswap(0, 2);
            cswap(1, 3);
            cswap(1, 2);
            if (key[3] < inf) stack[sp++] = idx[3];
            if (key[2] < inf) stack[sp++] = idx[2];
            if (key[1] < inf) stack[sp++] = idx[1];
            if (key[0] < inf) { node = idx[0]; continue; }
        }
        if (sp == 0) break;
        node = stack[--sp];
    }
    if (hit < 0) return false;
    rec = Hit<float>{closest, (int32_t)kt.order[hit]};
    return true;
}

template <class T> struct Cam {
    Vec3<T> center, p00, du, dv, disk_u, disk_v, background;
    T radius;
    uint32_t max_depth, seed, bg_mode, flags;
    uint32_t width, height;
    uint32_t sqrt_spp = 0;  // book 3: stratified samples
    T recip_sqrt_spp = T(0);
    bool no_exit_skip = false;  // diagnostic mode bit 0x200: f32 modes without exit_skip
};

// The kernel's unbounded media (rrt_host.cpp unbounded_media, restated): in medium order, at most
// 4, each sphere-bounded medium whose box [c - r, c + r] holds every other primitive's extent
// (sphere boxes and the ends of their motion, quad corners q, q + u, q + v, (q + u) + v, the other
// media's boundaries), in f64 from the f32 inputs. A scheduling choice of the kernel (such a
// medium is tested after the BVH walk, its hit unchanged); the f32 modes follow it so that the
// GPU's closest hits stay reproducible bit for bit.
std::vector<uint32_t> unbounded_media(const RrtSphere *s, uint32_t n, const RrtSceneExt *ext) {
    std::vector<uint32_t> out;
    const uint32_t nmd = ext && ext->media ? ext->n_media : 0u;
    const uint32_t nq = ext && ext->quads ? ext->n_quads : 0u;
    const float *motion = ext ? ext->sphere_motion : nullptr;
    for (uint32_t m = 0; m < nmd && out.size() < 4; ++m) {
        const RrtMedium &md = ext->media[m];
        if (md.boundary_kind != RRT_BOUNDARY_SPHERE) continue;
        const double r = std::max((double)md.sphere[3], 0.0);
        double lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = (double)md.sphere[a] - r;
            hi[a] = (double)md.sphere[a] + r;
        }
        bool inside = true;
        auto point = [&](double x, double y, double z, double ext_r) {
            const double v[3] = {x, y, z};
            for (int a = 0; a < 3; ++a)
                if (!(lo[a] <= v[a] - ext_r && v[a] + ext_r <= hi[a])) inside = false;
        };
        auto corners = [&](const RrtQuad &q) {
            point(q.q[0], q.q[1], q.q[2], 0.0);
            point((double)q.q[0] + q.u[0], (double)q.q[1] + q.u[1], (double)q.q[2] + q.u[2], 0.0);
            point((double)q.q[0] + q.v[0], (double)q.q[1] + q.v[1], (double)q.q[2] + q.v[2], 0.0);
            point(((double)q.q[0] + q.u[0]) + q.v[0], ((double)q.q[1] + q.u[1]) + q.v[1],
                  ((double)q.q[2] + q.u[2]) + q.v[2], 0.0);
        };
        for (uint32_t i = 0; i < n; ++i) {
            const float *c = s[i].center_radius;
            const double ri = std::max((double)c[3], 0.0);
            point(c[0], c[1], c[2], ri);
            if (motion) {
                const float *mv = motion + 4 * (size_t)i;
                point((double)(c[0] + mv[0]), (double)(c[1] + mv[1]), (double)(c[2] + mv[2]), ri);
            }
        }
        for (uint32_t j = 0; j < nq; ++j) corners(ext->quads[j]);
        for (uint32_t k = 0; k < nmd; ++k) {
            if (k == m) continue;
            const RrtMedium &o = ext->media[k];
            if (o.boundary_kind == RRT_BOUNDARY_SPHERE)
                point(o.sphere[0], o.sphere[1], o.sphere[2], std::max((double)o.sphere[3], 0.0));
            else
                for (uint32_t q = 0; q < o.count; ++q) corners(ext->boundary_quads[o.first + q]);
        }
        if (inside) out.push_back(m);
    }
    return out;
}

template <class T>
void load_world(World<T> &w, Cam<T> &cam, const RrtCamera *c, const RrtSphere *s, uint32_t n, const RrtMaterial *m,
                uint32_t nm, const RrtTexture *tex, uint32_t ntex, uint32_t flags, const RrtSceneExt *ext,
                bool all_in_tree = false) {
    auto v3 = [](const float *f) { return mk<T>((T)f[0], (T)f[1], (T)f[2]); };
    cam.center = v3(c->origin);
    cam.p00 = v3(c->pixel00);
    cam.du = v3(c->pixel_delta_u);
    cam.dv = v3(c->pixel_delta_v);
    cam.radius = (T)c->params_f[0];
    cam.disk_u = v3(c->u) * cam.radius;  // defocus_disk_u = u * defocus_radius (camera.rs:136-138)
    cam.disk_v = v3(c->v) * cam.radius;
    cam.background = v3(c->background);
    cam.max_depth = c->params_u[0];
    cam.seed = c->params_u[1];
    cam.bg_mode = c->params_u[3];
    cam.flags = flags;
    if (flags & RRT_FLAG_BOOK3) {  // Camera::initialize (the_rest_of_your_life/camera.rs:115-117)
        cam.sqrt_spp = (uint32_t)std::sqrt((double)std::max(c->params_f[3], 1.0f));
        cam.recip_sqrt_spp = (T)(1.0 / (double)cam.sqrt_spp);
    }
    cam.width = (uint32_t)c->params_f[1];
    cam.height = (uint32_t)c->params_f[2];
    const float *motion = ext ? ext->sphere_motion : nullptr;
    w.spheres.resize(n);
    for (uint32_t i = 0; i < n; ++i) {  // Sphere::new / new_moving (sphere.rs:16-21; the_next_week/sphere.rs:14-40)
        const Vec3<T> center = v3(s[i].center_radius);
        const T r = std::max((T)s[i].center_radius[3], T(0));
        const Vec3<T> rvec = mk(r, r, r);
        Sphere<T> sp{center, r, s[i].material_index, from_points(center - rvec, center + rvec), mk(T(0), T(0), T(0))};
        if (motion) {
            sp.motion = v3(motion + 4 * (size_t)i);
            w.book2 = w.book2 || motion[4 * i] != 0.0f || motion[4 * i + 1] != 0.0f || motion[4 * i + 2] != 0.0f;
            const Vec3<T> c2 = mk((T)(s[i].center_radius[0] + motion[4 * i]), (T)(s[i].center_radius[1] + motion[4 * i + 1]),
                                  (T)(s[i].center_radius[2] + motion[4 * i + 2]));
            sp.bbox = from_boxes(sp.bbox, from_points(c2 - rvec, c2 + rvec));
        }
        w.spheres[i] = sp;
    }
    w.mats.resize(nm);
    for (uint32_t i = 0; i < nm; ++i) {
        Material<T> &mm = w.mats[i];
        mm.kind = m[i].kind;
        mm.albedo = v3(m[i].albedo_fuzz);
        const T fuzz = (T)m[i].albedo_fuzz[3];
        mm.w = fuzz;
        mm.fuzz = (mm.kind == RRT_MAT_METAL && !(fuzz < T(1))) ? T(1) : fuzz;  // Metal::new (material.rs:48-50)
        mm.ref_idx = (T)m[i].ref_idx;
        mm.tex = m[i]._pad[0];
        float g, b;
        std::memcpy(&g, &m[i]._pad[0], 4);
        std::memcpy(&b, &m[i]._pad[1], 4);
        mm.odd = mk((T)m[i].ref_idx, (T)g, (T)b);
        if (mm.kind == RRT_MAT_CHECKER_LAMBERTIAN || mm.kind == RRT_MAT_NOISE_LAMBERTIAN) w.book2 = true;
    }
    for (uint32_t i = 0; i < ntex; ++i) w.texs.push_back(Texture{tex[i].rgb8, tex[i].width, tex[i].height});
    const uint32_t nq = ext && ext->quads ? ext->n_quads : 0u;
    for (uint32_t j = 0; j < nq; ++j) {
        w.quads.push_back(make_quad<T>(ext->quads[j]));
        w.book2 = true;
    }
    const uint32_t nbq = ext && ext->boundary_quads ? ext->n_boundary_quads : 0u;
    for (uint32_t j = 0; j < nbq; ++j) w.bquads.push_back(make_quad<T>(ext->boundary_quads[j]));
    const uint32_t nmd = ext && ext->media ? ext->n_media : 0u;
    for (uint32_t k = 0; k < nmd; ++k) {
        const RrtMedium &rm = ext->media[k];
        MediumT<T> md;
        md.kind = rm.boundary_kind;
        md.center = v3(rm.sphere);
        md.radius = std::max((T)rm.sphere[3], T(0));
        md.first = rm.first;
        md.count = rm.count;
        md.neg_inv_density = (T)(-1.0 / (double)rm.density);
        md.mat = rm.material_index;
        if (md.kind == RRT_BOUNDARY_SPHERE) {
            const Vec3<T> rv = mk(md.radius, md.radius, md.radius);
            md.bbox = from_points(md.center - rv, md.center + rv);
        } else {  // HittableList::bounding_box of the boundary faces
            md.bbox = empty_box<T>();
            for (uint32_t q = 0; q < md.count; ++q) md.bbox = from_boxes(md.bbox, w.bquads[md.first + q].bbox);
        }
        w.media.push_back(md);
        w.book2 = true;
    }
    if (ext && ext->perlin)
        for (uint32_t t = 0; t < ext->n_perlin; ++t) {
            PerlinT<T> pt;
            for (int i = 0; i < 256; ++i) {
                pt.randvec[i] = v3(ext->perlin[t].randvec[i]);
                pt.perm_x[i] = ext->perlin[t].perm_x[i] & 255u;
                pt.perm_y[i] = ext->perlin[t].perm_y[i] & 255u;
                pt.perm_z[i] = ext->perlin[t].perm_z[i] & 255u;
            }
            w.perlin.push_back(pt);
        }
    const uint32_t nl = ext && ext->lights ? ext->n_lights : 0u;
    for (uint32_t l = 0; l < nl; ++l) {
        const RrtLight &L = ext->lights[l];
        typename World<T>::LightT lt{};
        lt.kind = L.kind;
        lt.center = v3(L.a);
        lt.radius = std::max((T)L.a[3], T(0));
        if (L.kind == RRT_LIGHT_QUAD) {
            RrtQuad rq{};
            for (int i = 0; i < 3; ++i) rq.q[i] = L.a[i], rq.u[i] = L.u[i], rq.v[i] = L.v[i];
            lt.quad = make_quad<T>(rq);
            const Vec3<double> nv = cross(mk<double>(L.u[0], L.u[1], L.u[2]), mk<double>(L.v[0], L.v[1], L.v[2]));
            lt.area = (T)length(nv);  // quad.rs:28
        }
        w.lights.push_back(lt);
    }
    const uint32_t np = n + nq + nmd;
    std::vector<int32_t> objs;
    std::vector<bool> out_of_tree(np, false);
    if constexpr (std::is_same_v<T, float>)
        for (uint32_t m : all_in_tree ? std::vector<uint32_t>{} : unbounded_media(s, n, ext)) {
            out_of_tree[n + nq + m] = true;
            w.unbounded.push_back((int32_t)(n + nq + m));
        }
    for (uint32_t i = 0; i < np; ++i)
        if (!out_of_tree[i]) objs.push_back((int32_t)i);
    if (!objs.empty()) w.root = w.build(objs, 0, objs.size());
}

template <class T> struct Record {
    Vec3<T> p, normal, outward;
    bool front;
    uint32_t mat;
    int32_t prim;  // the hit primitive (sphere i, quad n_spheres + j, medium n_spheres + n_quads + m)
};

template <class T>
bool world_hit(const World<T> &w, Vec3<T> o, Vec3<T> d, T time, uint64_t seg, Record<T> &rec, uint64_t *tests,
               const KTree *kt = nullptr, int32_t skip = -1) {  // camera.rs:187
    Hit<T> h;
    if constexpr (std::is_same_v<T, float>) {
        bool any;
        if (kt) {
            any = kbvh_hit(w, *kt, o, d, time, h, tests, seg, skip);
        } else {
            any = w.root.index >= 0 &&
                  w.hit(w.root, o, d, time, Interval<T>{L(0.001), std::numeric_limits<T>::infinity()}, h, tests, seg, skip);
        }
        // the unbounded media, after the walk, against its closest hit (the kernel's order)
        const uint32_t nu = kt ? kt->n_unbounded : (uint32_t)w.unbounded.size();
        for (uint32_t g = 0; g < nu; ++g) {
            const int32_t p = kt ? (int32_t)kt->unbounded[g] : w.unbounded[g];
            T t;
            if (w.hit_prim(p, o, d, time, Interval<T>{L(0.001), any ? h.t : std::numeric_limits<T>::infinity()}, t,
                           tests, seg, skip)) {
                h = Hit<T>{t, p};
                any = true;
            }
        }
        if (!any) return false;
    } else {
        if (w.root.index < 0) return false;
        if (!w.hit(w.root, o, d, time, Interval<T>{L(0.001), std::numeric_limits<T>::infinity()}, h, tests, seg))
            return false;
    }
    rec.p = ray_at(o, d, h.t);  // Ray::at
    rec.prim = h.sphere;
    if ((size_t)h.sphere >= w.spheres.size() + w.quads.size()) {  // medium (constant_medium.rs:76-82)
        rec.outward = rec.normal = mk(T(1), T(0), T(0));
        rec.front = true;
        rec.mat = w.media[h.sphere - w.spheres.size() - w.quads.size()].mat;
        return true;
    }
    if ((size_t)h.sphere >= w.spheres.size()) {  // quad (quad.rs:79)
        const QuadT<T> &qd = w.quads[h.sphere - w.spheres.size()];
        rec.outward = qd.normal;
        rec.front = dot(d, rec.outward) < T(0);
        rec.normal = rec.front ? rec.outward : -rec.outward;
        rec.mat = qd.mat;
        return true;
    }
    const Sphere<T> &s = w.spheres[h.sphere];
    const Vec3<T> center = w.book2 ? s.at(time) : s.center;
    rec.outward = (rec.p - center) / s.radius;  // sphere.rs:48 (current_center: the_next_week/sphere.rs:64)
    rec.front = dot(d, rec.outward) < T(0);       // hittable.rs:28-29
    rec.normal = rec.front ? rec.outward : -rec.outward;
    rec.mat = s.mat;
    return true;
}

template <class T>
Vec3<T> texture_value(const World<T> &w, uint32_t tex, Vec3<T> outward) {
    // get_sphere_uv (the_next_week/sphere.rs:46-52)
    T theta, phi;
    if (std::is_same_v<T, double> && w.libm_trig) {
        theta = (T)std::acos((double)-outward.y());
        phi = (T)std::atan2((double)-outward.z(), (double)outward.x()) + t_pi<T>();
    } else {
        theta = t_acos<T>(-outward.y());
        phi = t_atan2<T>(-outward.z(), outward.x()) + t_pi<T>();
    }
    T u = phi / (T(2) * t_pi<T>());
    T v = theta / t_pi<T>();
    const Texture &t = w.texs[tex];
    if (t.height <= 0) return mk(T(0), T(1), T(1));  // texture.rs:91-93
    const Interval<T> unit{T(0), T(1)};
    u = unit.clamp(u);
    v = T(1) - unit.clamp(v);
    auto to_i32 = [](T x) -> int32_t {  // Rust `as i32`: saturating, NaN -> 0
        if (!(x == x)) return 0;
        if (x <= (T)INT32_MIN) return INT32_MIN;
        if (x >= (T)INT32_MAX) return INT32_MAX;
        return (int32_t)x;
    };
    int32_t i = to_i32(u * (T)t.width);
    int32_t j = to_i32(v * (T)t.height);
    auto clampi = [](int32_t x, int32_t lo, int32_t hi) { return x < lo ? lo : (x < hi ? x : hi - 1); };  // rtw_image.rs:51-52, 70-78
    if (!t.data) return mk(T(1), T(0), T(1));  // rtw_image.rs:47-49
    i = clampi(i, 0, t.width);
    j = clampi(j, 0, t.height);
    const uint8_t *px = t.data + ((size_t)j * t.width + i) * 3;
    const T cs = T(1) / T(255);
    return mk(cs * (T)px[0], cs * (T)px[1], cs * (T)px[2]);
}

// ---- book-2 procedural textures (the_next_week/texture.rs:39-77, 111-126; perlin.rs) -------
// f32 twin: Cephes sinf, the kernel's rrt_sinf op for op; f64 books: libm sin.
float cephes_sinf(float xx) {
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
template <class T> T t_sin(T x) { if constexpr (std::is_same_v<T, float>) return cephes_sinf(x); else return std::sin(x); }

template <class T> int32_t floor_as_i32(T x) {  // `x.floor() as i32`: saturating, NaN -> 0
    const T f = std::floor(x);
    if (!(f == f)) return 0;
    if (f <= (T)-2147483648.0) return INT32_MIN;
    if (f >= (T)2147483647.0) return INT32_MAX;
    return (int32_t)f;
}

template <class T> T perlin_noise(const PerlinT<T> &pt, Vec3<T> p) {  // perlin.rs:25-48, 79-98
    const T u = p.x() - std::floor(p.x());
    const T v = p.y() - std::floor(p.y());
    const T w = p.z() - std::floor(p.z());
    const int32_t i = floor_as_i32(p.x()), j = floor_as_i32(p.y()), k = floor_as_i32(p.z());
    const T uu = u * u * (T(3) - T(2) * u);
    const T vv = v * v * (T(3) - T(2) * v);
    const T ww = w * w * (T(3) - T(2) * w);
    T accum = T(0);
    for (int di = 0; di < 2; ++di)
        for (int dj = 0; dj < 2; ++dj)
            for (int dk = 0; dk < 2; ++dk) {
                const uint32_t idx = pt.perm_x[(uint32_t)(i + di) & 255u] ^ pt.perm_y[(uint32_t)(j + dj) & 255u] ^
                                     pt.perm_z[(uint32_t)(k + dk) & 255u];
                const Vec3<T> c = pt.randvec[idx];
                const Vec3<T> wv = mk(u - (T)di, v - (T)dj, w - (T)dk);
                const T fi = (T)di * uu + (T(1) - (T)di) * (T(1) - uu);
                const T fj = (T)dj * vv + (T(1) - (T)dj) * (T(1) - vv);
                const T fk = (T)dk * ww + (T(1) - (T)dk) * (T(1) - ww);
                accum += fi * fj * fk * dot(c, wv);
            }
    return accum;
}

template <class T> T noise_value(const PerlinT<T> &pt, T scale, Vec3<T> p) {  // texture.rs:122-126, perlin.rs:50-62
    T accum = T(0), weight = T(1);
    Vec3<T> tp = p;
    for (int o = 0; o < 7; ++o) {
        accum += weight * perlin_noise(pt, tp);
        weight *= L(0.5);
        tp = tp * T(2);
    }
    const T turb = std::fabs(accum);
    return L(0.5) * (T(1) + t_sin<T>(scale * p.z() + T(10) * turb));
}

template <class T> bool checker_even(T inv_scale, Vec3<T> p) {  // texture.rs:66-77
    const int32_t x = floor_as_i32(inv_scale * p.x()), y = floor_as_i32(inv_scale * p.y()), z = floor_as_i32(inv_scale * p.z());
    const int32_t sum = (int32_t)((uint32_t)x + (uint32_t)y + (uint32_t)z);
    return sum % 2 == 0;
}

// Material::scatter (material.rs:28-102; book 2 material.rs:41-53). Returns false for None.
template <class T>
bool scatter(const World<T> &w, PathRng &rng, Vec3<T> d_in, const Record<T> &rec, Vec3<T> &att, Vec3<T> &dir) {
    const Material<T> &m = w.mats[rec.mat];
    switch (m.kind) {
        case RRT_MAT_LAMBERTIAN:
        case RRT_MAT_TEXTURED_LAMBERTIAN:
        case RRT_MAT_CHECKER_LAMBERTIAN:
        case RRT_MAT_NOISE_LAMBERTIAN: {
            Vec3<T> sd = rec.normal + random_unit_vector<T>(rng);
            if (near_zero(sd)) sd = rec.normal;
            dir = sd;
            if (m.kind == RRT_MAT_TEXTURED_LAMBERTIAN) att = texture_value(w, m.tex, rec.outward);
            else if (m.kind == RRT_MAT_CHECKER_LAMBERTIAN) att = checker_even(m.w, rec.p) ? m.albedo : m.odd;
            else if (m.kind == RRT_MAT_NOISE_LAMBERTIAN) {
                const T g = noise_value(w.perlin[m.tex], m.w, rec.p);
                att = mk(g, g, g);
            } else att = m.albedo;
            return true;
        }
        case RRT_MAT_METAL: {
            Vec3<T> reflected = reflect(d_in, rec.normal);
            reflected = unit_vector(reflected) + m.fuzz * random_unit_vector<T>(rng);
            dir = reflected;
            att = m.albedo;
            return dot(dir, rec.normal) > T(0);
        }
        case RRT_MAT_DIELECTRIC: {
            att = mk(T(1), T(1), T(1));
            const T ri = rec.front ? T(1) / m.ref_idx : m.ref_idx;
            const Vec3<T> ud = unit_vector(d_in);
            const T cos_theta = rmin(-dot(ud, rec.normal), T(1));
            const T sin_theta = std::sqrt(T(1) - cos_theta * cos_theta);
            const bool cannot = ri * sin_theta > T(1);
            // reflectance (material.rs:75-80): powi(5) == x * ((x*x)*(x*x))
            auto reflectance = [&](T cosine, T rix) {
                T r0 = (T(1) - rix) / (T(1) + rix);
                r0 = r0 * r0;
                const T x = T(1) - cosine;
                const T x2 = x * x;
                const T x4 = x2 * x2;
                return r0 + (T(1) - r0) * (x * x4);
            };
            if (cannot || reflectance(cos_theta, ri) > rng.random_double<T>()) dir = reflect(ud, rec.normal);
            else dir = refract(ud, rec.normal, ri);
            return true;
        }
        case RRT_MAT_ISOTROPIC:  // material.rs:153-158
            dir = random_unit_vector<T>(rng);
            att = m.albedo;
            return true;
        default:  // DiffuseLight: scatter -> None
            return false;
    }
}

template <class T> Vec3<T> emitted(const World<T> &w, const Record<T> &rec) {
    const Material<T> &m = w.mats[rec.mat];
    return m.kind == RRT_MAT_DIFFUSE_LIGHT ? m.albedo : mk(T(0), T(0), T(0));
}

template <class T> Vec3<T> miss_color(const Cam<T> &cam, Vec3<T> d) {
    if (cam.bg_mode == 1u) return cam.background;  // book-2 background / reference GPU bg_mode
    const Vec3<T> ud = unit_vector(d);             // camera.rs:206-208
    const T a = L(0.5) * (ud.y() + T(1));
    return (T(1) - a) * mk(T(1), T(1), T(1)) + a * mk(L(0.5), L(0.7), T(1));
}

template <class T> T rr_probability(Vec3<T> att) {  // camera.rs:191-195
    T p = att.x();
    if (att.y() > p) p = att.y();
    if (att.z() > p) p = att.z();
    if (p < L(0.05)) p = L(0.05);
    if (p > L(0.95)) p = L(0.95);
    return p;
}

struct Tally {
    uint64_t rays = 0, tests = 0;
};

// The primitive a scattered ray cannot hit again in exact arithmetic, skipped by the f32 modes'
// (and the kernel's) next closest-hit query: the sphere it leaves outward (a sphere is convex:
// a ray from its surface with d.n_out > 0 meets it only at t = 0), or the quad it leaves (a
// plane is met once). In f32 the rounded hit point lies up to ~ulp(|center|) off the surface,
// and |oc|^2 - r^2 cancels two ~|oc|^2 values (r = 1000 ground sphere: ulp 0.0625), so a
// grazing ray would re-hit the surface it leaves past tmin = 0.001 and get trapped inside the
// ground sphere; the f64 reference never does. -1: a medium, or a ray entering / staying
// inside a sphere (it must meet that sphere again: refraction, internal reflection).
template <class T> int32_t exit_skip(const World<T> &w, const Cam<T> &cam, const Record<T> &rec, Vec3<T> dir) {
    if (cam.no_exit_skip) return -1;
    if ((size_t)rec.prim >= w.spheres.size() + w.quads.size()) return -1;  // medium
    if ((size_t)rec.prim >= w.spheres.size()) return rec.prim;            // quad
    const bool same_side = dot(dir, rec.normal) > T(0);  // rec.normal faces the incoming ray
    return same_side == rec.front ? rec.prim : -1;
}

// BOOKS: Camera::ray_color (camera.rs:182-209 / the_next_week/camera.rs:174-201), recursive.
template <class T>
Vec3<T> ray_color_books(const World<T> &w, const Cam<T> &cam, PathRng &rng, Vec3<T> o, Vec3<T> d, T time, int depth,
                        Tally &tl) {
    if (depth <= 0) return mk(T(0), T(0), T(0));
    tl.rays++;
    Record<T> rec;
    if (!world_hit(w, o, d, time, rng.key() ^ ((uint64_t)(cam.max_depth - depth) << 32), rec, &tl.tests))
        return miss_color(cam, d);
    const Vec3<T> em = emitted(w, rec);
    Vec3<T> att, dir;
    if (!scatter(w, rng, d, rec, att, dir)) return em;
    const int bounces = (int)cam.max_depth - depth;
    if (bounces >= 5) {
        const T p = rr_probability(att);
        if (rng.random_double<T>() > p) return em;
        return em + att * ray_color_books(w, cam, rng, rec.p, dir, time, depth - 1, tl) / p;
    }
    return em + att * ray_color_books(w, cam, rng, rec.p, dir, time, depth - 1, tl);
}

// TWIN: the same path, throughput front-to-back (the HIP kernel's order, rrt_kernel.hip).
template <class T>
Vec3<T> ray_color_twin(const World<T> &w, const Cam<T> &cam, PathRng &rng, Vec3<T> o, Vec3<T> d, T time, Tally &tl,
                       const KTree *kt = nullptr) {
    Vec3<T> Tp = mk(T(1), T(1), T(1)), Lp = mk(T(0), T(0), T(0));
    int32_t skip = -1;
    for (uint32_t k = 0; k < cam.max_depth; ++k) {
        tl.rays++;
        Record<T> rec;
        if (!world_hit(w, o, d, time, rng.key() ^ ((uint64_t)k << 32), rec, &tl.tests, kt, skip))
            return Lp + Tp * miss_color(cam, d);
        const Material<T> &m = w.mats[rec.mat];
        if (m.kind == RRT_MAT_DIFFUSE_LIGHT) return Lp + Tp * m.albedo;
        Vec3<T> att, dir;
        if (!scatter(w, rng, d, rec, att, dir)) return Lp;
        if (k >= 5u) {
            const T p = rr_probability(att);
            if (rng.random_double<T>() > p) return Lp;
            Tp = (Tp * att) * (T(1) / p);
        } else {
            Tp = Tp * att;
        }
        o = rec.p;
        d = dir;
        skip = exit_skip(w, cam, rec, dir);
    }
    return Lp;
}

// ---- book 3 (the_rest_of_your_life): pdf.rs, onb.rs, quad.rs / sphere.rs pdf_value and random ----
template <class T> T t_cos(T x) { if constexpr (std::is_same_v<T, float>) return cephes_cosf(x); else return std::cos(x); }
template <class T> T t_sin3(T x) { if constexpr (std::is_same_v<T, float>) return cephes_sinf(x); else return std::sin(x); }

template <class T> Vec3<T> onb_transform(Vec3<T> n, Vec3<T> a) {  // Onb::new(n).transform(a)
    const Vec3<T> w = unit_vector(n);
    const Vec3<T> ax = std::fabs(w[0]) > L(0.9) ? mk(T(0), T(1), T(0)) : mk(T(1), T(0), T(0));
    const Vec3<T> v = unit_vector(cross(w, ax));
    const Vec3<T> u = cross(w, v);
    return a[0] * u + a[1] * v + a[2] * w;
}

// HittableList::pdf_value over the light list (hittable_list.rs:60-69)
template <class T> T lights_pdf(const World<T> &w, Vec3<T> o, Vec3<T> d) {
    const T inf = std::numeric_limits<T>::infinity();
    const T weight = T(1) / (T)w.lights.size();
    T sum = T(0);
    for (const auto &lt : w.lights) {
        T pdf = T(0), t;
        if (lt.kind == RRT_LIGHT_QUAD) {  // quad.rs:93-102
            if (World<T>::quad_hit(lt.quad, o, d, Interval<T>{L(0.001), inf}, t)) {
                const T dist2 = t * t * length_squared(d);
                const T cosine = std::fabs(dot(d, lt.quad.normal)) / length(d);
                pdf = dist2 / (cosine * lt.area);
            }
        } else if (World<T>::sphere_root(lt.center, lt.radius, o, d, Interval<T>{L(0.001), inf}, t)) {  // sphere.rs:102-115
            const T dist2 = length_squared(lt.center - o);
            const T cos_max = std::sqrt(T(1) - lt.radius * lt.radius / dist2);
            pdf = T(1) / ((T(2) * t_pi<T>()) * (T(1) - cos_max));
        }
        sum = sum + weight * pdf;
    }
    return sum;
}

// HittableList::random (hittable_list.rs:71-75) + Quad::random / Sphere::random
template <class T> Vec3<T> lights_random(const World<T> &w, Vec3<T> o, PathRng &rng) {
    const int idx = (int)rng.random_double_range<T>(T(0), (T)w.lights.size());
    const auto &lt = w.lights[idx];
    if (lt.kind == RRT_LIGHT_QUAD) {
        const T r1 = rng.random_double<T>();
        const Vec3<T> a = lt.quad.q + r1 * lt.quad.u;
        const T r2 = rng.random_double<T>();
        return (a + r2 * lt.quad.v) - o;
    }
    const Vec3<T> dir = lt.center - o;
    const T d2 = length_squared(dir);
    const T r1 = rng.random_double<T>(), r2 = rng.random_double<T>();
    const T z = T(1) + r2 * (std::sqrt(T(1) - lt.radius * lt.radius / d2) - T(1));
    const T phi = (T(2) * t_pi<T>()) * r1;
    const T sxy = std::sqrt(T(1) - z * z);
    return onb_transform(dir, mk(t_cos(phi) * sxy, t_sin3(phi) * sxy, z));
}

// The attenuation of a pdf-sampled material (Lambertian textures / Isotropic albedo).
template <class T> Vec3<T> b3_attenuation(const World<T> &w, const Material<T> &m, const Record<T> &rec) {
    if (m.kind == RRT_MAT_TEXTURED_LAMBERTIAN) return texture_value(w, m.tex, rec.outward);
    if (m.kind == RRT_MAT_CHECKER_LAMBERTIAN) return checker_even(m.w, rec.p) ? m.albedo : m.odd;
    if (m.kind == RRT_MAT_NOISE_LAMBERTIAN) {
        const T g = noise_value(w.perlin[m.tex], m.w, rec.p);
        return mk(g, g, g);
    }
    return m.albedo;
}

// Mixture sample + pdf + scattering pdf of a Lambertian / Isotropic hit (camera.rs:226-248).
// Returns false when pdf_value <= 0 (the path ends with `emitted`).
template <class T>
bool b3_sample(const World<T> &w, PathRng &rng, const Record<T> &rec, bool iso, Vec3<T> &dir, T &pdf, T &spdf) {
    const T inv4pi = T(1) / (T(4) * t_pi<T>());
    if (rng.random_double<T>() < L(0.5)) {
        dir = lights_random(w, rec.p, rng);
    } else if (iso) {
        dir = random_unit_vector<T>(rng);
    } else {  // random_cosine_direction (vec3.rs:212-222)
        const T r1 = rng.random_double<T>(), r2 = rng.random_double<T>();
        const T phi = (T(2) * t_pi<T>()) * r1;
        const T sr2 = std::sqrt(r2);
        dir = onb_transform(rec.normal, mk(t_cos(phi) * sr2, t_sin3(phi) * sr2, std::sqrt(T(1) - r2)));
    }
    T mat_pdf;
    if (iso) {
        mat_pdf = inv4pi;
    } else {
        const T cosine = dot(unit_vector(dir), unit_vector(rec.normal));
        mat_pdf = cosine <= T(0) ? T(0) : cosine / t_pi<T>();
    }
    pdf = L(0.5) * lights_pdf(w, rec.p, dir) + L(0.5) * mat_pdf;
    if (pdf <= T(0)) return false;
    if (iso) {
        spdf = inv4pi;
    } else {
        const T cosine = dot(rec.normal, unit_vector(dir));
        spdf = cosine < T(0) ? T(0) : cosine / t_pi<T>();
    }
    return true;
}

// Book-3 metal (no absorption test) / dielectric scatter.
template <class T> void b3_skip_scatter(const Material<T> &m, PathRng &rng, Vec3<T> d_in, const Record<T> &rec,
                                        Vec3<T> &att, Vec3<T> &dir) {
    if (m.kind == RRT_MAT_METAL) {
        const Vec3<T> r = random_unit_vector<T>(rng);
        dir = unit_vector(reflect(d_in, rec.normal)) + m.fuzz * r;
        att = m.albedo;
        return;
    }
    att = mk(T(1), T(1), T(1));
    const T ri = rec.front ? T(1) / m.ref_idx : m.ref_idx;
    const Vec3<T> ud = unit_vector(d_in);
    const T cos_theta = rmin(-dot(ud, rec.normal), T(1));
    const T sin_theta = std::sqrt(T(1) - cos_theta * cos_theta);
    const bool cannot = ri * sin_theta > T(1);
    T r0 = (T(1) - ri) / (T(1) + ri);
    r0 = r0 * r0;
    const T x = T(1) - cos_theta;
    const T x2 = x * x;
    const T x4 = x2 * x2;
    const T refl = r0 + (T(1) - r0) * (x * x4);
    if (cannot || refl > rng.random_double<T>()) dir = reflect(ud, rec.normal);
    else dir = refract(ud, rec.normal, ri);
}

// BOOKS, book 3: the_rest_of_your_life/camera.rs:184-254, recursive, f64.
template <class T>
Vec3<T> ray_color_b3_books(const World<T> &w, const Cam<T> &cam, PathRng &rng, Vec3<T> o, Vec3<T> d, T time,
                           int depth, Tally &tl) {
    if (depth <= 0) return mk(T(0), T(0), T(0));
    tl.rays++;
    Record<T> rec;
    if (!world_hit(w, o, d, time, rng.key() ^ ((uint64_t)(cam.max_depth - depth) << 32), rec, &tl.tests))
        return cam.background;
    const Material<T> &m = w.mats[rec.mat];
    if (m.kind == RRT_MAT_DIFFUSE_LIGHT) return rec.front ? m.albedo : mk(T(0), T(0), T(0));
    const int bounces = (int)cam.max_depth - depth;
    if (m.kind == RRT_MAT_METAL || m.kind == RRT_MAT_DIELECTRIC) {
        Vec3<T> att, dir;
        b3_skip_scatter(m, rng, d, rec, att, dir);
        if (bounces >= 5) {
            const T p = rr_probability(att);
            if (rng.random_double<T>() > p) return mk(T(0), T(0), T(0));
            return att * ray_color_b3_books(w, cam, rng, rec.p, dir, time, depth - 1, tl) / p;
        }
        return att * ray_color_b3_books(w, cam, rng, rec.p, dir, time, depth - 1, tl);
    }
    const Vec3<T> att = b3_attenuation(w, m, rec);
    const T rr = bounces >= 5 ? rr_probability(att) : T(1);
    if (rr < T(1) && rng.random_double<T>() > rr) return mk(T(0), T(0), T(0));
    Vec3<T> dir;
    T pdf, spdf;
    if (!b3_sample(w, rng, rec, m.kind == RRT_MAT_ISOTROPIC, dir, pdf, spdf)) return mk(T(0), T(0), T(0));
    const Vec3<T> sample = ray_color_b3_books(w, cam, rng, rec.p, dir, time, depth - 1, tl);
    return ((att * spdf) * sample) / (pdf * rr);
}

// TWIN, book 3: the kernel's shade_b3 (throughput form), f32.
template <class T>
Vec3<T> ray_color_b3_twin(const World<T> &w, const Cam<T> &cam, PathRng &rng, Vec3<T> o, Vec3<T> d, T time, Tally &tl,
                          const KTree *kt = nullptr) {
    Vec3<T> Tp = mk(T(1), T(1), T(1)), Lp = mk(T(0), T(0), T(0));
    int32_t skip = -1;
    for (uint32_t k = 0; k < cam.max_depth; ++k) {
        tl.rays++;
        Record<T> rec;
        if (!world_hit(w, o, d, time, rng.key() ^ ((uint64_t)k << 32), rec, &tl.tests, kt, skip))
            return Lp + Tp * cam.background;
        const Material<T> &m = w.mats[rec.mat];
        if (m.kind == RRT_MAT_DIFFUSE_LIGHT) return rec.front ? Lp + Tp * m.albedo : Lp;
        Vec3<T> att, dir;
        if (m.kind == RRT_MAT_METAL || m.kind == RRT_MAT_DIELECTRIC) {
            b3_skip_scatter(m, rng, d, rec, att, dir);
            if (k >= 5u) {
                const T p = rr_probability(att);
                if (rng.random_double<T>() > p) return Lp;
                Tp = (Tp * att) * (T(1) / p);
            } else {
                Tp = Tp * att;
            }
        } else {
            att = b3_attenuation(w, m, rec);
            T rr = T(1);
            if (k >= 5u) {
                rr = rr_probability(att);
                if (rr < T(1) && rng.random_double<T>() > rr) return Lp;
            }
            T pdf, spdf;
            if (!b3_sample(w, rng, rec, m.kind == RRT_MAT_ISOTROPIC, dir, pdf, spdf)) return Lp;
            Tp = Tp * ((att * spdf) * (T(1) / (pdf * rr)));
        }
        o = rec.p;
        d = dir;
        skip = exit_skip(w, cam, rec, dir);
    }
    return Lp;
}

// Camera::get_ray (camera.rs:152-169, the_next_week/camera.rs:148-163)
template <class T>
void get_ray(const Cam<T> &cam, PathRng &rng, uint32_t i, uint32_t j, uint32_t s, Vec3<T> &o, Vec3<T> &d, T &time) {
    T ox, oy;
    if (cam.flags & RRT_FLAG_BOOK3) {  // sample_square_stratified (the_rest_of_your_life/camera.rs:173-177)
        const uint32_t sj = s / cam.sqrt_spp, si = s - sj * cam.sqrt_spp;
        ox = (((T)si + rng.random_double<T>()) * cam.recip_sqrt_spp) - L(0.5);
        oy = (((T)sj + rng.random_double<T>()) * cam.recip_sqrt_spp) - L(0.5);
    } else {
        ox = rng.random_double<T>() - L(0.5);
        oy = rng.random_double<T>() - L(0.5);
    }
    const Vec3<T> pixel_sample = cam.p00 + ((T)i + ox) * cam.du + ((T)j + oy) * cam.dv;
    if (cam.radius <= T(0)) {
        o = cam.center;
    } else {
        const Vec3<T> p = random_in_unit_disk<T>(rng);
        o = cam.center + (p[0] * cam.disk_u) + (p[1] * cam.disk_v);
    }
    d = pixel_sample - o;
    time = T(0);
    if (cam.flags & RRT_FLAG_RAY_TIME) time = rng.random_double<T>();  // the_next_week/camera.rs:160
}

template <class T>
int render(const RrtCamera *c, const RrtSphere *s, uint32_t n, const RrtMaterial *m, uint32_t nm, const RrtTexture *tex,
           uint32_t ntex, const RrtSceneExt *ext, uint32_t flags, int mode, uint32_t y0, uint32_t y1, uint32_t s0,
           uint32_t s1, int threads, double *accum, uint64_t *rays_out, uint64_t *tests_out, uint32_t chunk,
           const KTree *kt = nullptr) {
    World<T> w;
    Cam<T> cam;
    // diagnostic mode bit 0x400: the f32 TWIN tree keeps the unbounded media (tests: the scheduling
    // choice of testing them after the walk does not change the image)
    load_world(w, cam, c, s, n, m, nm, tex, ntex, flags, ext, (mode & 0x400) != 0);
    cam.no_exit_skip = (mode & 0x200) != 0;
    w.libm_trig = (mode & 0x800) != 0;
    if (y1 > cam.height) y1 = cam.height;
    if (y0 > y1) return -1;
    std::atomic<uint32_t> next_row{y0};
    std::atomic<uint64_t> rays{0}, tests{0};
    auto worker = [&]() {
        Tally tl;
        for (;;) {
            const uint32_t j = next_row.fetch_add(1);  // rayon-like dynamic row scheduling (camera.rs:66-88)
            if (j >= y1) break;
            for (uint32_t i = 0; i < cam.width; ++i) {
                const uint32_t pixel = j * cam.width + i;
                const uint64_t key = splitmix64(((uint64_t)cam.seed << 32) ^ (uint64_t)pixel);
                const uint64_t rays_before = tl.rays;
                // accum order of the kernel (rrt_accum_chunk, include/rrt_hip.h): in-order sums
                // over chunks from s0 — (S-1)/K chunks of K samples, then chunks of max(1, K/4)
                // (max(1, K/8) when S <= K0/4) for the rest (chunk 0 = one chunk) — chunk sums added
                // in order
                Vec3<T> sum = mk(T(0), T(0), T(0));
                const uint32_t S = s1 - s0;
                // the frame's chunk: K0 = chunk halved while S <= 2K, down to K0/4 (rrt_accum_chunk,
                // include/rrt_hip.h; rrt_host.cpp)
                uint32_t big = chunk ? chunk : (S ? S : 1);
                while (chunk && big > std::max(1u, chunk / 4u) && S <= 2u * big) big /= 2u;
                const uint32_t small = chunk ? std::max(1u, big / (S <= chunk / 4u ? 8u : 4u)) : big;
                const uint32_t nb = (chunk && S > big) ? (S - 1u) / big : 0u;
                for (uint32_t c0 = s0; c0 < s1;) {
                    const uint32_t step = (c0 - s0) < nb * big ? big : small;
                    Vec3<T> csum = mk(T(0), T(0), T(0));
                    for (uint32_t sidx = c0; sidx < std::min(s1, c0 + step); ++sidx) {
                        PathRng rng(splitmix64(key + sidx), key);
                        Vec3<T> o, d;
                        T time;
                        get_ray(cam, rng, i, j, sidx, o, d, time);
                        Vec3<T> c;
                        if (cam.flags & RRT_FLAG_BOOK3)
                            c = (mode & 0xff) == 1 ? ray_color_b3_books(w, cam, rng, o, d, time, (int)cam.max_depth, tl)
                                                   : ray_color_b3_twin(w, cam, rng, o, d, time, tl, kt);
                        else
                            c = (mode & 0xff) == 1 ? ray_color_books(w, cam, rng, o, d, time, (int)cam.max_depth, tl)
                                                   : ray_color_twin(w, cam, rng, o, d, time, tl, kt);
                        csum = csum + c;
                    }
                    sum = (c0 == s0) ? csum : sum + csum;
                    c0 += step;
                }
                double *px = accum + ((size_t)(j - y0) * cam.width + i) * 4;
                px[0] = (double)sum.x();
                px[1] = (double)sum.y();
                px[2] = (double)sum.z();
                // diagnostic mode bit 0x100: w = closest-hit queries of this pixel instead of the count
                px[3] = (mode & 0x100) ? (double)(tl.rays - rays_before) : (double)(s1 - s0);
            }
        }
        rays += tl.rays;
        tests += tl.tests;
    };
    if (threads <= 1) {
        worker();
    } else {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(worker);
        for (auto &t : th) t.join();
    }
    if (rays_out) *rays_out = rays.load();
    if (tests_out) *tests_out = tests.load();
    return 0;
}

// ---- gpu::build_in_one_weekend_scene restated (gpu/mod.rs:199-298 draw order) -------------------
struct Xoshiro256pp {
    uint64_t s[4];
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    explicit Xoshiro256pp(uint64_t seed) {  // SeedableRng::seed_from_u64 via SplitMix64
        for (int i = 0; i < 4; ++i) {
            seed += 0x9e3779b97f4a7c15ull;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            s[i] = z ^ (z >> 31);
        }
    }
    uint64_t next_u64() {
        const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0];
        s[3] ^= s[1];
        s[1] ^= s[2];
        s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    uint32_t next_u32() { return (uint32_t)(next_u64() >> 32); }
};

}  // namespace

extern "C" {

// mode 0 = TWIN (f32, kernel order), 1 = BOOKS (f64, recursive). Renders rows [y0,y1),
// chunk = the accum summation chunk (rrt_accum_chunk; 0 = one chunk),
// samples [s0,s1) into accum[(y1-y0)*W*4] (double; TWIN values are exact f32 sums).
int oracle_render(const RrtCamera *cam, const RrtSphere *s, uint32_t n, const RrtMaterial *m, uint32_t nm,
                  const RrtTexture *tex, uint32_t ntex, const RrtSceneExt *ext, uint32_t flags, int mode, uint32_t y0,
                  uint32_t y1, uint32_t s0, uint32_t s1, int threads, double *accum, uint64_t *rays,
                  uint64_t *sphere_tests, uint32_t chunk) {
    if (!cam || !accum) return -1;
    if ((mode & 0xff) == 1)
        return render<double>(cam, s, n, m, nm, tex, ntex, ext, flags, mode, y0, y1, s0, s1, threads, accum, rays,
                              sphere_tests, chunk);
    return render<float>(cam, s, n, m, nm, tex, ntex, ext, flags, mode & ~0xff, y0, y1, s0, s1, threads, accum, rays,
                         sphere_tests, chunk);
}

// mode 2 = KBVH: TWIN arithmetic, but closest hits found by walking the kernel's BVH
// (rrt_build_bvh output: `nodes` of n_nodes x node_stride B (80 or 32: BVH2, 128: BVH4), `order`).
int oracle_render_kbvh(const RrtCamera *cam, const RrtSphere *s, uint32_t n, const RrtMaterial *m, uint32_t nm,
                       const RrtTexture *tex, uint32_t ntex, const RrtSceneExt *ext, uint32_t flags, const void *nodes,
                       uint32_t n_nodes,
                       uint32_t width, const uint32_t *order, uint32_t n_unbounded, uint32_t y0, uint32_t y1,
                       uint32_t s0, uint32_t s1, int threads, double *accum, uint64_t *rays, uint64_t *sphere_tests,
                       uint32_t chunk) {
    // `width` is the node stride in bytes: 80 / 32 (BVH2 layouts), 128 (BVH4)
    if (!cam || !accum || !nodes || (width != 32 && width != 80 && width != 128)) return -1;
    const uint32_t np = n + (ext && ext->quads ? ext->n_quads : 0u) + (ext && ext->media ? ext->n_media : 0u);
    if (n_unbounded > np) return -1;
    KTree kt;
    kt.width = width == 128 ? 4 : 2;
    kt.stride = width;
    kt.nodes = static_cast<const uint8_t *>(nodes);
    kt.n_nodes = n_nodes;
    kt.order = order;
    kt.unbounded = order + (np - n_unbounded);
    kt.n_unbounded = n_unbounded;
    return render<float>(cam, s, n, m, nm, tex, ntex, ext, flags, 0, y0, y1, s0, s1, threads, accum, rays, sphere_tests,
                         chunk, &kt);
}

// gpu::build_in_one_weekend_scene's sphere/material list (no overrides, camera seed out).
int oracle_rtow_scene(uint64_t seed, int grid_half, float *center_radius, uint32_t *mat_index, float *albedo_fuzz,
                      uint32_t *kind, float *ref_idx, uint32_t cap, uint32_t *n_out, uint32_t *sample_seed) {
    std::vector<float> cr, af, ri;
    std::vector<uint32_t> mi, kd;
    auto add = [&](float x, float y, float z, float r, uint32_t k, float a0, float a1, float a2, float fz, float rf) {
        cr.insert(cr.end(), {x, y, z, r});
        mi.push_back((uint32_t)kd.size());
        kd.push_back(k);
        af.insert(af.end(), {a0, a1, a2, fz});
        ri.push_back(rf);
    };
    Xoshiro256pp rng(seed);
    auto f32 = [&]() { return (float)(rng.next_u32() >> 8) * (1.0f / 16777216.0f); };
    auto f64 = [&]() { return (double)(rng.next_u64() >> 11) * (1.0 / 9007199254740992.0); };
    auto range05_1 = [&]() {
        for (;;) {
            uint32_t bits = (rng.next_u32() >> 9) | 0x3f800000u;
            float v;
            std::memcpy(&v, &bits, 4);
            const float r = (v - 1.0f) * 0.5f + 0.5f;
            if (r < 1.0f) return r;
        }
    };
    add(0.0f, -1000.0f, 0.0f, 1000.0f, 0, 0.5f, 0.5f, 0.5f, 0.0f, 1.0f);
    for (int a = -grid_half; a < grid_half; ++a)
        for (int b = -grid_half; b < grid_half; ++b) {
            const float choose = f32();
            const double cx = (double)a + 0.9 * f64();
            const double cz = (double)b + 0.9 * f64();
            const double dx = cx - 4.0, dy = 0.2 - 0.2, dz = cz - 0.0;
            if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {
                if (choose < 0.8f) {
                    float al[3];
                    for (int c = 0; c < 3; ++c) { const float p = f32(); const float q = f32(); al[c] = p * q; }
                    add((float)cx, (float)0.2, (float)cz, 0.2f, 0, al[0], al[1], al[2], 0.0f, 1.0f);
                } else if (choose < 0.95f) {
                    float al[3];
                    for (int c = 0; c < 3; ++c) al[c] = range05_1();
                    const float fz = f32() * 0.5f;
                    add((float)cx, (float)0.2, (float)cz, 0.2f, 1, al[0], al[1], al[2], fz, 1.0f);
                } else {
                    add((float)cx, (float)0.2, (float)cz, 0.2f, 2, 1.0f, 1.0f, 1.0f, 0.0f, 1.5f);
                }
            }
        }
    add(0.0f, 1.0f, 0.0f, 1.0f, 2, 1.0f, 1.0f, 1.0f, 0.0f, 1.5f);
    add(-4.0f, 1.0f, 0.0f, 1.0f, 0, 0.4f, 0.2f, 0.1f, 0.0f, 1.0f);
    add(4.0f, 1.0f, 0.0f, 1.0f, 1, 0.7f, 0.6f, 0.5f, 0.0f, 1.0f);
    const uint32_t n = (uint32_t)kd.size();
    *n_out = n;
    if (sample_seed) *sample_seed = rng.next_u32();
    if (cap < n) return cap == 0 ? 0 : -1;
    std::memcpy(center_radius, cr.data(), cr.size() * 4);
    std::memcpy(mat_index, mi.data(), mi.size() * 4);
    std::memcpy(albedo_fuzz, af.data(), af.size() * 4);
    std::memcpy(kind, kd.data(), kd.size() * 4);
    std::memcpy(ref_idx, ri.data(), ri.size() * 4);
    return 0;
}

// color.rs:6-32 write_color (f64): returns the three i32 bytes for one pixel.
void oracle_write_color(const double *pixel_color_scaled, int32_t *rgb) {
    for (int c = 0; c < 3; ++c) {
        double x = pixel_color_scaled[c];
        x = x > 0.0 ? std::sqrt(x) : 0.0;            // linear_to_gamma
        const double cl = x < 0.0 ? 0.0 : (x > 0.999 ? 0.999 : x);  // Interval::clamp (NaN passes)
        const double v = 256.0 * cl;
        rgb[c] = (v != v) ? 0 : (int32_t)v;          // Rust `as i32`: NaN -> 0
    }
}

// render_io.rs:8-26 quantiser (f32) for W*H RGBA accum -> rgb8.
void oracle_quantize_render_io(uint32_t n_pixels, const float *accum, uint32_t spp, uint8_t *rgb8) {
    const float scale = spp > 0 ? 1.0f / (float)spp : 0.0f;
    for (uint32_t i = 0; i < n_pixels; ++i)
        for (int c = 0; c < 3; ++c) {
            float r = accum[i * 4 + c] * scale;
            if (!std::isfinite(r)) r = 0.0f;
            r = std::sqrt(r > 0.0f ? r : 0.0f);
            if (r < 0.0f) r = 0.0f;
            if (r > 0.999f) r = 0.999f;
            rgb8[i * 3 + c] = (uint8_t)(r * 256.0f);
        }
}

// ---- known-answer hooks for the restated primitives (T = float when f32 != 0) ----------------
int oracle_sphere_hit(int f32, const double *center, double radius, const double *o, const double *d, double tmin,
                      double tmax, double *t_out, double *normal_out, int *front_out) {
    auto run = [&](auto tag) -> int {
        using T = decltype(tag);
        World<T> w;
        const Vec3<T> c = mk((T)center[0], (T)center[1], (T)center[2]);
        const T r = std::max((T)radius, T(0));
        w.spheres.push_back(Sphere<T>{c, r, 0, from_points(c - mk(r, r, r), c + mk(r, r, r))});
        const Vec3<T> O = mk((T)o[0], (T)o[1], (T)o[2]), D = mk((T)d[0], (T)d[1], (T)d[2]);
        T t;
        if (!w.hit_sphere(0, O, D, T(0), Interval<T>{(T)tmin, (T)tmax}, t, nullptr)) return 0;
        const Vec3<T> p = ray_at(O, D, t);
        const Vec3<T> out = (p - c) / r;
        const bool front = dot(D, out) < T(0);
        const Vec3<T> n = front ? out : -out;
        *t_out = t;
        for (int i = 0; i < 3; ++i) normal_out[i] = n[i];
        *front_out = front;
        return 1;
    };
    return f32 ? run(0.0f) : run(0.0);
}

// Quad::hit for one quad (q, u, v: 3-vectors, rounded to f32 as RrtQuad stores them).
int oracle_quad_hit(int f32, const double *q, const double *u, const double *v, const double *o, const double *d,
                    double tmin, double tmax, double *t_out, double *normal_out, int *front_out) {
    RrtQuad rq{};
    for (int i = 0; i < 3; ++i) rq.q[i] = (float)q[i], rq.u[i] = (float)u[i], rq.v[i] = (float)v[i];
    auto run = [&](auto tag) -> int {
        using T = decltype(tag);
        World<T> w;
        w.quads.push_back(make_quad<T>(rq));
        const Vec3<T> O = mk((T)o[0], (T)o[1], (T)o[2]), D = mk((T)d[0], (T)d[1], (T)d[2]);
        T t;
        if (!w.hit_quad(0, O, D, Interval<T>{(T)tmin, (T)tmax}, t, nullptr)) return 0;
        const Vec3<T> out = w.quads[0].normal;
        const bool front = dot(D, out) < T(0);
        const Vec3<T> n = front ? out : -out;
        *t_out = t;
        for (int i = 0; i < 3; ++i) normal_out[i] = n[i];
        *front_out = front;
        return 1;
    };
    return f32 ? run(0.0f) : run(0.0);
}

int oracle_aabb_hit(int f32, const double *lo, const double *hi, const double *o, const double *d, double tmin, double tmax) {
    auto run = [&](auto tag) -> int {
        using T = decltype(tag);
        Aabb<T> b;
        for (int i = 0; i < 3; ++i) b.ax[i] = Interval<T>{(T)lo[i], (T)hi[i]};
        return aabb_hit(b, mk((T)o[0], (T)o[1], (T)o[2]), mk((T)d[0], (T)d[1], (T)d[2]), Interval<T>{(T)tmin, (T)tmax});
    };
    return f32 ? run(0.0f) : run(0.0);
}

void oracle_reflect_refract(int f32, const double *v, const double *n, double eta, double *refl, double *refr,
                            double *schlick_cos_eta) {
    auto run = [&](auto tag) {
        using T = decltype(tag);
        const Vec3<T> V = mk((T)v[0], (T)v[1], (T)v[2]), N = mk((T)n[0], (T)n[1], (T)n[2]);
        const Vec3<T> a = reflect(V, N), b = refract(V, N, (T)eta);
        for (int i = 0; i < 3; ++i) { refl[i] = a[i]; refr[i] = b[i]; }
        const T cosine = (T)schlick_cos_eta[0], rix = (T)schlick_cos_eta[1];
        T r0 = (T(1) - rix) / (T(1) + rix);
        r0 = r0 * r0;
        const T x = T(1) - cosine, x2 = x * x, x4 = x2 * x2;
        schlick_cos_eta[2] = r0 + (T(1) - r0) * (x * x4);
    };
    if (f32) run(0.0f); else run(0.0);
}

// The first `count` u32 draws of path (seed, pixel, sample).
void oracle_path_stream(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t count, uint32_t *out) {
    const uint64_t key = splitmix64(((uint64_t)seed << 32) ^ (uint64_t)pixel);
    PathRng rng(splitmix64(key + sample), key);
    for (uint32_t i = 0; i < count; ++i) out[i] = rng.next();
}

// fdlibm acos / atan2 as BOOKS (f64) evaluates them, over arrays (checked against libm by tests).
void oracle_acos_atan2_f64(uint32_t n, const double *x, const double *y, double *acos_out, double *atan2_out) {
    for (uint32_t i = 0; i < n; ++i) {
        if (acos_out) acos_out[i] = fdlibm_acos(x[i]);
        if (atan2_out) atan2_out[i] = fdlibm_atan2(y[i], x[i]);
    }
}

void oracle_acos_atan2_f32(float x, float y, float *acos_out, float *atan2_out) {
    *acos_out = cephes_acosf(x);
    *atan2_out = cephes_atan2f(y, x);
}

// Known-answer hooks for book-2 textures: f32 Cephes sin, and the Perlin noise / NoiseTexture
// value / checker parity at points p[n][3] with table `pt` (f32 != 0: twin arithmetic).
void oracle_sin_f32(uint32_t n, const float *x, float *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = cephes_sinf(x[i]);
}

void oracle_cos_f32(uint32_t n, const float *x, float *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = cephes_cosf(x[i]);
}

void oracle_log_f32(uint32_t n, const float *x, float *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = cephes_logf(x[i]);
}

// The media free-flight uniform of include/rrt_hip.h for (seg, medium) pairs.
void oracle_medium_u(uint32_t n, const uint64_t *seg, const uint32_t *medium, float *out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = (float)(uint32_t)(splitmix64(seg[i] ^ (uint64_t)medium[i]) >> 40) * 0x1.0p-24f;
}

void oracle_book2_textures(int f32, const RrtPerlin *pt, double scale, double inv_scale, uint32_t n, const double *p,
                           double *noise_out, double *value_out, int32_t *even_out) {
    auto run = [&](auto tag) {
        using T = decltype(tag);
        PerlinT<T> t;
        for (int i = 0; i < 256; ++i) {
            t.randvec[i] = mk((T)pt->randvec[i][0], (T)pt->randvec[i][1], (T)pt->randvec[i][2]);
            t.perm_x[i] = pt->perm_x[i] & 255u;
            t.perm_y[i] = pt->perm_y[i] & 255u;
            t.perm_z[i] = pt->perm_z[i] & 255u;
        }
        for (uint32_t k = 0; k < n; ++k) {
            const Vec3<T> q = mk((T)p[3 * k], (T)p[3 * k + 1], (T)p[3 * k + 2]);
            noise_out[k] = (double)perlin_noise(t, q);
            value_out[k] = (double)noise_value(t, (T)scale, q);
            even_out[k] = checker_even((T)inv_scale, q) ? 1 : 0;
        }
    };
    if (f32) run(0.0f); else run(0.0);
}

}  // extern "C"
