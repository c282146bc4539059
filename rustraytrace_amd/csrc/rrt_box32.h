// rrt_box32.h — the f64 books kernel's BVH box test, run in f32 and widened so that it can never
// reject a box the f64 ray meets (role of Aabb::hit, books/in_one_weekend/aabb.rs:52-85: a box test
// only prunes; which sphere is hit is decided by the f64 sphere test alone).
//
// Compiled for the device by rrt_books64.hip and for the host by tests/box32/box32_harness.cpp, which
// checks the bound below against exact rational arithmetic on adversarial rays, with the hardware
// reciprocal's estimate emulated 0, 1 and 2 ulps off either side of 1/x
// (tests/test_box32_conservative.py). IEEE f32 fma, mul, min, max, fabs, and v_rcp_f32.
//
// The f64 ray (o, d) is rounded once per ray: d32 = fl(d), o32 = fl(o), q = 1 / d32 to within 1.01 u
// (box32_recip), inv = q clamped to +-2^64, oi = fl(o32 * inv). A stored f32 plane P then gives
// t' = fl(fma(P, inv, -oi)) for the exact t = (P - o) / d. With u = 2^-24 and |q| <= 2^64:
//   inv = (1/d)(1 + eta), |eta| <= 2.02u         (d rounding, reciprocal error)
//   oi  = (o * inv)(1 + g), |g| <= 2u + u^2      (o rounding, product rounding)
//   t'  = (t (1 + eta) - (o * inv) g)(1 + e), |e| <= u
// so |t' - t| <= 3.03 u |t'| + 2.001 u |oi|. The test widens the entry distance down and the exit
// distance up by E = 8u (|t'| + m) + 2^-100, m = max |oi_a| over the ray's unclamped axes (the
// 2^-100 keeps E > 0): more than twice the bound, which also absorbs the rounding of E and of
// t' -+ E. The entry is nr = max(entry planes, 0.001 rounded down), the exit fr = min(exit planes,
// fl32(closest)). Let a sphere inside the box be hit by the f64 ray at t* in (0.001, closest), so
// t_entry,a <= t* <= t_exit,a on every axis. If nr is axis m's t', then nr <= t_m + err_m <= t* +
// err_m, and err_m < E(nr) because |nr| = |t'_m| and m >= |oi_m|; if nr is the tmin constant it
// is below t* already. Likewise fr >= t* - E(fr) (fl32(closest) >= closest (1 - u) > t* - E). So
// nr - E(nr) < t* < fr + E(fr): the box is accepted. Other axes need no widening of their own:
// only the attaining one enters the comparison.
// A clamped axis (|q| > 2^64: d_a = 0 or |d_a| < 2^-64) gives plane distances (P - o32) * 2^64 with
// the sign of P - o (the host grows every stored plane by more than u |o_a| for origins within the
// scene's extent, rrt_host.cpp BoxSlack): such a ray stays inside that slab, or outside it, for
// every t a scene of extent < 2^40 can produce, exactly as the f32 megakernel's test assumes.
#pragma once

#ifndef RRT_HD
#define RRT_HD __host__ __device__
#endif

constexpr float kBox32Widen = 0x1.0p-21f;   // 8u
constexpr float kBox32Abs = 0x1.0p-100f;
constexpr float kBox32Tmin = 0x1.0624dcp-10f;  // the largest f32 below 0.001 (camera.rs:187's tmin)

struct RayBox32 {
    float ix, iy, iz;     // inv
    float oix, oiy, oiz;  // o32 * inv
    float c;              // 8u * m + 2^-100
};

RRT_HD inline float box32_clamp(float v) { return __builtin_fmaxf(__builtin_fminf(v, 0x1.0p64f), -0x1.0p64f); }

// q ~ 1 / x: the hardware reciprocal (v_rcp_f32, <= 1 ulp) refined by one Newton step, which leaves
// a relative error below 1.01 u (the error of the estimate squared, plus the step's own rounding);
// no IEEE division is needed, only the bound. Skipped beyond 2^64 (x = +-0 or |x| < 2^-64: the
// step would meet 0 * inf), where the clamp takes over.
#ifndef RRT_BOX32_RCP
#define RRT_BOX32_RCP(x) __builtin_amdgcn_rcpf(x)
#endif
RRT_HD inline float box32_recip(float x) {
    const float r = RRT_BOX32_RCP(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fabsf(r) <= 0x1.0p64f ? __builtin_fmaf(e, r, r) : r;
}

RRT_HD inline RayBox32 box32_ray(double ox, double oy, double oz, double dx, double dy, double dz) {
    const float qx = box32_recip((float)dx), qy = box32_recip((float)dy), qz = box32_recip((float)dz);
    RayBox32 r;
    r.ix = box32_clamp(qx);
    r.iy = box32_clamp(qy);
    r.iz = box32_clamp(qz);
    r.oix = (float)ox * r.ix;
    r.oiy = (float)oy * r.iy;
    r.oiz = (float)oz * r.iz;
    float m = 0.0f;
    if (__builtin_fabsf(qx) <= 0x1.0p64f) m = __builtin_fmaxf(m, __builtin_fabsf(r.oix));
    if (__builtin_fabsf(qy) <= 0x1.0p64f) m = __builtin_fmaxf(m, __builtin_fabsf(r.oiy));
    if (__builtin_fabsf(qz) <= 0x1.0p64f) m = __builtin_fmaxf(m, __builtin_fabsf(r.oiz));
    r.c = __builtin_fmaf(m, kBox32Widen, kBox32Abs);
    return r;
}

// Planes in (entry, exit) order per axis (the ray's sign offsets into a GNode, or a GNodeH's halves
// rotated by the sign): fma(P, inv, -oi) is monotone in P for a fixed inv, so the entry plane's
// distance is the min of the axis pair and the exit plane's the max. tmax = fl32(closest).
RRT_HD inline bool box32_hit(float nx, float fx, float ny, float fy, float nz, float fz, const RayBox32 &r, float tmax,
                             float &tnear) {
    const float x0 = __builtin_fmaf(nx, r.ix, -r.oix), x1 = __builtin_fmaf(fx, r.ix, -r.oix);
    const float y0 = __builtin_fmaf(ny, r.iy, -r.oiy), y1 = __builtin_fmaf(fy, r.iy, -r.oiy);
    const float z0 = __builtin_fmaf(nz, r.iz, -r.oiz), z1 = __builtin_fmaf(fz, r.iz, -r.oiz);
    const float nr = __builtin_fmaxf(__builtin_fmaxf(x0, y0), __builtin_fmaxf(z0, kBox32Tmin));
    const float fr = __builtin_fminf(__builtin_fminf(x1, y1), __builtin_fminf(z1, tmax));
    tnear = nr;
    const float en = __builtin_fmaf(__builtin_fabsf(nr), kBox32Widen, r.c);
    const float ef = __builtin_fmaf(__builtin_fabsf(fr), kBox32Widen, r.c);
    return nr - en < fr + ef;
}
