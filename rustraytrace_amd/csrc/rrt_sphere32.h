// rrt_sphere32.h — the f64 books kernel's sphere pre-test, run in f32 with a proven error bound so
// that it rejects a sphere only when the kernel's f64 discriminant (sphere.rs:24-51: oc = center - o,
// a = |d|^2, h = d.oc, c = |oc|^2 - r*r, disc = h*h - a*c, computed unfused in f64) is negative.
// A rejected sphere is one the f64 test would `continue` past, so the closest hit, and every bit the
// kernel produces, is unchanged; a sphere the bound cannot decide runs the f64 test as before.
//
// Compiled for the device by rrt_books64.hip and for the host by tests/sphere32/sphere32_harness.cpp,
// which runs the test against the kernel's own f64 discriminant on adversarial rays (grazing within
// 1e-9 of tangency, origins on the sphere, far origins, tiny and huge directions):
// tests/test_sphere32_conservative.py. IEEE f32 fma, mul, add.
//
// Per ray: o32 = fl(o), d32 = fl(d), a32 = fl-dot(d32, d32), k = u 2^-6 fl-dot(o32, o32) + 2^-30.
// Per sphere (the f32 record: center c exact, radius r exact): oc = fl(c - o32),
// h = fma-dot(d32, oc), q = fma-dot(oc, oc), g = fma(q, 1 - 2048u, -fma(r, fl(r (1 + 128u)), k)),
// reject iff fl(h h) < fl(a32 g). With u = 2^-24, X = |c - o|, Y = |o|, A = |d|^2, R = r^2 and
// D the exact discriminant (H = d.(c - o), D = H^2 - A (X^2 - R)):
//   oc_i = (c_i - o_i)(1 + e1) + o_i e2 (1 + e1), |e1|, |e2| <= u
//   |h - H| <= sqrt(A) (5.001 u X + 1.001 u Y)      (d rounding, oc error, the dot's three roundings)
//   |a32 - A| <= 5.01 u A,  |q - X^2| <= 5.001 u X^2 + 2.001 u X Y
// so |h^2 - a32 (q - R) - D| <= A (20.02 u X^2 + 4.01 u X Y + 5.02 u R) + O(u^2), and with
// X Y <= (512 X^2 + Y^2 / 512) / 2 the bound is A (1047 u X^2 + 5.02 u R + 0.004 u Y^2). The test's
// own roundings (g, a32 g, h h: a factor 1 + 3.01 u) are absorbed by the margins: 1 - 2048u against
// the 1047u X^2 term (and the q / X^2 and a32 / A ratios), 1 + 128u on r twice against 5.02u R, and
// u 2^-6 Y^2 against 0.004 u Y^2. The f64 discriminant's own error, below A (X^2 + R) 2^-46, is in
// the same margins. So a rejection means D < -(the f64 rounding) and the f64 disc < 0.
// Domain (else the ray or the scene never rejects, k = +inf): a32 in [2^-40, 2^40], |o32|^2 <= 2^40,
// and the host enables the test only for scenes whose centers and radii are within 2^20
// (KParams.sphere32); there every value stays far from f32 overflow, and 2^-30 a32 >= 2^-70 covers
// the absolute errors of underflowing products (each <= 2^-126, times |h|, |q - R| <= 2^45: < 2^-78).
// A NaN anywhere makes the comparison false: no rejection.
#pragma once

#ifndef RRT_HD
#define RRT_HD __host__ __device__
#endif

constexpr float kS32Q = 1.0f - 0x1.0p-13f;      // 1 - 2048u
constexpr float kS32R = 1.0f + 0x1.0p-17f;      // 1 + 128u
constexpr float kS32Y = 0x1.0p-30f;             // u 2^-6
constexpr float kS32Abs = 0x1.0p-30f;

struct RaySphere32 {
    float ox, oy, oz, dx, dy, dz;
    float a;  // fl-dot(d32, d32)
    float k;  // u 2^-6 |o32|^2 + 2^-30, or +inf outside the domain (never rejects)
};

RRT_HD inline RaySphere32 sphere32_ray(double ox, double oy, double oz, double dx, double dy, double dz) {
    RaySphere32 r;
    r.ox = (float)ox;
    r.oy = (float)oy;
    r.oz = (float)oz;
    r.dx = (float)dx;
    r.dy = (float)dy;
    r.dz = (float)dz;
    r.a = __builtin_fmaf(r.dz, r.dz, __builtin_fmaf(r.dy, r.dy, r.dx * r.dx));
    const float y2 = __builtin_fmaf(r.oz, r.oz, __builtin_fmaf(r.oy, r.oy, r.ox * r.ox));
    const bool in = r.a >= 0x1.0p-40f && r.a <= 0x1.0p40f && y2 <= 0x1.0p40f;
    r.k = in ? __builtin_fmaf(y2, kS32Y, kS32Abs) : __builtin_inff();
    return r;
}

// true: the f64 discriminant of this sphere is negative (the f64 test may be skipped)
RRT_HD inline bool sphere32_miss(const RaySphere32 &r, float cx, float cy, float cz, float rad) {
    const float ocx = cx - r.ox, ocy = cy - r.oy, ocz = cz - r.oz;
    const float h = __builtin_fmaf(r.dz, ocz, __builtin_fmaf(r.dy, ocy, r.dx * ocx));
    const float q = __builtin_fmaf(ocz, ocz, __builtin_fmaf(ocy, ocy, ocx * ocx));
    const float rk = __builtin_fmaf(rad, rad * kS32R, r.k);
    const float g = __builtin_fmaf(q, kS32Q, -rk);
    return h * h < r.a * g;
}
