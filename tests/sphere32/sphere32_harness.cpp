// Host build of the f64 books kernel's sphere pre-test (rustraytrace_amd/csrc/rrt_sphere32.h, the
// same source the device compiles) for tests/test_sphere32_conservative.py. Test infrastructure only.
// g++ -O2 -std=c++17 -ffp-contract=off -fno-fast-math -shared -fPIC sphere32_harness.cpp
#include <cmath>
#include <cstdint>
#include <random>

#define RRT_HD
#include "../../rustraytrace_amd/csrc/rrt_sphere32.h"

namespace {
// the f64 kernel's discriminant (rrt_books64.hip leaves64 = sphere.rs:24-51): unfused, in the
// reference's operation order (this file is built with -ffp-contract=off)
double disc64(const double *o, const double *d, const float *c, float r) {
    const double ocx = (double)c[0] - o[0], ocy = (double)c[1] - o[1], ocz = (double)c[2] - o[2];
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double h = d[0] * ocx + d[1] * ocy + d[2] * ocz;
    const double cc = (ocx * ocx + ocy * ocy + ocz * ocz) - (double)r * (double)r;
    return h * h - a * cc;
}
bool miss32(const double *o, const double *d, const float *c, float r) {
    const RaySphere32 k = sphere32_ray(o[0], o[1], o[2], d[0], d[1], d[2]);
    return sphere32_miss(k, c[0], c[1], c[2], r);
}
}  // namespace

extern "C" {
void sphere32_eval(uint32_t n, const double *o, const double *d, const float *c, const float *r, uint8_t *miss,
                   double *disc) {
    for (uint32_t i = 0; i < n; ++i) {
        miss[i] = miss32(o + 3 * i, d + 3 * i, c + 3 * i, r[i]);
        disc[i] = disc64(o + 3 * i, d + 3 * i, c + 3 * i, r[i]);
    }
}

// Adversarial sweep. Spheres: centers up to 2^20 (the host's domain), radii 1e-4 .. 1e3. Origins on
// the sphere (a secondary ray leaves a hit point), inside it, or 1e-3 .. 1e5 away. Directions aimed
// at the tangent cone: the ray's distance to the center is r (1 + eps), eps = +-1e-12 .. 0.3 or 0,
// magnitudes 1e-6 .. 1e6, some components zeroed. out = {cases, disc >= 0, rejected, violations
// (rejected although disc >= 0), clear misses in the domain (disc < -1e-3 a (|oc|^2 + r^2 + 1e-6 |o|^2)),
// clear misses rejected}.
void sphere32_sweep(uint32_t n, uint64_t seed, uint64_t *out) {
    std::mt19937_64 g(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto logu = [&](double lo, double hi) { return std::exp(std::log(lo) + (std::log(hi) - std::log(lo)) * U(g)); };
    auto sgn = [&]() { return U(g) < 0.5 ? -1.0 : 1.0; };
    auto unit = [&](double *v) {
        double l;
        do {
            for (int a = 0; a < 3; ++a) v[a] = 2.0 * U(g) - 1.0;
            l = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        } while (l > 1.0 || l < 1e-6);
        l = std::sqrt(l);
        for (int a = 0; a < 3; ++a) v[a] /= l;
    };
    uint64_t hits = 0, rej = 0, viol = 0, clear = 0, clear_rej = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const double R = std::vector<double>{1.0, 20.0, 1e3, 1e5, 1e6}[i % 5];
        float c[3];
        for (int a = 0; a < 3; ++a) c[a] = (float)(sgn() * U(g) * R);
        const float r = (float)logu(1e-4, 1e3);
        double o[3], d[3], n0[3];
        unit(n0);
        const double mode = U(g);
        if (mode < 0.4) {  // on the sphere, nudged by a few f64 ulps
            for (int a = 0; a < 3; ++a) o[a] = (double)c[a] + (double)r * n0[a];
            if (U(g) < 0.5) {
                const int a = (int)(U(g) * 3);
                for (int k = (int)(U(g) * 4); k > 0; --k) o[a] = std::nextafter(o[a], U(g) < 0.5 ? -INFINITY : INFINITY);
            }
        } else if (mode < 0.5) {  // inside
            const double s = U(g);
            for (int a = 0; a < 3; ++a) o[a] = (double)c[a] + s * (double)r * n0[a];
        } else {  // outside, 1e-3 .. 1e5 beyond the surface
            const double L = (double)r + logu(1e-3, 1e5);
            for (int a = 0; a < 3; ++a) o[a] = (double)c[a] + L * n0[a];
        }
        // aim at distance r (1 + eps) from the center
        double v[3] = {(double)c[0] - o[0], (double)c[1] - o[1], (double)c[2] - o[2]};
        const double L = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double p[3];
        unit(p);
        if (L > 0) {
            const double pv = (p[0] * v[0] + p[1] * v[1] + p[2] * v[2]) / (L * L);
            for (int a = 0; a < 3; ++a) p[a] -= pv * v[a];
            const double pl = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
            for (int a = 0; a < 3; ++a) p[a] /= pl;
        }
        const double em = U(g);
        const double eps = em < 0.1 ? 0.0 : sgn() * logu(1e-12, 0.3);
        const double s = L > 0 ? std::min(1.0, (double)r * (1.0 + eps) / L) : 0.0;
        const double cs = std::sqrt(std::max(0.0, 1.0 - s * s));
        const double mag = logu(1e-6, 1e6);
        const double dir_sign = U(g) < 0.8 ? 1.0 : -1.0;  // some rays point away
        for (int a = 0; a < 3; ++a) d[a] = mag * (dir_sign * cs * (L > 0 ? v[a] / L : 0.0) + s * p[a]);
        const double m2 = U(g);
        if (m2 < 0.05) d[(int)(U(g) * 3)] = 0.0;
        else if (m2 < 0.08) d[(int)(U(g) * 3)] = -0.0;
        if (U(g) < 0.3) {
            const int a = (int)(U(g) * 3);
            for (int k = (int)(U(g) * 4); k > 0; --k) d[a] = std::nextafter(d[a], U(g) < 0.5 ? -INFINITY : INFINITY);
        }
        const double D = disc64(o, d, c, r);
        const bool m = miss32(o, d, c, r);
        const double a2 = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const double X2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
        hits += D >= 0.0;
        rej += m;
        viol += (m && !(D < 0.0));
        const double Y2 = o[0] * o[0] + o[1] * o[1] + o[2] * o[2];
        const bool domain = a2 >= 0x1.01p-40 && a2 <= 0x1.fep39 && Y2 <= 0x1.fep39;
        if (domain && D < -1e-3 * a2 * (X2 + (double)r * r + 1e-6 * Y2)) {
            ++clear;
            clear_rej += m;
        }
    }
    out[0] = n;
    out[1] = hits;
    out[2] = rej;
    out[3] = viol;
    out[4] = clear;
    out[5] = clear_rej;
}
}
