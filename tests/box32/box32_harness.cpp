// Host build of the f64 books kernel's box test (rustraytrace_amd/csrc/rrt_box32.h, the same source
// the device compiles) for tests/test_box32_conservative.py. Test infrastructure only.
// g++ -O2 -std=c++17 -ffp-contract=off -fno-fast-math -shared -fPIC box32_harness.cpp
#include <cmath>
#include <cstdint>
#include <random>

// v_rcp_f32 on the host: the correctly rounded 1/x moved g_rcp_ulps ulps (the device estimate is
// within 1 ulp; the test runs -2 .. 2)
static int g_rcp_ulps = 0;
static float host_rcp(float x) {
    float r = 1.0f / x;
    for (int k = 0; k < g_rcp_ulps; ++k) r = std::nextafter(r, INFINITY);
    for (int k = 0; k > g_rcp_ulps; --k) r = std::nextafter(r, -INFINITY);
    return r;
}
#define RRT_HD
#define RRT_BOX32_RCP(x) host_rcp(x)
#include "../../rustraytrace_amd/csrc/rrt_box32.h"

namespace {
// the kernel's plane selection: (entry, exit) = (lo, hi) when inv >= 0 (not negative), else (hi, lo)
bool eval_one(const double *o, const double *d, const float *lo, const float *hi, double closest, float *tnear) {
    const RayBox32 r = box32_ray(o[0], o[1], o[2], d[0], d[1], d[2]);
    const float inv[3] = {r.ix, r.iy, r.iz};
    float n[3], f[3];
    for (int a = 0; a < 3; ++a) {
        n[a] = inv[a] < 0.0f ? hi[a] : lo[a];
        f[a] = inv[a] < 0.0f ? lo[a] : hi[a];
    }
    return box32_hit(n[0], f[0], n[1], f[1], n[2], f[2], r, (float)closest, *tnear);
}

// exact-enough reference in long double (64-bit significand): is the ray's interval
// [max(t_entry, 0.001), min(t_exit, closest)] through the box nonempty? 1 yes, 0 no, -1 outside the
// test's contract: an axis the test clamps (1/d_a beyond 2^64, e.g. d_a = 0) with the origin within
// 4u |o_a| of one of that axis's planes. The product never meets such a case: rrt_host.cpp's
// BoxSlack grows every stored plane past the primitive's box by more than that for origins within
// the scene's extent, so a ray that runs inside a plane's rounding distance misses the primitive.
int meets_ld(const double *o, const double *d, const float *lo, const float *hi, double closest) {
    long double te = 0.001L, tx = (long double)closest;
    for (int a = 0; a < 3; ++a) {
        const long double L = lo[a], H = hi[a], oa = o[a], da = d[a];
        if (std::fabs(1.0f / (float)d[a]) > 0x1.0p64f) {
            const long double tol = 4.0L * 0x1.0p-24L * std::fabs(oa) + 0x1.0p-120L;
            if (std::fabs(oa - L) <= tol || std::fabs(oa - H) <= tol) return -1;
        }
        if (da == 0.0L) {
            if (oa < L || oa > H) return 0;
            continue;
        }
        long double t0 = (L - oa) / da, t1 = (H - oa) / da;
        if (t0 > t1) std::swap(t0, t1);
        te = std::max(te, t0);
        tx = std::min(tx, t1);
    }
    return te <= tx ? 1 : 0;
}
}  // namespace

extern "C" {
void box32_set_rcp_ulps(int k) { g_rcp_ulps = k; }

void box32_eval(uint32_t n, const double *o, const double *d, const float *lo, const float *hi, const double *closest,
                uint8_t *accept, float *tnear) {
    for (uint32_t i = 0; i < n; ++i) accept[i] = eval_one(o + 3 * i, d + 3 * i, lo + 3 * i, hi + 3 * i, closest[i], tnear + i);
}

// Random adversarial sweep: boxes at |center| up to 2e4 with extents 1e-6 .. 1e3, rays aimed at a
// corner, an edge or a face point of the box (optionally nudged off it by a few f64 ulps), from
// origins up to 1e5 away (and from inside the box), directions scaled by 1e-3 .. 1e3, some components
// zeroed or made tiny, closest hits just past the entry. out = {cases, exact-meets, accepted,
// violations (meets but rejected), rejected-non-meets}.
void box32_sweep(uint32_t n, uint64_t seed, uint64_t *out) {
    std::mt19937_64 g(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto logu = [&](double lo, double hi) { return std::exp(std::log(lo) + (std::log(hi) - std::log(lo)) * U(g)); };
    auto sgn = [&]() { return U(g) < 0.5 ? -1.0 : 1.0; };
    uint64_t meets = 0, acc = 0, viol = 0, rej = 0, skipped = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const double R = (i % 3 == 0) ? 1.0 : (i % 3 == 1 ? 1e3 : 2e4);
        float lo[3], hi[3];
        double c[3];
        for (int a = 0; a < 3; ++a) {
            c[a] = sgn() * U(g) * R;
            const double e = logu(1e-6, 1e3);
            lo[a] = (float)(c[a] - e);
            hi[a] = (float)(c[a] + e);
            if (lo[a] > hi[a]) std::swap(lo[a], hi[a]);
        }
        // target: a corner, an edge point or a face point of the stored box
        double p[3];
        const int kind = (int)(U(g) * 3.0);
        for (int a = 0; a < 3; ++a) {
            const bool on_plane = (kind == 0) || (kind == 1 && a < 2) || (kind == 2 && a == 0);
            p[a] = on_plane ? (U(g) < 0.5 ? lo[a] : hi[a]) : lo[a] + (hi[a] - lo[a]) * U(g);
        }
        double o[3], d[3];
        const double dist = logu(1e-3, 1e5);
        const bool inside = U(g) < 0.1;
        for (int a = 0; a < 3; ++a) {
            o[a] = inside ? lo[a] + (hi[a] - lo[a]) * U(g) : p[a] + sgn() * U(g) * dist;
        }
        const double scale = logu(1e-3, 1e3);
        for (int a = 0; a < 3; ++a) d[a] = (p[a] - o[a]) * scale;
        const double mode = U(g);
        if (mode < 0.05) d[(int)(U(g) * 3)] = 0.0;
        else if (mode < 0.08) d[(int)(U(g) * 3)] = -0.0;
        else if (mode < 0.12) d[(int)(U(g) * 3)] = sgn() * logu(1e-30, 1e-8);
        if (U(g) < 0.3) {  // nudge the target by a few ulps
            const int a = (int)(U(g) * 3);
            for (int k = (int)(U(g) * 4); k > 0; --k) d[a] = std::nextafter(d[a], U(g) < 0.5 ? -INFINITY : INFINITY);
        }
        double closest = INFINITY;
        if (U(g) < 0.5) {  // a closest hit just past the box entry
            long double te = 0.001L;
            for (int a = 0; a < 3; ++a)
                if (d[a] != 0.0) {
                    long double t0 = ((long double)lo[a] - o[a]) / d[a], t1 = ((long double)hi[a] - o[a]) / d[a];
                    te = std::max(te, std::min(t0, t1));
                }
            closest = (double)te;
            for (int k = (int)(U(g) * 3); k > 0; --k) closest = std::nextafter(closest, INFINITY);
        }
        float tn;
        const int mc = meets_ld(o, d, lo, hi, closest);
        if (mc < 0) {
            ++skipped;
            continue;
        }
        const bool m = mc == 1;
        const bool a = eval_one(o, d, lo, hi, closest, &tn);
        meets += m;
        acc += a;
        viol += (m && !a);
        rej += (!m && !a);
    }
    out[0] = n - skipped;
    out[1] = meets;
    out[2] = acc;
    out[3] = viol;
    out[4] = rej;
    out[5] = skipped;
}
}
