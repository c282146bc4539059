/* Checks the kernels' division by a constant (rrt_kernel.hip div_by_const, rrt_books64.hip
 * div_by_const64): q = x * RN(1/c), result fma(fma(-q, c, x), RN(1/c), q), against the IEEE quotient
 * x / c computed by the CPU, for c = 2 pi and pi as the kernels spell them.
 *   f32: every float in [2^-100, 8] and +0 (exhaustive);
 *   f64: N random doubles in [2^-60, 8) (uniform exponent and mantissa bits).
 * Prints "f32 <c> <checked> <mismatches>" / "f64 <c> <checked> <mismatches>" lines.
 * Built with -ffp-contract=off -mfma (host FMA = the device's fused multiply-add). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f32_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t state = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) { state ^= state << 13; state ^= state >> 7; state ^= state << 17; return state; }

int main(int argc, char **argv) {
    const long long n64 = argc > 1 ? atoll(argv[1]) : 20000000ll;
    const float pi32 = 3.14159265358979323846f;            /* rrt_kernel.hip kPi */
    const double pi64 = 3.14159265358979311600e+00;        /* rrt_books64.hip kPiD */
    const float c32[2] = {2.0f * pi32, pi32};
    const double c64[2] = {2.0 * pi64, pi64};
    for (int k = 0; k < 2; ++k) {
        const volatile float c = c32[k];
        const volatile float rc = 1.0f / c;
        long long checked = 0, bad = 0;
        const uint32_t lo = 0x0d800000u /* 2^-100 */, hi = 0x41000000u /* 8 */;
        for (uint32_t u = lo; ; ++u) {
            const float x = u == lo - 1 ? 0.0f : f32_of(u);
            const float q = x * rc;
            const float r = fmaf(-q, c, x);
            const float got = fmaf(r, rc, q);
            const float ref = x / c;
            ++checked;
            if (memcmp(&got, &ref, 4) != 0) ++bad;
            if (u == hi) break;
        }
        { /* +0 */
            const float x = 0.0f, q = x * rc, got = fmaf(fmaf(-q, c, x), rc, q), ref = x / c;
            ++checked;
            if (memcmp(&got, &ref, 4) != 0) ++bad;
        }
        printf("f32 %.9g %lld %lld\n", (double)c, checked, bad);
    }
    for (int k = 0; k < 2; ++k) {
        const volatile double c = c64[k];
        const volatile double rc = 1.0 / c;
        long long bad = 0;
        for (long long i = 0; i < n64; ++i) {
            const int e = (int)(next() % 63) - 60;
            const uint64_t b = ((uint64_t)(e + 1023) << 52) | (next() & 0xFFFFFFFFFFFFFull);
            double x;
            memcpy(&x, &b, 8);
            const double q = x * rc;
            const double got = fma(fma(-q, c, x), rc, q);
            const double ref = x / c;
            if (memcmp(&got, &ref, 8) != 0) ++bad;
        }
        printf("f64 %.17g %lld %lld\n", c, n64, bad);
    }
    return 0;
}
