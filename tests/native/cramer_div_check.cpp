// Property check of the triangle test's shared-reciprocal quotients (rt_device.hpp cramer_div3):
// r0 = an f32 reciprocal of den with relative error up to 2^-21 (the device's v_rcp_f32 is
// within 1 ulp; the check perturbs it much further), two Newton steps in double, q = RN_53(n * r),
// RN_24(q) -- must equal the IEEE float quotient RN_24(n / den) whenever the fast path is taken
// (|den| in [2^-100, 2^100] and |RN_24(q)| >= 2^-125).  Cases: random numerators/denominators over
// the whole exponent range, and the hard ones: numerators chosen so n / den lies within a few ulps
// of the float grid's rounding midpoints, and exactly representable quotients.  Plain C++ with
// the same float/double operations as the device (fma = one rounding; -ffp-contract=off).
// Prints "<quotients checked> <mismatches> <fast-path fraction>".  With one Newton step instead of
// two (argv[2] = 1, a control) the near-midpoint cases must mismatch.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

static int g_newton = 2;   // argv[2]: Newton steps (the device takes 2; fewer must fail: a control)

static bool fast_path(float den, const float* n, float* q, double rel) {
    const double D = (double)den;
    const float r0f = (float)((1.0 / D) * (1.0 + rel));          // a reciprocal off by `rel`
    double r = (double)r0f;
    for (int it = 0; it < g_newton; ++it) {
        const double e = std::fma(-D, r, 1.0);
        r = std::fma(e, r, r);
    }
    for (int j = 0; j < 3; ++j) q[j] = (float)((double)n[j] * r);
    const float ad = std::fabs(den);
    const float m = std::fmin(std::fmin(std::fabs(q[0]), std::fabs(q[1])), std::fabs(q[2]));
    return ad >= 0x1p-100f && ad <= 0x1p100f && m >= 0x1p-125f;
}

static float rnd_float(std::mt19937_64& g, int emin, int emax) {
    std::uniform_int_distribution<int> E(emin, emax);
    std::uniform_int_distribution<uint32_t> M(0, (1u << 23) - 1);
    const float v = std::ldexp(1.0f + (float)M(g) * 0x1p-23f, E(g));
    return (g() & 1) ? -v : v;
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    if (argc > 2) g_newton = atoi(argv[2]);
    std::mt19937_64 g(20261017);
    const double rels[] = {0.0, 0x1p-21, -0x1p-21, 0x1p-24, -0x1p-23};
    long checked = 0, bad = 0, fast = 0;
    for (long i = 0; i < n; ++i) {
        const int kind = (int)(i % 4);
        const float den = kind == 3 ? rnd_float(g, -140, 120) : rnd_float(g, -60, 60);
        float num[3];
        for (int j = 0; j < 3; ++j) {
            if (kind == 0 || kind == 3) {
                num[j] = rnd_float(g, -149, 127);
                if (kind == 0) num[j] = rnd_float(g, -60, 60);
            } else {
                // a quotient near a rounding midpoint (kind 1) or exactly on the float grid (kind 2):
                // q0 on the grid, m = q0 + ulp/2; num = RN_24(m * den) (or q0 * den) then nudged
                const float q0 = rnd_float(g, -40, 40);
                const double ulp = std::ldexp(1.0, std::ilogb(q0) - 23);
                const double target = kind == 1 ? (double)q0 + std::copysign(ulp / 2, q0) : (double)q0;
                float v = (float)(target * (double)den);
                const int nudge = (int)(g() % 5) - 2;
                for (int k = 0; k < std::abs(nudge); ++k) v = std::nextafter(v, nudge > 0 ? INFINITY : -INFINITY);
                num[j] = v;
            }
        }
        for (double rel : rels) {
            float q[3];
            if (!fast_path(den, num, q, rel)) continue;
            ++fast;
            for (int j = 0; j < 3; ++j) {
                const float ref = num[j] / den;          // IEEE float division (SSE)
                ++checked;
                if (std::memcmp(&ref, &q[j], 4) != 0) {
                    if (bad < 5)
                        std::printf("mismatch den=%a num=%a ref=%a got=%a rel=%a\n", den, num[j], ref, q[j], rel);
                    ++bad;
                }
            }
        }
    }
    std::printf("%ld %ld %.3f\n", checked, bad, (double)fast / (double)(n * 5));
    return 0;
}
