// CPU check of phong_pow.hpp against the reference's (float)pow((double)b, (double)p)
// (raytracer.cpp:414) under glibc.
//
// Part 1: phong_pow (fast path + fallback) on random and typical bases for a
//         spread of exponents.
// Part 2: pow_full (the double-double fallback) on its own, for every input
//         class: the exponents {3, 50, 100, 2.5} and others, random bases,
//         bases whose power is EXACTLY a float rounding midpoint (odd mantissas
//         m with m^p of 25 significant bits; perfect squares for p = 2.5 / 0.5),
//         bases searched to put the power within a few thousand double ulps of
//         a float midpoint, and the C library's special cases.
// Prints "<checked> <fast> <mismatches> <full_checked> <near_midpoint> <exact_midpoint>".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
#include "phong_pow.hpp"

static long g_bad = 0;

static bool same(float a, float b) {
    if (a != a && b != b) return true;                   // NaN payload/sign: not observable after shading
    return std::memcmp(&a, &b, 4) == 0;
}
static void check_full(float b, float p) {
    const float want = (float)std::pow((double)b, (double)p);
    const float got = rtp::pow_full(b, p);
    if (!same(got, want) && ++g_bad < 20) std::printf("MISMATCH pow_full b=%a p=%a got=%a want=%a\n", b, p, got, want);
}

// distance of y (> 0) from the nearest float rounding midpoint, in units of ulp(y) as a double
static double midpoint_distance_ulps(double y) {
    const float f = (float)y;
    const float up = std::nextafter(f, INFINITY), dn = std::nextafter(f, 0.0f);
    const double hi = 0.5 * ((double)f + (double)up), lo = 0.5 * ((double)f + (double)dn);
    const double d = std::fmin(std::fabs(y - hi), std::fabs(y - lo));
    int e;
    std::frexp(y, &e);
    return d / std::ldexp(1.0, e - 53);
}

int main(int argc, char** argv) {
    const long per = argc > 1 ? atol(argv[1]) : 200000;
    const float exps[] = {1, 2, 3, 5, 7, 10, 16, 32, 50, 64, 99, 100, 127, 128, 200, 500, 1000, 4096, 0.5f, 2.5f, 8192};
    std::mt19937_64 rng(12345);
    long checked = 0, fast = 0;
    for (float p : exps) {
        for (long i = 0; i < per; ++i) {
            float b;
            const uint64_t r = rng();
            if (i % 4 == 0) {                        // random bit patterns in (0, 1.25]
                uint32_t u = (uint32_t)(r >> 32) % 0x3fa00000u;
                std::memcpy(&b, &u, 4);
            } else {                                 // uniform in [0, 1.0001]: typical cosines
                b = (float)((double)(r >> 11) * 0x1p-53 * 1.0001);
            }
            if (i == 0) b = 0.0f;
            if (i == 1) b = 1.0f;
            if (i == 2) b = -0.0f;
            if (i % 16 == 3) b = 0.0f;                 // smax(0, n.h) clamps often
            if (i % 16 == 5) b = (float)((double)(r >> 11) * 0x1p-53 * 0.01);   // tiny results (underflow)
            const float want = (float)std::pow((double)b, (double)p);
            float got = rtp::phong_pow(b, p), f;
            if (p != 1.0f && (float)(int)p == p && rtp::pow_int_fast(b, (int)p, &f)) ++fast;
            ++checked;
            if (!same(got, want) && ++g_bad < 20) std::printf("MISMATCH b=%a p=%g got=%a want=%a\n", b, p, got, want);
        }
    }

    // ---- part 2: the double-double fallback on its own ----
    long full = 0, near_mid = 0, exact_mid = 0;
    const float fexps[] = {3, 50, 100, 2.5f, 0.5f, 1.5f, 7.25f, 33.3f, 0.1f, 4097, 123457, 0x1p25f, -2, -2.5f, -50, 1e-3f};
    const long fper = per / 4;
    for (float p : fexps) {
        for (long i = 0; i < fper; ++i) {
            const uint64_t r = rng();
            float b;
            if (i % 3 == 0) b = (float)((double)(r >> 11) * 0x1p-53);                  // [0, 1)
            else if (i % 3 == 1) { uint32_t u = (uint32_t)(r >> 33) % 0x40800000u; std::memcpy(&b, &u, 4); }  // (0, 4]
            else b = (float)(1.0 + ((double)(r >> 11) * 0x1p-53 - 0.5) * 0x1p-10);    // near 1: deep powers
            check_full(b, p);
            ++full;
        }
    }
    // exact float midpoints: b = m * 2^e with m odd and m^p of exactly 25 significant bits
    struct Case { int p; int mlo, mhi; };
    const Case cases[] = {{2, 4097, 5792}, {3, 257, 322}, {5, 29, 31}};
    for (const Case& c : cases)
        for (int m = c.mlo | 1; m <= c.mhi; m += 2)
            for (int e = -20; e <= 8; ++e) {
                const float b = std::ldexp((float)m, e) / (float)(1 << 12);
                const double y = std::pow((double)b, (double)c.p);
                if (midpoint_distance_ulps(y) == 0.0) ++exact_mid;
                check_full(b, (float)c.p);
                const float want = (float)y;
                if (!same(rtp::phong_pow(b, (float)c.p), want) && ++g_bad < 20)
                    std::printf("MISMATCH phong_pow(midpoint) b=%a p=%d\n", b, c.p);
                ++full;
            }
    // p = 2.5 and 0.5 on perfect squares: b = m^2 2^(2e) gives b^2.5 = m^5 2^(5e) (exact midpoints for m = 29, 31)
    for (int m = 1; m <= 4097; m += 2)
        for (int e = -6; e <= 3; ++e) {
            const float b = std::ldexp((float)m * (float)m, 2 * e);
            for (float p : {2.5f, 0.5f, 1.5f}) {
                const double y = std::pow((double)b, (double)p);
                if (std::isfinite(y) && y > 0 && midpoint_distance_ulps(y) == 0.0) ++exact_mid;
                check_full(b, p);
                ++full;
            }
        }
    // searched near-midpoint bases: float neighbours of b0 = T^(1/p) for random float midpoints T
    for (float p : {3.0f, 50.0f, 100.0f, 2.5f}) {
        for (long i = 0; i < fper; ++i) {
            const uint64_t r = rng();
            const double T = std::ldexp(1.0 + (double)(r >> 11) * 0x1p-53, -(int)(r % 40));
            float b = (float)std::pow(T, 1.0 / p);
            uint32_t u;
            std::memcpy(&u, &b, 4);
            u += (uint32_t)(i % 33) - 16u;
            std::memcpy(&b, &u, 4);
            const double y = std::pow((double)b, (double)p);
            if (y > 0 && std::isfinite(y) && midpoint_distance_ulps(y) < 4096.0) ++near_mid;
            check_full(b, p);
            ++full;
        }
    }
    // special cases of the C library
    const float sp[] = {0.0f, -0.0f, 1.0f, -1.0f, 2.0f, -2.0f, 0.5f, -0.5f, INFINITY, -INFINITY, NAN, 0x1p-149f, 3.0f};
    for (float b : sp)
        for (float p : sp) {
            check_full(b, p);
            ++full;
        }
    std::printf("%ld %ld %ld %ld %ld %ld\n", checked, fast, g_bad, full, near_mid, exact_mid);
    return g_bad != 0;
}
