// CPU check of phong_pow.hpp against the reference's (float)pow((double)b, (double)p)
// (raytracer.cpp:414) under glibc.  Prints "<checked> <fast> <mismatches>".
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include "phong_pow.hpp"

int main(int argc, char** argv) {
    const long per = argc > 1 ? atol(argv[1]) : 200000;
    const float exps[] = {1, 2, 3, 5, 7, 10, 16, 32, 50, 64, 99, 100, 127, 128, 200, 500, 1000, 4096, 0.5f, 2.5f, 8192};
    std::mt19937_64 rng(12345);
    long checked = 0, fast = 0, bad = 0;
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
            if (std::memcmp(&got, &want, 4) != 0) {
                if (++bad < 10) std::printf("MISMATCH b=%a p=%g got=%a want=%a\n", b, p, got, want);
            }
        }
    }
    std::printf("%ld %ld %ld\n", checked, fast, bad);
    return bad != 0;
}
