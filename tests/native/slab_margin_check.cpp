// Property check of the wide trees' fused slab arithmetic (traverse2.hpp
// wide_slabs, RT_SLAB_FMA): for random wide-node planes (fp16 offsets on a
// power-of-two scale, origins and scales over many magnitudes) and random rays
// (directions down to |d| = 2^-64, origins far from the node), the fused near
// value t = fma(h, 2^e*inv, (origin-o)*inv - M) must never exceed the exact
// decode-then-slab value RN(RN(RN(origin + h*2^e) - o) * inv), and the fused
// far value (+M) never fall below it.  The exact form is what the host's
// containment check and the monotonicity argument are stated for, so this
// bound is what makes the fused test conservative.  Plain C++ with the same
// float operations as the device (fma = one rounding; -ffp-contract=off).
// Prints "<pairs checked> <violations> <smallest fraction of the margin left>".
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

static float h16(uint16_t b) {
    const int ex = (b >> 10) & 31, man = b & 1023;
    return ex == 0 ? std::ldexp((float)man, -24) : std::ldexp((float)(1024 + man), ex - 25);
}

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 2000000;
    std::mt19937_64 rng(20261016);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long checked = 0, bad = 0;
    double worst = 1e300;   // smallest (exact - fused_near) / M and (fused_far - exact) / M: the margin left
    for (long i = 0; i < n; ++i) {
        // node: origin G, scale S = 2^e (|G| <= 2^60, S <= 2^40, as the host enforces)
        const int eg = (int)(U(rng) * 80.0) - 40;
        const float G = (float)((U(rng) * 2.0 - 1.0) * std::ldexp(1.0, eg));
        const int es = std::max(-126, std::min(40, eg - 15 - (int)(U(rng) * 12.0)));
        const float S = std::ldexp(1.0f, es);
        // ray: origin within a few node extents .. far away; |inv| up to 2^64
        const int eo = eg + (int)(U(rng) * 30.0) - 10;
        const float O = (float)((U(rng) * 2.0 - 1.0) * std::ldexp(1.0, std::min(60, eo)));
        const int ed = -(int)(U(rng) * 64.0);
        float d = (float)((U(rng) * 2.0 - 1.0) * std::ldexp(1.0, ed));
        if (d == 0.0f) d = 1.0f;
        const float I = 1.0f / d;
        if (!(std::fabs(I) <= 0x1p64f)) continue;
        // the per-node, per-axis margin (device code, same operation order)
        const float si = S * I;
        const float z = G - O;
        const float oi = z * I;
        const float c = std::fma(S, 0x1p-5f, std::fabs(G) * 0x1p-23f);
        const float m = std::fma(std::fabs(z), 6.0f * 0x1p-23f, c);
        const float M = std::fma(m, std::fabs(I), 0x1p-126f);
        const float on = oi - M, of = oi + M;
        for (int k = 0; k < 8; ++k) {
            uint16_t code = (uint16_t)(rng() % 0x7bffu);
            if (k == 0) code = 0;
            if (code != 0 && code < 1024) code += 1024;         // the host never emits fp16 denormals
            const float h = h16(code);
            const float P = std::fma(h, S, G);                   // the exact form's decoded plane
            const float t_exact = (P - O) * I;
            const float t_near = std::fma(h, si, on), t_far = std::fma(h, si, of);
            ++checked;
            if (!(t_near <= t_exact) || !(t_far >= t_exact) || std::isnan(t_near) || std::isnan(t_far)) {
                if (++bad < 10)
                    std::printf("VIOLATION G=%a S=%a O=%a I=%a h=%a exact=%a near=%a far=%a M=%a\n", G, S, O, I, h,
                                t_exact, t_near, t_far, M);
            } else if (M > 0 && t_exact != 0.0f) {
                worst = std::min(worst, std::min((double)(t_exact - t_near), (double)(t_far - t_exact)) / M);
            }
        }
    }
    std::printf("%ld %ld %.3f\n", checked, bad, worst);
    return bad != 0;
}
