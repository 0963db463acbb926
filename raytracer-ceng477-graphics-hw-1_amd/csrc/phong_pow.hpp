// (float)pow((double)base, (double)phong), the reference's specular term
// (raytracer.cpp:414), without a full double pow for integer exponents.
//
// Plain C++ on purpose (host and device): tests/test_host.py compiles it with
// g++ and checks it against glibc pow.
//
// For an integer exponent 2 <= n <= 4096 and a finite positive base the power
// is formed by squaring in double.  Each product rounds once; an error eps in
// a factor becomes k*eps in its k-th power, so the result y carries a relative
// error below 2n * 2^-53.  glibc's pow is within one double ulp (2^-52
// relative) of the exact value.  When y lies farther than the sum of both
// bounds from either rounding boundary of its nearest float (the midpoints to
// the float's neighbours), the exact value, glibc's result and y all round to
// that float, so it is returned.  Otherwise -- and for every other exponent,
// base or an out-of-range result -- the full double pow decides, so the
// function always equals (float)pow((double)base, (double)phong).
#pragma once
#include <cmath>
#include <cfloat>

#if defined(__HIPCC__)
#define RT_PP_FN __host__ __device__ __forceinline__
#else
#define RT_PP_FN inline
#endif

namespace rtp {

RT_PP_FN bool pow_int_fast(float base, int n, float* out) {
    if (n < 2 || n > 4096 || !(base <= 4.0f)) return false;
    if (base == 0.0f) {                                    // pow(+-0, n > 0): +0, or the zero itself for odd n
        *out = (n & 1) ? base : 0.0f;
        return true;
    }
    if (!(base > 0.0f)) return false;
    double x = base, y = 1.0;
    for (int e = n; e; e >>= 1) {
        if (e & 1) y *= x;
        x *= x;
    }
    if (!(y >= 1e-300)) {
        // an exact value >= 2^-151 keeps every factor x^k (k <= n) >= 2^-151, far above the
        // double subnormals, so y would be within the error bound of it; hence the exact
        // value (and glibc's) is below 2^-151 and rounds to +0 as a float
        *out = 0.0f;
        return true;
    }
    const float f = (float)y;
    const float up = std::nextafter(f, FLT_MAX * 2.0f), dn = std::nextafter(f, -1.0f);
    if (!(up <= FLT_MAX)) return false;                    // f or its neighbour is not finite
    const double hi = 0.5 * ((double)f + (double)up);      // exact: float sums fit a double
    const double lo = 0.5 * ((double)f + (double)dn);
    const double tol = y * ((double)(2 * n + 4) * 0x1p-53);
    if (!(y - lo > tol) || !(hi - y > tol)) return false;
    *out = f;
    return true;
}

// The full double pow, out of line on the device: it needs ~55 more VGPRs than
// the shading kernels' own code and is taken only in rare cases.
#if defined(__HIPCC__)
inline __host__ __device__ __attribute__((noinline))
#else
inline
#endif
float pow_full(float base, float phong) {
    return (float)std::pow((double)base, (double)phong);
}

RT_PP_FN float phong_pow(float base, float phong) {
    if (phong == 1.0f) return base;   // glibc pow(x, 1) is x
    const int n = (int)phong;
    float f;
    if (phong >= 2.0f && phong <= 4096.0f && (float)n == phong && pow_int_fast(base, n, &f)) return f;
    return pow_full(base, phong);
}

}  // namespace rtp
