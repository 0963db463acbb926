// (float)pow((double)base, (double)phong), the reference's specular term
// (raytracer.cpp:414: `pow(std::max(0.0f, n.h), phong_exponent)` resolves to
// the C library's double pow; the float result is its conversion).
//
// Plain C++ on purpose (host and device): tests/test_host.py compiles it with
// g++ and checks it against glibc pow (tests/native/phong_pow_check.cpp).
//
// Two paths:
//
// 1. Fast path, integer exponent 2 <= n <= 4096 and a finite positive base:
//    the power by squaring in double.  Each product rounds once; an error eps
//    in a factor becomes k*eps in its k-th power, so the result y carries a
//    relative error below 2n * 2^-53.  glibc's pow is within 0.52 double ulp
//    of the exact value.  When y lies farther than the sum of both bounds from
//    either rounding boundary of its nearest float (the midpoints to the
//    float's neighbours), the exact value, glibc's result and y all round to
//    that float, so it is returned.  Otherwise (the boundary band) and for
//    every other exponent or base, path 2 decides.
//
// 2. pow_full: the power in double-double (about 2^-100 relative error),
//    rounded to double and then to float -- the reference's own two
//    roundings (glibc's pow is correctly rounded to double except within
//    ~0.02 ulp of a double rounding boundary).  Integer exponents |n| <= 2^24
//    by binary powering of exact products (TwoProd via fma); every other
//    exponent as exp(phong * log(base)) with a table-free double-double log
//    (atanh series) and exp (Taylor series), ln 2 as a triple-double.  The C
//    library's special cases (zeros, infinities, NaN, negative bases, y = 0,
//    base = 1) are glibc's.  Residual: a result within ~2^-96 (relative) of a
//    double rounding boundary can round to either neighbouring double (and
//    exact double midpoints follow ties-to-even where glibc may not); such a
//    double changes the float only if it also sits on a float rounding
//    boundary.
#pragma once
#include <cmath>
#include <cfloat>
#include <cstdint>
#include <cstring>

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

// ---------------------------------------------------------------------------
// Double-double arithmetic (value = hi + lo, |lo| <= ulp(hi)/2).  Every
// operation is written out in IEEE double operations (-ffp-contract=off keeps
// them separate); fma is used only where an exact product error is wanted.
// ---------------------------------------------------------------------------
struct DD {
    double hi, lo;
};

RT_PP_FN DD dd_two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return DD{s, (a - (s - bb)) + (b - bb)};
}
RT_PP_FN DD dd_fast_two_sum(double a, double b) {          // |a| >= |b| (or a == 0)
    const double s = a + b;
    return DD{s, b - (s - a)};
}
RT_PP_FN DD dd_two_prod(double a, double b) {
    const double p = a * b;
    return DD{p, __builtin_fma(a, b, -p)};
}
RT_PP_FN DD dd_add(DD a, DD b) {
    DD s = dd_two_sum(a.hi, b.hi);
    const DD t = dd_two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = dd_fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return dd_fast_two_sum(s.hi, s.lo);
}
RT_PP_FN DD dd_neg(DD a) { return DD{-a.hi, -a.lo}; }
RT_PP_FN DD dd_mul(DD a, DD b) {
    DD p = dd_two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return dd_fast_two_sum(p.hi, p.lo);
}
RT_PP_FN DD dd_mul_d(DD a, double b) {
    DD p = dd_two_prod(a.hi, b);
    p.lo += a.lo * b;
    return dd_fast_two_sum(p.hi, p.lo);
}
RT_PP_FN DD dd_div(DD a, DD b) {                            // three quotient digits
    const double q1 = a.hi / b.hi;
    DD r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
    const double q2 = r.hi / b.hi;
    r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
    const double q3 = r.hi / b.hi;
    return dd_add(dd_fast_two_sum(q1, q2), DD{q3, 0.0});
}
RT_PP_FN DD dd_div_d(DD a, double b) { return dd_div(a, DD{b, 0.0}); }

// 2^k for |k| <= 1022, exactly
RT_PP_FN double pp_exp2i(int k) {
    const uint64_t bits = (uint64_t)(k + 1023) << 52;
    double d;
    std::memcpy(&d, &bits, sizeof d);
    return d;
}

// ln 2 = L1 + L2 + L3 (triple-double, ~160 bits)
constexpr double kLn2_1 = 0x1.62e42fefa39efp-1;
constexpr double kLn2_2 = 0x1.abc9e3b39803fp-56;
constexpr double kLn2_3 = 0x1.7b57a079a1934p-111;

// k * ln 2 in double-double (|k| < 2^11)
RT_PP_FN DD dd_k_ln2(double k) {
    return dd_add(dd_add(dd_two_prod(k, kLn2_1), dd_two_prod(k, kLn2_2)), DD{k * kLn2_3, 0.0});
}

// ln(x) for a finite x > 0 given as a double of float precision (the base):
// x = 2^k * m with m in [sqrt(1/2), sqrt(2)); ln m = 2 atanh(f), f = (m-1)/(m+1)
// (m-1 and m+1 are exact), |f| <= 0.1716, series to f^43 (< 2^-106 relative).
RT_PP_FN DD dd_log(double x) {
    int k = 0;
    double m = x;
    while (m >= 0x1.6a09e667f3bcdp+0) { m *= 0.5; ++k; }   // sqrt(2)
    while (m < 0x1.6a09e667f3bcdp-1) { m *= 2.0; --k; }    // sqrt(1/2)
    const DD f = dd_div(DD{m - 1.0, 0.0}, DD{m + 1.0, 0.0});
    const DD s = dd_mul(f, f);
    // P(s) = sum_{j=0}^{21} s^j / (2j+1), Horner from the top
    DD p = dd_div_d(DD{1.0, 0.0}, 43.0);
#pragma unroll 1
    for (int j = 20; j >= 0; --j) p = dd_add(dd_mul(p, s), dd_div_d(DD{1.0, 0.0}, (double)(2 * j + 1)));
    DD lnm = dd_mul(f, p);
    lnm.hi *= 2.0;
    lnm.lo *= 2.0;
    return dd_add(dd_k_ln2((double)k), lnm);
}

// exp(z) for a double-double z with -110 < z < 92: z = k ln 2 + r, |r| <= 0.35,
// exp(r) = 1 + r(1 + r/2(1 + r/3(... (1 + r/24)))) (remainder < 2^-116).
RT_PP_FN DD dd_exp(DD z) {
    const double k = __builtin_rint(z.hi * 0x1.71547652b82fep+0);   // z / ln 2
    const DD r = dd_add(z, dd_neg(dd_k_ln2(k)));
    DD t{1.0, 0.0};
#pragma unroll 1
    for (int n = 24; n >= 1; --n) t = dd_add(DD{1.0, 0.0}, dd_div_d(dd_mul(r, t), (double)n));
    const double sc = pp_exp2i((int)k);                     // |k| < 160: exact scaling
    return DD{t.hi * sc, t.lo * sc};
}

// x^n for a finite x > 0 and 1 <= n <= 2^24, by binary powering of exact
// products (relative error < 2 log2(n) * 2^-104).  A non-finite hi means the
// true power overflowed the double range (x > 1): every partial product and
// every squared factor is used, and is at most the result.
RT_PP_FN DD dd_powi(double x, uint32_t n) {
    DD r{1.0, 0.0}, b{x, 0.0};
#pragma unroll 1
    for (uint32_t e = n;;) {
        if (e & 1u) {
            r = dd_mul(r, b);
            if (!(r.hi <= DBL_MAX)) return DD{HUGE_VAL, 0.0};
        }
        e >>= 1;
        if (!e) break;
        b = dd_mul(b, b);
        if (!(b.hi <= DBL_MAX)) return DD{HUGE_VAL, 0.0};
    }
    return r;
}

// pow(x, y) of the C library for float arguments, correctly rounded to double
// (up to the residual above), then to float.
#if defined(__HIPCC__)
inline __host__ __device__ __attribute__((noinline))
#else
inline
#endif
float pow_full(float base, float phong) {
    const double x = base, y = phong;
    if (y == 0.0) return 1.0f;                                   // pow(x, +-0) = 1, even for NaN x
    if (x == 1.0) return 1.0f;                                   // pow(1, y) = 1, even for NaN y
    if (x != x || y != y) return (float)(x + y);                 // NaN
    const bool yint = __builtin_floor(y) == y;                   // +-inf counts as an (even) integer here
    const bool yodd = yint && __builtin_fabs(y) < 0x1p53 && __builtin_floor(y * 0.5) != y * 0.5;
    if (__builtin_isinf(y)) {
        if (x == -1.0) return 1.0f;
        const bool small = __builtin_fabs(x) < 1.0;
        return (small == (y < 0.0)) ? (float)HUGE_VAL : 0.0f;
    }
    if (x == 0.0 || __builtin_isinf(x)) {                        // glibc: x2 = x*x, sign for odd y, 1/x2 for y < 0
        double x2 = x * x;
        if (__builtin_signbit(x) && yodd) x2 = -x2;
        return (float)(y < 0.0 ? 1.0 / x2 : x2);
    }
    double sign = 1.0;
    double ax = x;
    if (x < 0.0) {
        if (!yint) return (float)((x - x) / (x - x));            // domain error: NaN
        if (yodd) sign = -1.0;
        ax = -x;
    }
    DD r;
    if (__builtin_fabs(y) <= 0x1p24) {                           // integer or not, |y| fits the powering
        if (yint) {
            r = dd_powi(ax, (uint32_t)__builtin_fabs(y));
            if (y < 0.0) {
                if (!(r.hi <= DBL_MAX)) return (float)(sign * 0.0);
                if (r.hi < 0x1p-1000) return (float)(sign * HUGE_VAL);
                r = dd_div(DD{1.0, 0.0}, r);
            }
            return (float)(sign * r.hi);
        }
    }
    // exp(y ln x): float results lie in [2^-150, 2^128], so |y ln x| < 104 matters
    const DD l = dd_log(ax);
    const DD z = dd_mul_d(l, y);
    if (z.hi > 92.0) return (float)(sign * HUGE_VAL);
    if (z.hi < -110.0) return (float)(sign * 0.0);
    r = dd_exp(z);
    return (float)(sign * r.hi);
}

RT_PP_FN float phong_pow(float base, float phong) {
    if (phong == 1.0f) return base;   // glibc pow(x, 1) is x
    const int n = (int)phong;
    float f;
    if (phong >= 2.0f && phong <= 4096.0f && (float)n == phong && pow_int_fast(base, n, &f)) return f;
    return pow_full(base, phong);
}

}  // namespace rtp
