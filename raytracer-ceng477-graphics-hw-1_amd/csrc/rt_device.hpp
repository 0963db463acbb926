// Device-side math and intersection routines (HIP, gfx950).
//
// Bit-exact restatement contract (corrected):
//   * compiled with -ffp-contract=off (reference is SSE2 x86-64: no FMA);
//   * std::min/std::max are explicit selects ((b<a)?b:a, (a<b)?b:a) — NOT
//     fminf/fmaxf/v_min_f32, whose NaN semantics differ;
//   * every expression keeps the reference's association;
//   * IEEE-correct f32 divide and sqrt (hipcc default; never rcp/rsq);
//   * three double islands: sphere roots, acos (replaced by an exact
//     host-computed threshold, see rt_api.cpp), pow.
//   * Ray::Ray keeps the UN-normalised direction as its member
//     (raytracer.cpp:61-67: the body normalises the shadowing parameter), so
//     tests, getPoint and child order use the raw direction.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "device_layout.hpp"
#include "phong_pow.hpp"

namespace rtd {

struct V { float x, y, z; };

__device__ __forceinline__ V add(V a, V b) { return V{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V sub(V a, V b) { return V{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V mul(V a, float f) { return V{a.x * f, a.y * f, a.z * f}; }
__device__ __forceinline__ V divs(V a, float f) { return V{a.x / f, a.y / f, a.z / f}; }
__device__ __forceinline__ V neg(V a) { return V{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ V had(V a, V b) { return V{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len(V a) { return __builtin_sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
__device__ __forceinline__ V nrm(V a) { const float l = len(a); return V{a.x / l, a.y / l, a.z / l}; }
__device__ __forceinline__ float comp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }   // std::min
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }   // std::max
__device__ __forceinline__ V vclamp(V a, float lo, float hi) {                          // parser.h:81-86
    return V{smax(lo, smin(a.x, hi)), smax(lo, smin(a.y, hi)), smax(lo, smin(a.z, hi))};
}

struct Ray { V o, d, inv; };

__device__ __forceinline__ Ray make_ray(V o, V dir) {                                   // raytracer.cpp:61-67
    Ray r;
    r.o = o;
    r.d = dir;
    r.inv = V{1.0f / dir.x, 1.0f / dir.y, 1.0f / dir.z};
    return r;
}

// Ray::intersects(Box) (raytracer.cpp:101-126).  Returns exists; *t = tmin.
__device__ __forceinline__ bool box_hit(const Ray& r, const float4 lo, const float4 hi, float* t) {
    const float tx1 = (lo.x - r.o.x) * r.inv.x;
    const float tx2 = (hi.x - r.o.x) * r.inv.x;
    float tmin = smin(tx1, tx2);
    float tmax = smax(tx1, tx2);
    const float ty1 = (lo.y - r.o.y) * r.inv.y;
    const float ty2 = (hi.y - r.o.y) * r.inv.y;
    tmin = smax(tmin, smin(ty1, ty2));
    tmax = smin(tmax, smax(ty1, ty2));
    const float tz1 = (lo.z - r.o.z) * r.inv.z;
    const float tz2 = (hi.z - r.o.z) * r.inv.z;
    tmin = smax(tmin, smin(tz1, tz2));
    tmax = smin(tmax, smax(tz1, tz2));
    *t = tmin;
    return tmax >= smax(0.0f, tmin);
}

// Same test with v_min/v_max(3) instead of compare+select.  Valid only when
// no slab value can be NaN, i.e. the ray origin and 1/dir are finite
// (ray_nan_free): then min/max agree with std::min/std::max except for the
// sign of a zero result, and tmin/tmax are only ever compared (never used in
// arithmetic), where -0 == +0.  Halves the box test's instruction count.
__device__ __forceinline__ bool box_hit_fast(const Ray& r, const float4 lo, const float4 hi, float* t) {
    const float tx1 = (lo.x - r.o.x) * r.inv.x;
    const float tx2 = (hi.x - r.o.x) * r.inv.x;
    const float ty1 = (lo.y - r.o.y) * r.inv.y;
    const float ty2 = (hi.y - r.o.y) * r.inv.y;
    const float tz1 = (lo.z - r.o.z) * r.inv.z;
    const float tz2 = (hi.z - r.o.z) * r.inv.z;
    const float tmin = __builtin_fmaxf(__builtin_fmaxf(__builtin_fminf(tx1, tx2), __builtin_fminf(ty1, ty2)),
                                       __builtin_fminf(tz1, tz2));
    const float tmax = __builtin_fminf(__builtin_fminf(__builtin_fmaxf(tx1, tx2), __builtin_fmaxf(ty1, ty2)),
                                       __builtin_fmaxf(tz1, tz2));
    *t = tmin;
    return tmax >= __builtin_fmaxf(0.0f, tmin);
}

// Finite origin, finite dir (so 1/dir != 0) and finite 1/dir: every
// (bound - o) * inv is finite or +-inf, never NaN (bounds are finite).
__device__ __forceinline__ bool ray_nan_free(const Ray& r) {
    return __builtin_isfinite(r.o.x) && __builtin_isfinite(r.o.y) && __builtin_isfinite(r.o.z) &&
           __builtin_isfinite(r.d.x) && __builtin_isfinite(r.d.y) && __builtin_isfinite(r.d.z) &&
           __builtin_isfinite(r.inv.x) && __builtin_isfinite(r.inv.y) && __builtin_isfinite(r.inv.z);
}

// det (raytracer.cpp:15-19), rows m0 m1 m2.
__device__ __forceinline__ float det3(float m00, float m01, float m02, float m10, float m11, float m12,
                                      float m20, float m21, float m22) {
    return m00 * (m11 * m22 - m12 * m21) - m01 * (m10 * m22 - m12 * m20) + m02 * (m10 * m21 - m11 * m20);
}

// The three Cramer quotients n_i / den (raytracer.cpp:147, 154, 161), each the correctly rounded float
// quotient, from ONE reciprocal instead of three IEEE division sequences:
//   r = 1/den in double (the f32 reciprocal, ~2^-22, and two Newton steps: relative error
//   < 2^-52.9), q_i = RN_53(n_i * r) (relative error < 2^-51.9), then RN_24(q_i).
// Exact: for floats a, b (24-bit significands) the quotient a/b is never a rounding midpoint of
// the float grid and lies at relative distance > 2^-49 from every one (a - m b is a non-zero
// multiple of 2^min(e_a, e_m + e_b); |a/b| < 2^24 ulp), so a value within 2^-51.9 of a/b rounds to
// RN_24(a/b).  That argument needs a normal-range result; zero is exact (sign included).  Lanes
// with |den| outside [2^-100, 2^100] (or not finite) or any |q_i| < 2^-125 (zero included) take the IEEE
// divisions (a wave-uniform branch, taken only when some lane needs it).  The float results are
// checked: |RN_24(q)| >= 2^-125 implies q > 2^-126 (normal).
__device__ __forceinline__ void cramer_div3(float den, float n0, float n1, float n2, float& q0, float& q1,
                                            float& q2) {
    const double D = (double)den;
    double r = (double)__builtin_amdgcn_rcpf(den);
    double e = __builtin_fma(-D, r, 1.0);
    r = __builtin_fma(e, r, r);
    e = __builtin_fma(-D, r, 1.0);
    r = __builtin_fma(e, r, r);
    const double d0 = (double)n0 * r, d1 = (double)n1 * r, d2 = (double)n2 * r;
    q0 = (float)d0;
    q1 = (float)d1;
    q2 = (float)d2;
    const float ad = __builtin_fabsf(den);
    // (a zero quotient is exact too, but rare enough to send along: one min3 and one compare)
    const bool tiny = !(__builtin_fminf(__builtin_fminf(__builtin_fabsf(q0), __builtin_fabsf(q1)), __builtin_fabsf(q2)) >=
                        0x1p-125f);
    const bool exact = !(ad >= 0x1p-100f && ad <= 0x1p100f) || tiny;
    if (__builtin_expect(__any(exact), 0)) {
        if (exact) {
            q0 = n0 / den;
            q1 = n1 / den;
            q2 = n2 / den;
        }
    }
}

// Ray::intersects(Scene&, Triangle&) (raytracer.cpp:129-175), Cramer's rule.
// e1 = a-b, e2 = a-c (precomputed bit-identically at build time).
__device__ __forceinline__ bool tri_hit(const Ray& r, const float4 a, const float4 e1, const float4 e2, float* tout) {
    const V d = r.d;
    const float aox = a.x - r.o.x, aoy = a.y - r.o.y, aoz = a.z - r.o.z;
    const float detA = det3(e1.x, e2.x, d.x, e1.y, e2.y, d.y, e1.z, e2.z, d.z);
    float beta, gamma, t;
    cramer_div3(detA, det3(aox, e2.x, d.x, aoy, e2.y, d.y, aoz, e2.z, d.z),
                det3(e1.x, aox, d.x, e1.y, aoy, d.y, e1.z, aoz, d.z),
                det3(e1.x, e2.x, aox, e1.y, e2.y, aoy, e1.z, e2.z, aoz), beta, gamma, t);
    const float alpha = 1.0f - beta - gamma;
    *tout = t;
    return alpha >= 0 && beta >= 0 && gamma >= 0 && t >= 0.0f;
}

// (float)pow((double)base, (double)phong) (raytracer.cpp:414): phong_pow.hpp
// (integer exponents by squaring with an exact rounding test, else the double pow).
using rtp::phong_pow;

// Ray::intersects(Sphere) (raytracer.cpp:70-96) without the normal (computed
// for the winner only; it is a pure function of ray, sphere and t1).
__device__ __forceinline__ bool sphere_hit(const Ray& r, const float4 c, const float4 rr, float* tout) {
    const V oc = V{r.o.x - c.x, r.o.y - c.y, r.o.z - c.z};
    const float B = 2.0f * dot(r.d, oc);
    const float A = dot(r.d, r.d);
    const float C = dot(oc, oc) - rr.y;           // rr.y = r*r (float product, exact copy)
    const float disc = B * B - 4.0f * A * C;
    if (!(disc >= 0)) return false;
    const double sq = __builtin_sqrt((double)disc);
    const double den = (double)(2.0f * A);
    const float t1 = (float)(((double)(-B) - sq) / den);
    const float t2 = (float)(((double)(-B) + sq) / den);
    *tout = t1;
    return !(t1 < 0 && t2 < 0);
}

__device__ __forceinline__ V sphere_normal(const Ray& r, const float4 c, float radius, float t1) {
    const V p = add(r.o, mul(r.d, t1));                     // getPoint (raytracer.cpp:49-51)
    return nrm(divs(sub(p, V{c.x, c.y, c.z}), radius));     // :91
}

}  // namespace rtd
