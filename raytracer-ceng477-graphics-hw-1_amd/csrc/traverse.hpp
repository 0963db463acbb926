// Ordered-DFS BVH traversal (closest-hit and any-hit) shared by the kernels.
//
// Order contract (raytracer.cpp:177-225, 227-280): the box test happens when a
// node is popped, against the tMax current at that moment; an interior node
// pushes (far, near) where near = left (i+1) iff d[axis] > 0, so near is
// popped next.  Here the near child is not pushed and popped but kept in a
// register (`ni`) — the same visit sequence without an LDS round trip — and
// only the far child goes to the LDS stack.  Leaves test their triangles then
// their spheres in stored order; a hit replaces the best iff
// t < best.t || best.t == -1 (a negative sphere t1 can win, as in the
// reference).
//
// Stack layout: stk points at this thread's slot 0; entry e lives at
// stk[e * STRIDE] (STRIDE = threads per block) so the 64 lanes of a wave hit
// 64 distinct LDS banks whatever their depths.
#pragma once

#include "render_kernels.hpp"
#include "rt_device.hpp"

namespace rtd {

struct Work {
    uint32_t nodes = 0, tris = 0, spheres = 0;
};

struct HitRec {
    float t;
    int prim;   // leaf-prim slot of the winner, -1 = none
};

__device__ __forceinline__ float4 ld4(const void* p) { return *reinterpret_cast<const float4*>(p); }

template <bool COUNT, int STRIDE>
__device__ __forceinline__ HitRec closest_hit(const rtk::DevScene& s, const Ray& r, int* stk, Work& w) {
    HitRec best{-1.0f, -1};
    if (s.nnodes <= 0) return best;
    float tmax = FLT_MAX;
    int sp = 0;
    int ni = 0;
    while (true) {
        const float4 lo = ld4(&s.nodes[ni].minx);
        const float4 hi = ld4(&s.nodes[ni].maxx);
        if (COUNT) w.nodes++;
        float bt;
        if (box_hit(r, lo, hi, &bt) && bt <= tmax) {
            const int b = __float_as_int(hi.w);
            const int a = __float_as_int(lo.w);
            if (b >= 0) {                       // interior: a = right child, b = axis
                const bool left_first = comp(r.d, b) > 0;
                stk[sp * STRIDE] = left_first ? a : ni + 1;
                ++sp;
                ni = left_first ? ni + 1 : a;
                continue;
            }
            const int ntri = b & dl::kNtriMask;
            const int nsph = (b >> dl::kNtriBits) & dl::kMaxLeafSpheres;
            for (int i = a; i < a + ntri; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                if (COUNT) w.tris++;
                float t;
                if (tri_hit(r, pr[0], pr[1], pr[2], &t) && (t < best.t || best.t == -1.0f)) {
                    best.t = t; best.prim = i; tmax = t;
                }
            }
            for (int i = a + ntri; i < a + ntri + nsph; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                if (COUNT) w.spheres++;
                float t;
                if (sphere_hit(r, pr[0], pr[1], &t) && (t < best.t || best.t == -1.0f)) {
                    best.t = t; best.prim = i; tmax = t;
                }
            }
        }
        if (sp == 0) break;
        --sp;
        ni = stk[sp * STRIDE];
    }
    return best;
}

// Any-hit: no t pruning of boxes, stop at the first primitive with t < tlim.
template <bool COUNT, int STRIDE>
__device__ __forceinline__ bool any_hit(const rtk::DevScene& s, const Ray& r, float tlim, int* stk, Work& w) {
    if (s.nnodes <= 0) return false;
    int sp = 0;
    int ni = 0;
    while (true) {
        const float4 lo = ld4(&s.nodes[ni].minx);
        const float4 hi = ld4(&s.nodes[ni].maxx);
        if (COUNT) w.nodes++;
        float bt;
        if (box_hit(r, lo, hi, &bt)) {
            const int b = __float_as_int(hi.w);
            const int a = __float_as_int(lo.w);
            if (b >= 0) {
                const bool left_first = comp(r.d, b) > 0;
                stk[sp * STRIDE] = left_first ? a : ni + 1;
                ++sp;
                ni = left_first ? ni + 1 : a;
                continue;
            }
            const int ntri = b & dl::kNtriMask;
            const int nsph = (b >> dl::kNtriBits) & dl::kMaxLeafSpheres;
            for (int i = a; i < a + ntri; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                if (COUNT) w.tris++;
                float t;
                if (tri_hit(r, pr[0], pr[1], pr[2], &t) && t < tlim) return true;
            }
            for (int i = a + ntri; i < a + ntri + nsph; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                if (COUNT) w.spheres++;
                float t;
                if (sphere_hit(r, pr[0], pr[1], &t) && t < tlim) return true;
            }
        }
        if (sp == 0) break;
        --sp;
        ni = stk[sp * STRIDE];
    }
    return false;
}

// Winner's normal and material (Intersection::normal / material_id); *code
// names the surface for surface_normal: the triangle index (>= 0) or ~slot of
// the sphere's primitive slot.
__device__ __forceinline__ void hit_surface(const rtk::DevScene& s, const Ray& r, const HitRec& h, V* n, int* mat,
                                            int* code = nullptr) {
    const float4* pr = reinterpret_cast<const float4*>(&s.prims[h.prim]);
    const float4 p0 = pr[0];
    if (__float_as_int(p0.w) < 0) {             // sphere
        const float4 p1 = pr[1];
        *n = sphere_normal(r, p0, p1.x, h.t);
        *mat = __float_as_int(pr[2].w);
        if (code) *code = ~h.prim;
    } else {
        const float4 ts = ld4(&s.tri_shade[__float_as_int(p0.w)]);
        *n = V{ts.x, ts.y, ts.z};
        *mat = __float_as_int(ts.w);
        if (code) *code = __float_as_int(p0.w);
    }
}

// The same normal from the hit point and the surface code: a triangle's face
// normal, or a sphere's (hitp - c) / r normalised -- sphere_normal's own
// arithmetic on the same hit point (its getPoint is hitp's expression), so
// bit-identical to what hit_surface returned.
__device__ __forceinline__ V surface_normal(const rtk::DevScene& s, const V& hitp, int code) {
    if (code >= 0) {
        const float4 ts = ld4(&s.tri_shade[code]);
        return V{ts.x, ts.y, ts.z};
    }
    const float4* pr = reinterpret_cast<const float4*>(&s.prims[~code]);
    const float4 c = pr[0];
    const float rad = pr[1].x;
    return nrm(divs(sub(hitp, V{c.x, c.y, c.z}), rad));
}

// EyeRayGenerator::generate (raytracer.cpp:319-324).  (col+0.5)*su is a double
// expression in the reference whose value is the exact product of two floats,
// so the correctly rounded fp32 product is bit-identical.
__device__ __forceinline__ Ray eye_ray(const rtk::Eye& e, int row, int col) {
    const float su = ((float)col + 0.5f) * e.su;
    const float sv = ((float)row + 0.5f) * e.sv;
    const V q{e.qx, e.qy, e.qz}, u{e.ux, e.uy, e.uz}, v{e.vx, e.vy, e.vz}, eye{e.ex, e.ey, e.ez};
    const V sp = sub(add(q, mul(u, su)), mul(v, sv));
    return make_ray(eye, sub(sp, eye));
}

__device__ __forceinline__ uint32_t quantise(float x) {       // toPixel parser.h:88-93
    const float k = smax(0.0f, smin(x, 255.0f));
    return (uint32_t)__builtin_roundf(k);
}

}  // namespace rtd
