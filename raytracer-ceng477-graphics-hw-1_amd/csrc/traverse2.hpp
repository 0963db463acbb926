// Ordered-DFS traversal over the child-pair layout (device_layout.hpp dl::Pair).
//
// Same visit order, same pruning, same counts as the reference's stack walk
// (raytracer.cpp:177-280), re-timed for the GPU:
//   * expanding an interior node loads ONE 64-B pair and box-tests both
//     children at once (two independent slab tests -> ILP); a child box that
//     misses is never pushed, so it costs no further load or LDS traffic;
//   * the near child (left iff d[axis] > 0) continues in registers; only the
//     far child is pushed, with its slab tmin.  A box's tmin does not depend
//     on tMax, so testing it early and comparing `bt <= tMax` when the entry is
//     popped is exactly the reference's test-at-pop (closest-hit only;
//     any-hit has no t pruning);
//   * counters: the reference counts a box test per pop.  Closest-hit pops
//     every pushed node, so each expansion counts 2.  Any-hit can stop early,
//     so in COUNT builds missed far children are pushed (flagged) and counted
//     only if popped before the first hit — exactly the reference's count.
//
// LDS stack: entry e of this thread at stk[e * STRIDE], 8 B {info, tmin bits}.
#pragma once

#include "render_kernels.hpp"
#include "rt_device.hpp"
#include "traverse.hpp"

namespace rtd {

__device__ __forceinline__ void leaf_range(const rtk::DevScene& s, int info, int* start, int* count) {
    const int c = (info >> dl::kLeafCountShift) & dl::kLeafMaxCount;
    const int st = info & dl::kLeafStartMask;
    if (c != 0) {
        *start = st;
        *count = c;
    } else {
        const dl::LeafBig b = s.leaf_big[st];
        *start = b.start;
        *count = b.count;
    }
}

template <bool COUNT, int STRIDE>
__device__ __forceinline__ HitRec closest_hit2(const rtk::DevScene& s, const Ray& r, int2* stk, Work& w) {
    HitRec best{-1.0f, -1};
    if (s.nnodes <= 0) return best;
    float tmax = FLT_MAX;
    {
        float bt;
        if (COUNT) w.nodes++;
        const float4 lo = make_float4(s.root_lo[0], s.root_lo[1], s.root_lo[2], 0.0f);
        const float4 hi = make_float4(s.root_hi[0], s.root_hi[1], s.root_hi[2], 0.0f);
        if (!(box_hit(r, lo, hi, &bt) && bt <= tmax)) return best;
    }
    int cur = s.root_info;
    int sp = 0;
    while (true) {
        if (cur >= 0) {
            // expand interior node: both children from one pair record
            const float4* P = reinterpret_cast<const float4*>(&s.pairs[cur]);
            const float4 l0 = P[0], l1 = P[1], r0 = P[2], r1 = P[3];
            if (COUNT) w.nodes += 2;
            float tl, tr;
            const bool hl = box_hit(r, l0, l1, &tl);
            const bool hr = box_hit(r, r0, r1, &tr);
            const bool left_first = comp(r.d, __float_as_int(l1.w)) > 0;
            const int il = __float_as_int(l0.w), ir = __float_as_int(r0.w);
            const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
            const float tn = left_first ? tl : tr, tf = left_first ? tr : tl;
            const int in_ = left_first ? il : ir, if_ = left_first ? ir : il;
            if (hf) {
                stk[sp * STRIDE] = make_int2(if_, __float_as_int(tf));
                ++sp;
            }
            if (hn && tn <= tmax) {
                cur = in_;
                continue;
            }
        } else {
            int a, cnt;
            leaf_range(s, cur, &a, &cnt);
            for (int i = a; i < a + cnt; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                const float4 p0 = pr[0], p1 = pr[1];
                float t;
                bool h;
                if (__float_as_int(p0.w) >= 0) {
                    if (COUNT) w.tris++;
                    h = tri_hit(r, p0, p1, pr[2], &t);
                } else {
                    if (COUNT) w.spheres++;
                    h = sphere_hit(r, p0, p1, &t);
                }
                if (h && (t < best.t || best.t == -1.0f)) {
                    best.t = t;
                    best.prim = i;
                    tmax = t;
                }
            }
        }
        // pop until an entry passes its (deferred) tMax check
        bool found = false;
        while (sp > 0) {
            --sp;
            const int2 e = stk[sp * STRIDE];
            if (__int_as_float(e.y) <= tmax) {
                cur = e.x;
                found = true;
                break;
            }
        }
        if (!found) break;
    }
    return best;
}

template <bool COUNT, int STRIDE>
__device__ __forceinline__ bool any_hit2(const rtk::DevScene& s, const Ray& r, float tlim, int2* stk, Work& w) {
    if (s.nnodes <= 0) return false;
    {
        float bt;
        if (COUNT) w.nodes++;
        const float4 lo = make_float4(s.root_lo[0], s.root_lo[1], s.root_lo[2], 0.0f);
        const float4 hi = make_float4(s.root_hi[0], s.root_hi[1], s.root_hi[2], 0.0f);
        if (!box_hit(r, lo, hi, &bt)) return false;
    }
    int cur = s.root_info;
    int sp = 0;
    while (true) {
        if (cur >= 0) {
            const float4* P = reinterpret_cast<const float4*>(&s.pairs[cur]);
            const float4 l0 = P[0], l1 = P[1], r0 = P[2], r1 = P[3];
            float tl, tr;
            const bool hl = box_hit(r, l0, l1, &tl);
            const bool hr = box_hit(r, r0, r1, &tr);
            const bool left_first = comp(r.d, __float_as_int(l1.w)) > 0;
            const int il = __float_as_int(l0.w), ir = __float_as_int(r0.w);
            const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
            const int in_ = left_first ? il : ir, if_ = left_first ? ir : il;
            if (COUNT) w.nodes++;                       // near child popped now
            if (hf || COUNT) {                          // far child: popped later (if at all)
                stk[sp * STRIDE] = make_int2(if_, hf ? 1 : 0);
                ++sp;
            }
            if (hn) {
                cur = in_;
                continue;
            }
        } else {
            int a, cnt;
            leaf_range(s, cur, &a, &cnt);
            for (int i = a; i < a + cnt; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                const float4 p0 = pr[0], p1 = pr[1];
                float t;
                bool h;
                if (__float_as_int(p0.w) >= 0) {
                    if (COUNT) w.tris++;
                    h = tri_hit(r, p0, p1, pr[2], &t);
                } else {
                    if (COUNT) w.spheres++;
                    h = sphere_hit(r, p0, p1, &t);
                }
                if (h && t < tlim) return true;
            }
        }
        bool found = false;
        while (sp > 0) {
            --sp;
            const int2 e = stk[sp * STRIDE];
            if (COUNT) w.nodes++;                       // popped (box tested) in the reference
            if (e.y) {
                cur = e.x;
                found = true;
                break;
            }
        }
        if (!found) break;
    }
    return false;
}

}  // namespace rtd
