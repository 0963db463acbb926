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

// The primitives [a, a+cnt) of a leaf, each passed to f(i, p0, p1, p2) with
// all three of its float4 already loaded (a sphere ignores p2), stopping when
// f returns true.  The three loads of a primitive are issued together (left
// to itself the compiler sinks p2 - and parts of p1 - into the triangle branch,
// a second dependent round trip), and the next primitive's loads are in flight
// while the current one is tested.
#ifndef RT_CLOSEST_PIPE
#define RT_CLOSEST_PIPE 0     // closest-hit leaves through for_prims too
#endif
#ifndef RT_PRIM_PREFETCH
#define RT_PRIM_PREFETCH 1
#endif
__device__ __forceinline__ void prim_ready(const float4& a, const float4& b, const float4& c) {
    asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(c.x),
                 "v"(c.y), "v"(c.z), "v"(c.w));
}
template <class F>
__device__ __forceinline__ bool for_prims(const rtk::DevScene& s, int a, int cnt, F&& f) {
    if (cnt <= 0) return false;
    const float4* base = reinterpret_cast<const float4*>(s.prims);
    float4 c0 = base[3 * a], c1 = base[3 * a + 1], c2 = base[3 * a + 2];
    for (int i = a; i < a + cnt; ++i) {
        prim_ready(c0, c1, c2);
        const float4 p0 = c0, p1 = c1, p2 = c2;
#if RT_PRIM_PREFETCH
        const int nx = min(i + 1, a + cnt - 1);
#else
        const int nx = i + 1;
        if (nx < a + cnt)
#endif
        { c0 = base[3 * nx]; c1 = base[3 * nx + 1]; c2 = base[3 * nx + 2]; }
        if (f(i, p0, p1, p2)) return true;
    }
    return false;
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

// ---------------------------------------------------------------------------
// Resumable form of the same two walks, one node expansion (or one leaf) per
// call, for persistent kernels that refill finished lanes with new rays.
// Pairs [0, s.top_pairs) (the top levels) are read from an LDS copy.
// ---------------------------------------------------------------------------
struct Walk {
    const dl::Pair* tree;   // pair array the walk indexes (BVH or binary occlusion tree); null: a 4-wide tree
    int cur;       // node to process (pair/quad index or leaf code)
    int sp;        // stack depth
    float tmax;    // closest-hit pruning bound (the reference's tMax)
    HitRec best;   // closest-hit result so far
    bool fast;     // ray_nan_free: box tests may use v_min/v_max
    int sgn;       // closest hit on the reference-order wide nodes: bit a set iff d[a] > 0
    int steps;     // step calls of this walk (walk_runaway)
};

// Always-on bound on one walk's step calls.  A DFS pops each node at most
// once, so a walk takes at most as many expanding steps as its tree has nodes
// and leaves, plus postponed steps (leaf_postponed: a lane waits only while
// other lanes of its wave expand); s.walk_cap = 64 x that.  A walk that
// exceeds it can only be a broken tree or a miscompiled walk: it is ended,
// and the scene's device error word is set, which the host turns into
// RT_ERR_LIMIT instead of a kernel that never finishes.
__device__ __forceinline__ bool walk_runaway(const rtk::DevScene& s, Walk& k) {
    if (++k.steps <= s.walk_cap) return false;
    __hip_atomic_fetch_or(s.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Both child boxes of a pair; the min/max form when every active lane's ray
// is NaN-free (wave-uniform branch, so no divergence between the two forms).
__device__ __forceinline__ void box_pair(const Ray& r, bool fast, const float4 l0, const float4 l1, const float4 r0,
                                         const float4 r1, bool& hl, bool& hr, float& tl, float& tr) {
    if (__all(fast)) {
        hl = box_hit_fast(r, l0, l1, &tl);
        hr = box_hit_fast(r, r0, r1, &tr);
    } else {
        hl = box_hit(r, l0, l1, &tl);
        hr = box_hit(r, r0, r1, &tr);
    }
}

// Memory policies.  The walks are templated on
//   FETCH::pair(s, p, l0, l1, r0, r1)    read child pair p
//   STK::put(i, v) / STK::at(i)           per-lane stack entry i
// Entry {info, tmin bits} (closest) or {info, hit flag} (any).  LDS-backed
// policies must name their __shared__ arrays directly (not through a stored
// generic pointer), or hipcc falls back to flat loads that wait on both
// vmcnt and lgkmcnt — see pathchain.hip.
struct FetchGlobal {
    __device__ static __forceinline__ void pair(const rtk::DevScene& s, int p, float4& l0, float4& l1, float4& r0,
                                                float4& r1) {
        const float4* q = reinterpret_cast<const float4*>(&s.pairs[p]);
        l0 = q[0]; l1 = q[1]; r0 = q[2]; r1 = q[3];
    }
};

// Fetch from the walk's own tree (BVH or occlusion tree).
__device__ __forceinline__ void fetch_pair(const Walk& k, float4& l0, float4& l1, float4& r0, float4& r1) {
    const float4* q = reinterpret_cast<const float4*>(&k.tree[k.cur]);
    l0 = q[0]; l1 = q[1]; r0 = q[2]; r1 = q[3];
}

// Private (scratch) stack whose top entry lives in registers.  The walks use
// it strictly LIFO: put(sp, v) then ++sp (push), --sp then at(sp) (pop).  A
// pop returns the register copy at once and starts the scratch load of the
// entry below, which has completed by the time it is needed (after the next
// node fetch), so pops no longer put a scratch round trip on the walk's
// dependency chain.
struct StackPriv {
    int2 e[dl::kMaxStack];   // entries [0, sp-1); entry sp-1 is `top`
    int2 top;
    __device__ __forceinline__ void put(int i, int2 v) {
        if (i > 0) e[i - 1] = top;
        top = v;
    }
    __device__ __forceinline__ int2 at(int i) {
        const int2 v = top;
        if (i > 0) top = e[i - 1];
        return v;
    }
};

// Rays the wide trees' fused slab arithmetic (wide_slabs, RT_SLAB_FMA) takes:
// NaN-free and |o|, |1/d| <= 2^64 per axis, so with the host's bounds on the
// nodes (|origin| <= 2^60, scale <= 2^40) no product or margin can overflow.
// Others walk the binary trees (never seen in practice: |d| < 2^-64).
__device__ __forceinline__ bool wide_ray_ok(const Ray& r) {
    constexpr float B = 0x1p64f;
    return __builtin_fabsf(r.o.x) <= B && __builtin_fabsf(r.o.y) <= B && __builtin_fabsf(r.o.z) <= B &&
           __builtin_fabsf(r.inv.x) <= B && __builtin_fabsf(r.inv.y) <= B && __builtin_fabsf(r.inv.z) <= B;
}

// Root test (the reference's first pop).  false: nothing to traverse.
// Any-hit pops test the box only (raytracer.cpp:268-271); closest-hit also
// needs bt <= tMax (:184), which prunes a NaN bt.
// Any-hit walks of NaN-free rays use the occlusion tree and closest-hit walks
// the reference tree's wide form outside counting passes (exact: see
// build_shadow_tree and wide_closest_step); reference counting passes and
// other rays walk the reference BVH.  Production-fetch counting passes
// (s.count_prod) walk exactly like the production kernels and count, in
// w.nodes, the BYTES each walk fetches (bench.py roofline).
template <bool COUNT>
__device__ __forceinline__ bool walk_begin(const rtk::DevScene& s, const Ray& r, Walk& k, Work& w,
                                           bool any = false) {
    k.best = HitRec{-1.0f, -1};
    k.tmax = FLT_MAX;
    k.sp = 0;
    k.steps = 0;
    k.fast = ray_nan_free(r);
    const bool wide_ok = k.fast && wide_ray_ok(r);    // the wide trees' slab arithmetic (wide_slabs)
    if (s.nnodes <= 0) return false;
    if (COUNT && !s.count_prod) w.nodes++;    // the reference's root pop (the root box is a kernel argument)
    float bt;
    if ((!COUNT || s.count_prod) && any && wide_ok && s.use_stree == 2) {
        k.tree = nullptr;                    // the occlusion tree's wide form (wide_any_step)
        k.cur = s.swroot;
        return true;
    }
    if ((!COUNT || s.count_prod) && any && k.fast && s.use_stree) {
        k.tree = s.spairs;
        k.cur = s.sroot_info;
        const float4 lo = make_float4(s.sroot_lo[0], s.sroot_lo[1], s.sroot_lo[2], 0.0f);
        const float4 hi = make_float4(s.sroot_hi[0], s.sroot_hi[1], s.sroot_hi[2], 0.0f);
        return box_hit(r, lo, hi, &bt);
    }
    if ((!COUNT || s.count_prod) && !any && wide_ok && s.use_wide) {
        k.tree = nullptr;                    // the reference tree's wide form, reference order
        k.cur = s.wroot;
        k.sgn = (r.d.x > 0.0f ? 1 : 0) | (r.d.y > 0.0f ? 2 : 0) | (r.d.z > 0.0f ? 4 : 0);
        return true;
    }
    k.tree = s.pairs;
    k.cur = s.root_info;
    const float4 lo = make_float4(s.root_lo[0], s.root_lo[1], s.root_lo[2], 0.0f);
    const float4 hi = make_float4(s.root_hi[0], s.root_hi[1], s.root_hi[2], 0.0f);
    return box_hit(r, lo, hi, &bt) && (any || bt <= k.tmax);
}

// walk_begin for the timed kernels, whose rays have already passed defer_closest / defer_any (NaN-free, in
// range of the wide trees' slab test, the wide trees built): the wide-tree branch only, so the production
// walkers carry no root box, pair pointers or binary-tree set-up (their kernel arguments otherwise stayed
// live in SGPRs across the walk loops).  false: nothing to traverse.
__device__ __forceinline__ bool walk_begin_wide(const rtk::DevScene& s, const Ray& r, Walk& k, bool any = false) {
    k.best = HitRec{-1.0f, -1};
    k.tmax = FLT_MAX;
    k.sp = 0;
    k.steps = 0;
    k.fast = true;
    k.tree = nullptr;
    k.cur = any ? s.swroot : s.wroot;
    k.sgn = (r.d.x > 0.0f ? 1 : 0) | (r.d.y > 0.0f ? 2 : 0) | (r.d.z > 0.0f ? 4 : 0);
    return s.nnodes > 0;
}

// Child boxes of a wide node (dl::Wide), slab-tested against a NaN-free ray.
typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2v h2_to_f2(uint32_t w) {
    return f2v{(float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu)),
               (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16))};
}

struct WideNode {
    float4 q[7];     // dw 0-27: header, planes, child codes
};
__device__ __forceinline__ void wide_load(const dl::Wide* nodes, int i, WideNode& n) {
    const float4* N = reinterpret_cast<const float4*>(&nodes[i]);
#pragma unroll
    for (int j = 0; j < 7; ++j) n.q[j] = N[j];
}
__device__ __forceinline__ uint32_t wide_dw(const WideNode& n, int d) {
    const float4 v = n.q[d >> 2];
    const int c = d & 3;
    return __float_as_uint(c == 0 ? v.x : (c == 1 ? v.y : (c == 2 ? v.z : v.w)));
}
// v_fma_mix_f32: fma(f16 half of w (low or high), a, b) in f32, one rounding
// (the f16 -> f32 conversion is exact).
template <int HI>
__device__ __forceinline__ float fma_mix_h(uint32_t w, float a, float b) {
    float r;
    if (HI)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(a), "v"(b));
    else
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(w), "v"(a), "v"(b));
    return r;
}

// Entry / exit t of every slot box (slots outside the mask: garbage).
//
// RT_SLAB_FMA (default): t = fma(h, 2^e * inv, (origin - o) * inv -/+ M), one
// v_fma_mix_f32 per plane, where M is a per-node, per-axis margin that makes
// the result a bound on the exact form below: with u = 2^-24, X = origin + h*2^e
// - o, the exact form's t_x = RN(RN(RN(origin + h*2^e) - o) * inv) is within
// |inv| u (|origin| + |h 2^e| + 2.0001 |X|) of X * inv, and the fused form
// within |inv| (2.0001 u |origin - o| + u |t|) of (X * inv -/+ M); with
// h * 2^e <= 2^16 * 2^e (fp16 offsets < 2^16) both stay inside
// M = |inv| 2^-23 (6 |origin - o| + |origin| + 2^18 2^e) + 2^-126
// (twice the first-order sum, which also absorbs the roundings of M itself).
// So the fused near value is <= the exact near value and the fused far value
// >= the exact far value: the test is conservative wherever the exact form's
// is (its argument is at the top of this block), the boxes only grow, and
// every leaf is still tested exactly.  No overflow, no NaN: |o|, |inv| <= 2^64
// (wide_ray_ok) and the host's node bounds (|origin| <= 2^60, 2^e <= 2^40).
//
// Otherwise the exact form: the fp16 offset converted to f32 (exact), then
// origin + h * 2^e as one fma (h * 2^e exact; the host checks containment with
// the same fma), then box_hit_fast's plane arithmetic (p - o) * inv, two
// children per packed instruction.
//
// Both forms choose the near plane of each axis up front by the sign of inv
// (the axis's lo and hi dwords swap) instead of by a min/max per child: with o,
// inv and the planes finite, lo <= hi gives (lo - o) * inv <= (hi - o) * inv for
// inv > 0 and >= for inv < 0 (rounding is monotone), so the near value is
// exactly box_hit_fast's min and the far value its max (up to the sign of a
// zero, which no comparison sees).
#ifndef RT_SLAB_FMA
#define RT_SLAB_FMA 1
#endif
__device__ __forceinline__ void wide_slabs(const WideNode& n, const Ray& r, float* tmn, float* tmx) {
    constexpr int W = dl::kWideSlots;
    const uint32_t ex = wide_dw(n, 3);
    const float sc[3] = {__uint_as_float((ex & 255u) << 23), __uint_as_float(((ex >> 8) & 255u) << 23),
                         __uint_as_float(((ex >> 16) & 255u) << 23)};
    const float org[3] = {n.q[0].x, n.q[0].y, n.q[0].z};
    const float ro[3] = {r.o.x, r.o.y, r.o.z}, ri[3] = {r.inv.x, r.inv.y, r.inv.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const bool neg = __float_as_int(ri[a]) < 0;   // near plane: lo for inv > 0, hi for inv < 0
#if RT_SLAB_FMA
        const float si = sc[a] * ri[a];                                   // exact (power of two)
        const float z = org[a] - ro[a];
        const float oi = z * ri[a];
        const float c = __builtin_fmaf(sc[a], 0x1p-5f, __builtin_fabsf(org[a]) * 0x1p-23f);
        const float m = __builtin_fmaf(__builtin_fabsf(z), 6.0f * 0x1p-23f, c);
        const float M = __builtin_fmaf(m, __builtin_fabsf(ri[a]), 0x1p-126f);
        const float on = oi - M, of = oi + M;
#pragma unroll
        for (int pr = 0; pr < W / 2; ++pr) {            // slots 2pr, 2pr+1
            const uint32_t lw = wide_dw(n, 4 + a * 3 + pr), hw = wide_dw(n, 4 + 9 + a * 3 + pr);
            const uint32_t nw = neg ? hw : lw, fw = neg ? lw : hw;
            const float tn[2] = {fma_mix_h<0>(nw, si, on), fma_mix_h<1>(nw, si, on)};
            const float tf[2] = {fma_mix_h<0>(fw, si, of), fma_mix_h<1>(fw, si, of)};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c2 = 2 * pr + h;
                tmn[c2] = a == 0 ? tn[h] : __builtin_fmaxf(tmn[c2], tn[h]);
                tmx[c2] = a == 0 ? tf[h] : __builtin_fminf(tmx[c2], tf[h]);
            }
        }
#else
        const f2v s2 = {sc[a], sc[a]}, o2 = {org[a], org[a]}, rr = {ro[a], ro[a]}, iv = {ri[a], ri[a]};
#pragma unroll
        for (int pr = 0; pr < W / 2; ++pr) {            // slots 2pr, 2pr+1
            const uint32_t lw = wide_dw(n, 4 + a * 3 + pr), hw = wide_dw(n, 4 + 9 + a * 3 + pr);
            const uint32_t nw = neg ? hw : lw, fw = neg ? lw : hw;
            const f2v tn = (__builtin_elementwise_fma(h2_to_f2(nw), s2, o2) - rr) * iv;
            const f2v tf = (__builtin_elementwise_fma(h2_to_f2(fw), s2, o2) - rr) * iv;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = 2 * pr + h;
                tmn[c] = a == 0 ? tn[h] : __builtin_fmaxf(tmn[c], tn[h]);
                tmx[c] = a == 0 ? tf[h] : __builtin_fminf(tmx[c], tf[h]);
            }
        }
#endif
    }
}
__device__ __forceinline__ int wide_code(const WideNode& n, int c) { return (int)wide_dw(n, 22 + c); }

// Any-hit slot validity, tmx >= max(0, tmn), with the max as one v_max_f32 on the slab values.  Written
// as fmaxf, the compiler regroups max(0, max(x, y, z)) as max3(max(x, y), z, 0) and quiets both inputs
// of the two-input max first (v_max_f32 v, v, v: fma_mix_h's results come from asm, so it cannot prove
// them canonical) -- 12 extra instructions per wide any-hit step.  Same result: arithmetic never
// yields a signalling NaN, which is all the quieting would change.
__device__ __forceinline__ bool any_slot_valid(float tmn, float tmx) {
    float m;
    asm("v_max_f32 %0, 0, %1" : "=v"(m) : "v"(tmn));
    return tmx >= m;
}

// Primitives of a leaf record (header at L[0..1], prims from L[2]); the first
// one is passed in already loaded, the next one is in flight while the
// current one is tested.  f(slot, p0, p1, p2) with slot = its Prim[] index;
// stops when f returns true.
template <class F>
__device__ __forceinline__ bool for_leaf_prims(const float4* L, int slot0, int cnt, float4 c0, float4 c1, float4 c2,
                                               F&& f) {
    const float4* base = L + 2;
    for (int j = 0; j < cnt; ++j) {
        prim_ready(c0, c1, c2);
        const float4 p0 = c0, p1 = c1, p2 = c2;
        const int nx = min(j + 1, cnt - 1);
        c0 = base[3 * nx];
        c1 = base[3 * nx + 1];
        c2 = base[3 * nx + 2];
        if (f(slot0 + j, p0, p1, p2)) return true;
    }
    return false;
}

// Leaf postponing (SIMD efficiency): the interior and leaf branches of a step
// are both executed whenever the wave's walking lanes straddle them, so a lane
// holding a leaf record skips steps while fewer than leaf_wait/64 of the
// walking lanes hold one; the others' interior steps then run alone.  The
// visit sequence of every lane is unchanged.
__device__ __forceinline__ bool leaf_postponed(int wait, const Walk& k) {
    if (wait <= 0) return false;
    const unsigned long long lm = __ballot(k.cur < 0), am = __ballot(1);
    return k.cur < 0 && __popcll(lm) * 64 < __popcll(am) * wait;
}

// One step of the closest-hit walk over the reference-order wide nodes
// (host_scene.cpp build_ref_wide), NaN-free rays only; true when finished
// (result in k.best).  Exactly the reference's walk (raytracer.cpp:177-225),
// re-timed:
//   * order: a node's slots are visited in the reference's DFS order (the
//     left child first iff d[axis] > 0 at every node of the collapsed levels;
//     the node stores each slot's rank per octant of d), the first passing
//     slot next, the other passing ones pushed behind it, highest rank
//     deepest;
//   * pruning: a slot passes when its (conservative, quantized) box is hit
//     with entry t <= tMax, re-checked against the then-current tMax when
//     popped; a leaf record's EXACT box is tested like the reference's leaf
//     pop (hit and entry t <= tMax) before its primitives, which are tested
//     in stored order with the reference's update rule (:210-222);
//   * why that is exact: boxes nest (a child's exact box lies in its
//     parent's, a quantized box contains its exact box) and for a NaN-free
//     ray the slab test is monotone under nesting, so a leaf whose exact test
//     passes at its pop has every ancestor passing at its earlier pop (larger
//     or equal tMax); a subtree the reference prunes (box missed, or entry
//     > tMax) contains only leaves whose exact test fails here too.  Leaves are
//     therefore tested in the reference's order with the reference's tMax,
//     so every update - and the final (t, primitive) - is the reference's.
//     Only interior work differs (skipped intermediate boxes, conservative
//     quantized tests).  No tolerance, no restart.
template <bool COUNT, class STK>
__device__ __forceinline__ bool wide_closest_step(const rtk::DevScene& s, const Ray& r, STK& stk, Walk& k,
                                                  Work& w) {
    constexpr int W = dl::kWideSlots;
    if (!COUNT && leaf_postponed(s.leaf_wait, k)) return false;
    if (k.cur >= 0) {
        if (COUNT) w.nodes += 7 * 16 + 4;                  // the node's seven dwordx4 loads + the octant's rank word
        WideNode n;
        wide_load(s.wnodes, k.cur, n);
        const int ridx = (k.sgn & 4) ? (k.sgn ^ 7) : k.sgn;
        uint32_t rw = reinterpret_cast<const uint32_t*>(&s.wnodes[k.cur])[28 + ridx];
        const uint32_t mask = wide_dw(n, 3) >> 24;
        if (k.sgn & 4)    // the reverse of octant sgn ^ 7: rank n-1-r in every 3-bit field (no borrow: r <= n-1)
            rw = (uint32_t)(__builtin_popcount(mask) - 1) * 0111111u - rw;
        float tmn[W], tmx[W];
        wide_slabs(n, r, tmn, tmx);
        int code[W];
#pragma unroll
        for (int c = 0; c < W; ++c) code[c] = wide_code(n, c);
        // valid slots as a mask in RANK order (the reference's visiting order for this octant);
        // bitwise, not short-circuit, so no slot test becomes a branch
        uint32_t vm = 0, vs = 0;
        uint32_t rank[W];
#pragma unroll
        for (int c = 0; c < W; ++c) {
            rank[c] = (rw >> (3 * c)) & 7u;
            // empty slots hold +inf / -inf planes (quantize_wide): never valid, no mask test
            const uint32_t v = (uint32_t)(tmx[c] >= __builtin_fmaxf(0.0f, tmn[c])) & (uint32_t)(tmn[c] <= k.tmax);
            vm |= v << rank[c];
            vs |= v << c;
        }
        if (vm) {
            int pos[W];
#pragma unroll
            for (int c = 0; c < W; ++c)
                pos[c] = k.sp + __builtin_popcount(vm >> (rank[c] + 1u));   // deeper the later it is visited
            if (__all(k.sp + W <= STK::kLds)) {
                // every valid slot of the wave lands in LDS, the first one (rank order) on top: one
                // unconditional write per slot, then the next node is read back from the top (cheaper
                // than selecting it and the pushes apart)
#pragma unroll
                for (int c = 0; c < W; ++c)
                    stk.put_lds(((vs >> c) & 1u) ? pos[c] : STK::kLds, make_int2(code[c], __float_as_int(tmn[c])));
                k.sp += __builtin_popcount(vm) - 1;
                k.cur = stk.code_lds(k.sp);
                return false;
            }
            const uint32_t first = (uint32_t)__builtin_ctz(vm);
            int next = 0;
            bool push[W];
#pragma unroll
            for (int c = 0; c < W; ++c) {
                const bool v = (vs >> c) & 1u;
                next = (v && rank[c] == first) ? code[c] : next;
                push[c] = v && rank[c] != first;
            }
            {
#pragma unroll
                for (int c = 0; c < W; ++c)
                    if (push[c]) stk.put(pos[c], make_int2(code[c], __float_as_int(tmn[c])));
            }
            k.sp += __builtin_popcount(vm) - 1;
            k.cur = next;
            return false;
        }
    } else {
        const float4* L = s.lrec + (k.cur & ~dl::kLeafBit);
        const float4 h0 = L[0], h1 = L[1], c0 = L[2], c1 = L[3], c2 = L[4];
        float lt;
        if (COUNT) w.nodes += 80;                 // leaf head + first primitive
        if (box_hit_fast(r, h0, h1, &lt) && lt <= k.tmax) {   // the reference leaf's exact box (:184)
            const int cnt = __float_as_int(h0.w), slot0 = __float_as_int(h1.w);
            for_leaf_prims(L, slot0, cnt, c0, c1, c2,
                           [&](int slot, const float4& p0, const float4& p1, const float4& p2) {
                               float ti;
                               if (COUNT) {
                                   if (slot - slot0 + 1 < cnt) w.nodes += 48;     // the next primitive's loads
                                   if (__float_as_int(p0.w) >= 0) w.tris++; else w.spheres++;
                               }
                               const bool h = __float_as_int(p0.w) >= 0 ? tri_hit(r, p0, p1, p2, &ti)
                                                                        : sphere_hit(r, p0, p1, &ti);
                               if (h && (ti < k.best.t || k.best.t == -1.0f)) {   // :213-221
                                   k.best.t = ti;
                                   k.best.prim = slot;
                                   k.tmax = ti;
                               }
                               return false;
                           });
        }
    }
    while (k.sp > 0) {
        --k.sp;
        const int2 e = stk.at(k.sp);
        if (__int_as_float(e.y) <= k.tmax) {
            k.cur = e.x;
            return false;
        }
    }
    return true;
}

// One closest-hit step; returns true when the walk is finished (result in k.best).
template <bool COUNT, class FETCH, class STK, bool PIPE = false>
__device__ __forceinline__ bool closest_step(const rtk::DevScene& s, const Ray& r, STK& stk, Walk& k, Work& w) {
    if ((!COUNT || s.count_prod) && k.tree == nullptr) return wide_closest_step<COUNT>(s, r, stk, k, w);
    if (k.cur >= 0) {
        float4 l0, l1, r0, r1;
        fetch_pair(k, l0, l1, r0, r1);
        if (COUNT) w.nodes += s.count_prod ? 64 : 2;
        float tl, tr;
        bool hl, hr;
        box_pair(r, k.fast, l0, l1, r0, r1, hl, hr, tl, tr);
        const bool left_first = comp(r.d, __float_as_int(l1.w)) > 0;
        const int il = __float_as_int(l0.w), ir = __float_as_int(r0.w);
        const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
        const float tn = left_first ? tl : tr, tf = left_first ? tr : tl;
        const int in_ = left_first ? il : ir, if_ = left_first ? ir : il;
        if (hf) {
            stk.put(k.sp, make_int2(if_, __float_as_int(tf)));
            ++k.sp;
        }
        if (hn && tn <= k.tmax) {
            k.cur = in_;
            return false;
        }
    } else {
        int a, cnt;
        leaf_range(s, k.cur, &a, &cnt);
        auto test = [&](int i, const float4& p0, const float4& p1, const float4& p2) {
            float t;
            bool h;
            if (COUNT && s.count_prod) w.nodes += 48;
            if (__float_as_int(p0.w) >= 0) {
                if (COUNT) w.tris++;
                h = tri_hit(r, p0, p1, p2, &t);
            } else {
                if (COUNT) w.spheres++;
                h = sphere_hit(r, p0, p1, &t);
            }
            if (h && (t < k.best.t || k.best.t == -1.0f)) {
                k.best.t = t;
                k.best.prim = i;
                k.tmax = t;
            }
            return false;
        };
        if (PIPE || RT_CLOSEST_PIPE) {
            for_prims(s, a, cnt, test);
        } else {
            // plain loop: the pipelined one costs k_chain a wave per SIMD (VGPRs)
            for (int i = a; i < a + cnt; ++i) {
                const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
                test(i, pr[0], pr[1], pr[2]);
            }
        }
    }
    while (k.sp > 0) {
        --k.sp;
        const int2 e = stk.at(k.sp);
        if (__int_as_float(e.y) <= k.tmax) {
            k.cur = e.x;
            return false;
        }
    }
    return true;
}

// One any-hit step: 0 = continue, 1 = finished unoccluded, 2 = finished occluded.
template <bool COUNT, class FETCH, class STK>
__device__ __forceinline__ int any_step(const rtk::DevScene& s, const Ray& r, float tlim, STK& stk, Walk& k,
                                        Work& w) {
    if (k.cur >= 0) {
        float4 l0, l1, r0, r1;
        fetch_pair(k, l0, l1, r0, r1);
        float tl, tr;
        bool hl, hr;
        box_pair(r, k.fast, l0, l1, r0, r1, hl, hr, tl, tr);
        const bool left_first = comp(r.d, __float_as_int(l1.w)) > 0;
        const int il = __float_as_int(l0.w), ir = __float_as_int(r0.w);
        const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
        const int in_ = left_first ? il : ir, if_ = left_first ? ir : il;
        if (COUNT) w.nodes += s.count_prod ? 64 : 1;
        if (hf || (COUNT && !s.count_prod)) {
            stk.put(k.sp, make_int2(if_, hf ? 1 : 0));
            ++k.sp;
        }
        if (hn) {
            k.cur = in_;
            return 0;
        }
    } else {
        int a, cnt;
        leaf_range(s, k.cur, &a, &cnt);
        if (for_prims(s, a, cnt, [&](int, const float4& p0, const float4& p1, const float4& p2) {
                float t;
                bool h;
                if (COUNT && s.count_prod) w.nodes += 48;
                if (__float_as_int(p0.w) >= 0) {
                    if (COUNT) w.tris++;
                    h = tri_hit(r, p0, p1, p2, &t);
                } else {
                    if (COUNT) w.spheres++;
                    h = sphere_hit(r, p0, p1, &t);
                }
                return h && t < tlim;
            }))
            return 2;
    }
    while (k.sp > 0) {
        --k.sp;
        const int2 e = stk.at(k.sp);
        if (COUNT && !s.count_prod) w.nodes++;
        if (e.y) {
            k.cur = e.x;
            return 0;
        }
    }
    return 1;
}

// One any-hit step over the occlusion tree's wide form (dl::Wide), NaN-free
// rays only (walk_begin).  Interior: decode and test the (conservative) child
// boxes, continue with the first hit child, push the others.  Leaf item: test
// the reference leaf's EXACT box, then its primitives (raytracer.cpp:264-277).
// Order is free: the any-hit answer does not depend on it.
// 0 = continue, 1 = finished unoccluded, 2 = finished occluded.
template <bool COUNT, class STK>
__device__ __forceinline__ int wide_any_step(const rtk::DevScene& s, const Ray& r, float tlim, STK& stk, Walk& k,
                                             Work& w) {
    constexpr int W = dl::kWideSlots;
    if (!COUNT && leaf_postponed(s.leaf_wait_any, k)) return 0;
    if (k.cur >= 0) {
        if (COUNT) w.nodes += 7 * 16;
        WideNode n;
        wide_load(s.swnodes, k.cur, n);
        float tmn[W], tmx[W];
        wide_slabs(n, r, tmn, tmx);
        uint32_t vs = 0;                  // empty slots: +inf / -inf planes, never valid (quantize_wide)
#pragma unroll
        for (int c = 0; c < W; ++c) vs |= (uint32_t)any_slot_valid(tmn[c], tmx[c]) << c;
        if (vs) {
            if (__all(k.sp + W <= STK::kLds)) {
                // the whole wave has LDS room: every hit slot written unconditionally, the first one
                // on top, and the next node read back from the top
#pragma unroll
                for (int c = 0; c < W; ++c)
                    stk.put_lds(((vs >> c) & 1u) ? k.sp + __builtin_popcount(vs >> (c + 1)) : STK::kLds,
                                make_int2(wide_code(n, c), 0));
                k.sp += __builtin_popcount(vs) - 1;
                k.cur = stk.code_lds(k.sp);
                return 0;
            }
            // continue with the first hit slot, push the others in slot order
            const uint32_t first = (uint32_t)__builtin_ctz(vs), pm = vs & (vs - 1u);
            int next = 0;
#pragma unroll
            for (int c = 0; c < W; ++c) next = (uint32_t)c == first ? wide_code(n, c) : next;
            {
#pragma unroll
                for (int c = 0; c < W; ++c)
                    if ((pm >> c) & 1u) stk.put(k.sp + __builtin_popcount(pm & ((1u << c) - 1u)), make_int2(wide_code(n, c), 0));
            }
            k.sp += __builtin_popcount(pm);
            k.cur = next;
            return 0;
        }
    } else {
        const float4* L = s.lrec + (k.cur & ~dl::kLeafBit);
        const float4 h0 = L[0], h1 = L[1], c0 = L[2], c1 = L[3], c2 = L[4];
        float bt;
        if (COUNT) w.nodes += 80;                    // leaf head + first primitive
        if (box_hit_fast(r, h0, h1, &bt)) {          // the reference leaf's exact box (NaN-free ray)
            const int cnt = __float_as_int(h0.w), slot0 = __float_as_int(h1.w);
            if (for_leaf_prims(L, slot0, cnt, c0, c1, c2,
                               [&](int slot, const float4& p0, const float4& p1, const float4& p2) {
                                   float t;
                                   bool h;
                                   if (COUNT && slot - slot0 + 1 < cnt) w.nodes += 48;   // next primitive
                                   if (__float_as_int(p0.w) >= 0) {
                                       if (COUNT) w.tris++;
                                       h = tri_hit(r, p0, p1, p2, &t);
                                   } else {
                                       if (COUNT) w.spheres++;
                                       h = sphere_hit(r, p0, p1, &t);
                                   }
                                   return h && t < tlim;
                               }))
                return 2;
        }
    }
    if (k.sp > 0) {
        --k.sp;
        k.cur = stk.at(k.sp).x;
        return 0;
    }
    return 1;
}

// Any-hit step on whichever tree the walk is on.
template <bool COUNT, class FETCH, class STK>
__device__ __forceinline__ int occl_step(const rtk::DevScene& s, const Ray& r, float tlim, STK& stk, Walk& k,
                                         Work& w);

// One step of EITHER walk, selected per lane by `any`, on one code path (no
// divergence between lanes doing closest-hit and lanes doing any-hit):
//   closest  tmax = best t so far; entries {info, tmin} pruned at pop by
//            tmin <= tmax (the reference's test-at-pop);
//   any      k.tmax = +inf; entries {info, 0 (child hit) | NaN (missed, COUNT
//            builds only)}, so the same pop test expands exactly the hit ones;
//            a hit closer than tlim ends the walk (occluded).
// Returns 0 = continue, 1 = finished (closest: k.best; any: unoccluded),
// 2 = finished occluded.
template <bool COUNT, class FETCH, class STK>
__device__ __forceinline__ int dual_step(const rtk::DevScene& s, const Ray& r, bool any, float tlim, STK& stk,
                                         Walk& k, Work& w) {
    if (k.cur >= 0) {
        float4 l0, l1, r0, r1;
        fetch_pair(k, l0, l1, r0, r1);
        float tl, tr;
        bool hl, hr;
        box_pair(r, k.fast, l0, l1, r0, r1, hl, hr, tl, tr);
        const bool left_first = comp(r.d, __float_as_int(l1.w)) > 0;
        const int il = __float_as_int(l0.w), ir = __float_as_int(r0.w);
        const bool hn = left_first ? hl : hr, hf = left_first ? hr : hl;
        const float tn = left_first ? tl : tr, tf = left_first ? tr : tl;
        const int in_ = left_first ? il : ir, if_ = left_first ? ir : il;
        if (COUNT) w.nodes += any ? 1 : 2;
        if (hf || (COUNT && any)) {
            const float key = any ? (hf ? 0.0f : __int_as_float(0x7fc00000)) : tf;
            stk.put(k.sp, make_int2(if_, __float_as_int(key)));
            ++k.sp;
        }
        if (hn && (any || tn <= k.tmax)) {
            k.cur = in_;
            return 0;
        }
    } else {
        int a, cnt;
        leaf_range(s, k.cur, &a, &cnt);
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
            if (any) {
                if (h && t < tlim) return 2;
            } else if (h && (t < k.best.t || k.best.t == -1.0f)) {
                k.best.t = t;
                k.best.prim = i;
                k.tmax = t;
            }
        }
    }
    while (k.sp > 0) {
        --k.sp;
        const int2 e = stk.at(k.sp);
        if (COUNT && any) w.nodes++;               // any-hit: far child counted when popped
        if (__int_as_float(e.y) <= k.tmax) {
            k.cur = e.x;
            return 0;
        }
    }
    return 1;
}

template <bool COUNT, class FETCH, class STK>
__device__ __forceinline__ int occl_step(const rtk::DevScene& s, const Ray& r, float tlim, STK& stk, Walk& k,
                                         Work& w) {
    if (k.tree == nullptr) return wide_any_step<COUNT>(s, r, tlim, stk, k, w);
    return any_step<COUNT, FETCH>(s, r, tlim, stk, k, w);
}

// The timed (non-counting) kernels walk only the wide trees: a ray the wide trees' slab test does
// not take is deferred to k_fallback before its walk begins (pathchain.hip defer_closest /
// defer_any), so these kernels carry no binary-tree walk code and fit their register budgets without
// spills.  Counting kernels keep the general steps (the reference tree, the production-fetch pass).
template <bool COUNT, bool PIPE, class STK>
__device__ __forceinline__ bool closest_step_timed(const rtk::DevScene& s, const Ray& r, STK& stk, Walk& k, Work& w) {
    if constexpr (COUNT) return closest_step<COUNT, FetchGlobal, STK, PIPE>(s, r, stk, k, w);
    else return wide_closest_step<false>(s, r, stk, k, w);
}
template <bool COUNT, class STK>
__device__ __forceinline__ int occl_step_timed(const rtk::DevScene& s, const Ray& r, float tlim, STK& stk, Walk& k,
                                               Work& w) {
    if constexpr (COUNT) return occl_step<COUNT, FetchGlobal>(s, r, tlim, stk, k, w);
    else return wide_any_step<false>(s, r, tlim, stk, k, w);
}

}  // namespace rtd
