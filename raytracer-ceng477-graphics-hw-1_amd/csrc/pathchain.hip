// Chain renderer kernels (see pathchain.hpp).
//
// Work distribution without global atomics.  A single device-scope counter
// saturates at ~88 grabs/us on MI355X (MI355X_MICROARCH.md, "dequeue"), i.e.
// ~0.4 ms per frame for the ~32 K sample grabs plus ~60 K shadow-queue appends
// of a 1080p frame.  Instead every workgroup of the persistent grid owns a
// fixed, interleaved set of 256-sample units (unit u -> block u mod G) and a
// private region of the shadow-ray queue; lanes take samples and queue slots
// through LDS atomics (one per wave per refill).  k_occlude's block b walks
// the rays of region b.
//
// Lanes of a wave refill together once at most PcParams.refill of them are
// still walking (refill = 0: a wave takes new samples only when all its lanes
// are done; coherence of the 8x8 tiles is kept).
//
// Memory behaviour (rocprofv3, C3 frame): the walks are bound by vector-L1
// miss handling (TCP_PENDING_STALL ~50 % of cycles, ~330-cycle L2 latency).
// Hence: the top BVH levels (which every walk crosses) are read from an LDS
// copy; the traversal stack keeps its first entries in LDS; streaming records
// (shadow rays, hit records) use non-temporal accesses; shadow rays are
// queued light-major within each wave, so a wave of k_occlude walks rays
// toward one light from neighbouring surface points.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include "pathchain.hpp"
#include "traverse2.hpp"
#include "wave_util.hpp"

using namespace rtd;

namespace rtc {

namespace {

constexpr int kBlock = 256;
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 5     // k_chain: 5 waves/SIMD (96 VGPRs, no spills since the binary-tree walks moved to
                              // k_fallback; 4 waves: 100 VGPRs): C3 batches 0.480-0.486 -> 0.468-0.472 ms/frame
#endif
#ifndef RT_FINISH_PREFETCH
#define RT_FINISH_PREFETCH 1   // k_finish: next level's record in flight while shading
#endif
#ifndef RT_FINISH_CMP_WAVES
#define RT_FINISH_CMP_WAVES 3 // k_finish<true> (compact records: the rebuilt directions): 4 waves spilled 28 VGPRs,
                              // whose scratch traffic reached HBM (k_finish 150 MB per batched frame, 77 MB of
                              // algorithmic bytes); 3 waves: no spills
#endif
#ifndef RT_FINISH_WAVES
#define RT_FINISH_WAVES 4     // k_finish: 128 VGPRs, 4 waves/SIMD, no spills (unbounded: 129, 3 waves): C3 batches
                              // 0.507-0.508 -> 0.502-0.504 ms/frame; 5 (spills) 0.532, 6 0.559
#endif
#ifndef RT_FINISH_ANY_WAVES
#define RT_FINISH_ANY_WAVES 1 // k_finish_any (large scenes): at 4 waves it spills a VGPR
#endif
#ifndef RT_OCC_WAVES_PER_EU
#define RT_OCC_WAVES_PER_EU 6     // k_occlude (the any-hit bulk): 79 VGPRs, no spills (round 3; was 5)
#endif

enum LaneState : int { kIdle = 0, kTrav = 1, kDone = 2 };

// Diagnostics build (RT_STEP_STATS=1): per-role wave-step statistics of the
// walk loops, read by rt_debug_step_stats.  Slot r*8 + {0: wave iterations,
// 1: walking lanes, 2: lanes at an interior node, 3: lanes stepping a leaf
// record (not postponed), 4: iterations that step a leaf record, 5: refills,
// 6: lanes refilled, 7: iterations that step an interior node}; role 0 =
// phase-A chains, 1 = phase-B chains, 2 = shadow rays, 3 = phase-B queue.
#ifndef RT_STEP_STATS
#define RT_STEP_STATS 0
#endif
__device__ unsigned long long g_step_stat[32];
struct StepStat {
    unsigned long long v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void step(bool walking, bool interior, bool postponed) {
        if (!RT_STEP_STATS) return;
        const unsigned long long wm = __ballot(walking), im = __ballot(walking && interior),
                                 lm = __ballot(walking && !interior && !postponed);
        const int nw = __popcll(wm), ni = __popcll(im), nl = __popcll(lm);
        v[0] += 1; v[1] += nw; v[2] += ni; v[3] += nl; v[4] += nl > 0 ? 1 : 0; v[7] += ni > 0 ? 1 : 0;
    }
    __device__ __forceinline__ void refill(unsigned long long mask) {
        if (!RT_STEP_STATS) return;
        v[5] += 1; v[6] += __popcll(mask);
    }
    __device__ __forceinline__ void flush(int role) {
        if (!RT_STEP_STATS) return;
        if ((threadIdx.x & 63) == 0)
            for (int i = 0; i < 8; ++i) atomicAdd(&g_step_stat[role * 8 + i], v[i]);
    }
};



// LDS, named directly so every access is a ds_read/ds_write (a generic
// pointer to them would compile to flat loads that wait on vmcnt + lgkmcnt).

#ifndef RT_LDS_STACK
#define RT_LDS_STACK 12
#endif
// Traversal stack: entries [0, kLdsStackEntries) in LDS ([entry][thread], so
// a wave's lanes hit distinct banks), deeper ones in scratch.  LDS keeps the
// pushes and pops off the vector-memory (TA) path that the node fetches use.
constexpr int kLdsStackEntries = RT_LDS_STACK;
#if RT_LDS_STACK <= 0
#error "the wide walks push out of order: they need the random-access StackLds (RT_LDS_STACK > 0)"
#endif
struct StackLds {
    // put_lds(i, v): i < kLds (the caller has checked the whole wave has room), or kLds itself, a
    // per-lane scratch entry that absorbs the writes of slots that push nothing (branch-free pushes)
    static constexpr int kLds = kLdsStackEntries;
    __device__ __forceinline__ void put_lds(int i, int2 v);
    __device__ __forceinline__ int code_lds(int i);      // entry i (< kLds) .x
    // Deep tier as two int arrays: loads shaped unlike the LDS int2 read, so
    // the compiler cannot sink both tiers into one flat load through a
    // selected pointer (which waits on vmcnt and lgkmcnt at every pop).
    int dx[dl::kMaxStack > kLdsStackEntries ? dl::kMaxStack - kLdsStackEntries : 1];
    int dy[dl::kMaxStack > kLdsStackEntries ? dl::kMaxStack - kLdsStackEntries : 1];
    __device__ __forceinline__ void put(int i, int2 v);
    __device__ __forceinline__ int2 at(int i);
};
#if RT_LDS_STACK > 0
__shared__ int2 g_lstk[(kLdsStackEntries + 1) * kBlock];
__device__ __forceinline__ void StackLds::put_lds(int i, int2 v) { g_lstk[i * kBlock + threadIdx.x] = v; }
__device__ __forceinline__ int StackLds::code_lds(int i) { return g_lstk[i * kBlock + threadIdx.x].x; }
__device__ __forceinline__ void StackLds::put(int i, int2 v) {
    if (i < kLdsStackEntries) {
        g_lstk[i * kBlock + threadIdx.x] = v;
    } else {
        dx[i - kLdsStackEntries] = v.x;
        dy[i - kLdsStackEntries] = v.y;
    }
}
__device__ __forceinline__ int2 StackLds::at(int i) {
    if (i < kLdsStackEntries) return g_lstk[i * kBlock + threadIdx.x];
    return make_int2(dx[i - kLdsStackEntries], dy[i - kLdsStackEntries]);
}
using WalkStack = StackLds;
#else
using WalkStack = StackPriv;
#endif
__shared__ unsigned g_head;                    // block-local work queue head
__shared__ unsigned g_scnt;                    // block-local shadow-task count

// Pair fetches go to global memory: caching the top BVH levels in LDS showed
// no gain (their loads are wave-coherent and hit the L1).
using FetchTop = FetchGlobal;

__device__ __forceinline__ void block_init(const rtk::DevScene& s) {
    if (threadIdx.x == 0) {
        g_head = 0;
        g_scnt = 0;
    }
    __syncthreads();
}

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Always-on bound on a loop that waits on other lanes or waves of the workgroup without progress of
// its own (the phase-A unit hand-off, the phase-B LDS shadow queue, the wave leaf queue): after
// s.spin_cap such iterations it gives up, sets bit 1 of the scene's device error word (rt_render* /
// rt_scene_check return RT_ERR_LIMIT) and the caller leaves the loop, so a scheduling bug ends the
// kernel with an error instead of hanging the GPU.  n counts the iterations of the current wait.
__device__ __forceinline__ bool spin_over(const rtk::DevScene& s, unsigned& n) {
    if (++n <= (unsigned)s.spin_cap) return false;
    __hip_atomic_fetch_or(s.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// LDS words written by other waves of the workgroup: atomic loads and stores (a plain or volatile
// load may be kept in a register across the wait loop).
__device__ __forceinline__ unsigned lds_load(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ unsigned lane_rank(unsigned long long mask) {
    const int lane = threadIdx.x & 63;
    return (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
}

// One LDS atomic per wave: popc(mask) consecutive indices from *ctr.
__device__ __forceinline__ unsigned wave_grab_lds(unsigned* ctr, unsigned long long mask) {
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)mask) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(ctr, (unsigned)__popcll(mask));
    return __shfl(base, leader, 64);
}

// ---------------------------------------------------------------------------
// Chain phases.  Phase A (k_chain) walks every sample's closest-hit chain up
// to level `kinline`; a mirror bounce below it is handed on as a
// continuation task (the record's owner id; the reflected ray is re-derived
// from the record, raytracer.cpp:430-435).  Phase B (the chain role of k_mix)
// walks those continuations to the end, while the other k_mix workgroups
// already run phase A's shadow rays.  So the long mirror chains of a few
// pixels overlap the bulk of the shadow work instead of preceding all of it.
// Shadow tasks are u32 owner ids ((level*cap + sample)*nlights + light); the
// shadow ray is re-derived from the hit record by the walking lane
// (raytracer.cpp:397-404), bit-identically.
// Work is split per workgroup (interleaved, no global atomics): samples by
// 256-sample units, continuation and shadow tasks by index j -> j mod G.
// ---------------------------------------------------------------------------
__shared__ unsigned g_ccnt;    // block-local continuation count
__shared__ unsigned g_dcnt;    // ... of those queued at the region's end (PcParams::pdepth: deep last frame)
__shared__ unsigned g_uid[kDynUnits];   // dynamic phase-A units: the workgroup's k-th unit (kUidUnset: not yet taken)
constexpr unsigned kUidUnset = ~0u, kUidNone = ~0u - 1u;
// A mixed-deal virtual unit (PcParams::ugrp): kUidMix | log2 G << 28 | sub-unit << 24 | group.
constexpr unsigned kUidMix = 0x80000000u;

struct PhaseOut {              // where a chain phase writes its tasks
    unsigned* sq;              // shadow tasks, region blk at sq + blk * scap
    unsigned scap;
    unsigned* scount;          // tasks per region
    unsigned* cq;              // continuations (phase A only), region blk at cq + blk * ccap
    unsigned ccap;
    unsigned* ccount;
    int kinline;               // deepest level walked here
};

// Hit records (one per recorded level, by record id lvp):
//   rec[lvp]           = {hit point xyz, surface code (hit_surface: triangle index or ~sphere slot)}
//   recd[lvp - dbase]  = {ray direction xyz, material id}, for lvp >= p.dbase only
// The normal is not stored: surface_normal rebuilds it bit-identically from
// the hit point and the code (a 16-byte face-normal read from the L2-resident
// scene instead of 16 more bytes per record through HBM, written once and read
// by every shadow task, the mirror bounce and the shading of the record).  Nor,
// below dbase (phase A's levels 0 and 1 of every sample, most of a frame's
// records), are the direction and material: the direction of level 0 is the
// sample's eye ray's and that of level 1 the reflection of level 0's (k_finish
// path_shade_fold: the chain's arithmetic on the same values, so bit-identical),
// the material is the surface's (surface_mat); where a phase-A record's
// reflection is read back later (a continuation, a deferred reflected ray) the
// chain leaves the direction in tail[sample] (reflect_from_record).  16 bytes
// per phase-A record through HBM instead of 32, written by k_chain, read by
// k_finish and by the shadow walks.

// Record id of level k of sample `path` (continuation index c when k >= p.la): levels below la at
// k * cap + path, deeper ones (phase B) only for the first cb continuations, after them.
// (Record ids, and owner ids rid * nl + l, stay below 2^31: rt_api.cpp checks cap * levels * nl.)
__device__ __forceinline__ unsigned rec_id(const PcParams& p, int k, unsigned path, unsigned c) {
    return k < p.la ? (unsigned)k * (unsigned)p.cap + path
                    : (unsigned)p.la * (unsigned)p.cap + (unsigned)(k - p.la) * p.cb + c;
}
__device__ __forceinline__ void rec_write(const PcParams& p, size_t lvp, const V& hitp, int code, const V& d,
                                          int mat) {
    p.rec[lvp] = make_float4(hitp.x, hitp.y, hitp.z, __int_as_float(code));
    if (lvp >= p.dbase) p.recd[lvp - p.dbase] = make_float4(d.x, d.y, d.z, __int_as_float(mat));
}

// The surface's material id (hit_surface's *mat): the triangle's shading word, or the sphere
// primitive's material word.
__device__ __forceinline__ int surface_mat(const rtk::DevScene& s, int code) {
    if (code >= 0) return __float_as_int(ld4(&s.tri_shade[code]).w);
    return __float_as_int(reinterpret_cast<const float4*>(&s.prims[~code])[2].w);
}

// Can light l's shadow ray from this hit change the pixel?  The shading
// (shade_words, raytracer.cpp:405-425) adds nothing for an occluded light; for
// a visible one with cos < cos_thr it adds no specular term (its test fails)
// and the diffuse term kd * 0 * E = +-0 (the clamp gives 0).  With kd (host:
// s.cull_shadows) and E finite the sum is the same either way, so the ray is
// not traced and the light is recorded as occluded.  The same arithmetic as
// shade_words on the same record values, so the decision is exact.
__device__ __forceinline__ bool light_needed(const rtk::DevScene& s, const V& hitp, const V& nn, int l) {
    const float4 lp = ld4(&s.lights[l].px), li4 = ld4(&s.lights[l].ix);
    const V lpos{lp.x, lp.y, lp.z};
    const V pnt = add(hitp, mul(nn, s.eps));
    const float dist = len(sub(lpos, pnt));
    const float cos_t = dot(nrm(sub(lpos, hitp)), nn);
    if (!(cos_t < s.cos_thr)) return true;
    const V E = divs(V{li4.x, li4.y, li4.z}, dist * dist);
    return !(__builtin_isfinite(E.x) && __builtin_isfinite(E.y) && __builtin_isfinite(E.z));
}

// Reflected ray at hit point hitp with normal nn of a ray along d (raytracer.cpp:430-435).
__device__ __forceinline__ Ray reflect_ray(const rtk::DevScene& s, const V& hitp, const V& nn, const V& d) {
    const V pnt = add(hitp, mul(nn, s.eps));                                            // :397
    const V d2 = nrm(d);
    const V n2 = nrm(nn);
    const float rcos = dot(neg(d2), n2);
    return make_ray(pnt, add(d2, mul(mul(n2, 2.0f), rcos)));
}

// Reflected ray of recorded level lvp of sample `path`.  A phase-A record below dbase has no direction;
// the chain left it in tail[path] where a reflection is read back (a continuation handed to phase B or
// k_fallback, or a deferred reflected ray), tail's colour use coming later (k_fallback's kEndTail).
__device__ __forceinline__ Ray reflect_from_record(const rtk::DevScene& s, const PcParams& p, size_t lvp,
                                                   unsigned path) {
    const float4 a = p.rec[lvp];
    const V hitp{a.x, a.y, a.z};
    const float4 c = lvp >= p.dbase ? p.recd[lvp - p.dbase] : p.tail[path];
    return reflect_ray(s, hitp, surface_normal(s, hitp, __float_as_int(a.w)), V{c.x, c.y, c.z});
}

// Shadow ray toward light l from a hit (raytracer.cpp:397-404): origin hitp + n * eps, direction
// normalize(L - origin), length |L - origin|.
__device__ __forceinline__ Ray shadow_ray(const rtk::DevScene& s, const V& hitp, const V& nn, int l, float* tlim) {
    const V pnt = add(hitp, mul(nn, s.eps));
    const float4 lp = ld4(&s.lights[l].px);
    const V lpos{lp.x, lp.y, lp.z};
    *tlim = len(sub(lpos, pnt));
    return make_ray(pnt, nrm(sub(lpos, pnt)));
}

// Shadow ray of task `owner` (raytracer.cpp:397-404).
__device__ __forceinline__ Ray shadow_from_record(const rtk::DevScene& s, const PcParams& p, unsigned owner,
                                                  float* tlim) {
    const unsigned lvp = owner / (unsigned)s.nlights;
    const int l = (int)(owner - lvp * (unsigned)s.nlights);
    const float4 a = p.rec[lvp];
    const V hitp{a.x, a.y, a.z};
    return shadow_ray(s, hitp, surface_normal(s, hitp, __float_as_int(a.w)), l, tlim);
}

// Rays the timed walks leave to k_fallback: not NaN-free, or beyond the range of the wide trees' fused
// slab test (wide_ray_ok; in practice a direction component of exactly 0, whose 1/d is infinite).
// The production kernels then carry only the wide-tree walks (fewer registers: no VGPR spills).
// (tests: force_fb bit 0 defers every closest-hit ray, bit 2 only reflected ones -- refl)
__device__ __forceinline__ bool defer_closest(const rtk::DevScene& s, const Ray& r, bool refl) {
    return s.nnodes > 0 && ((s.force_fb & (refl ? 5 : 1)) || !(s.use_wide && ray_nan_free(r) && wide_ray_ok(r)));
}
__device__ __forceinline__ bool defer_any(const rtk::DevScene& s, const Ray& r) {
    return s.nnodes > 0 && ((s.force_fb & 2) || !(s.use_stree == 2 && ray_nan_free(r) && wide_ray_ok(r)));
}
__device__ __forceinline__ void fb_chain(const PcParams& p, unsigned entry) {
    const unsigned i = atomicAdd(&p.totals[4], 1u);
    if (i < p.fbc_cap) p.fbc[i] = entry;       // fbc_cap = cap: a sample defers at most one ray per launch
}
__device__ __forceinline__ void fb_shadow(const PcParams& p, unsigned owner) {
    const unsigned i = atomicAdd(&p.totals[5], 1u);
    if (i < p.fbs_cap) {
        p.fbs[i] = owner;
    } else {                                   // queue full: mark the byte, k_fallback scans for it
        p.occ[owner] = kOccDeferred;
        __hip_atomic_store(&p.totals[6], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The same shadow ray for a task produced by another wave of the workgroup
// (bq_consume): the record is read past the CU's L1 (sc0 loads), which may
// still hold an older copy of its line.
__device__ __forceinline__ float4 ld4_l2(const float4* ptr) {
    float4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(ptr) : "memory");
    return v;
}
__device__ __forceinline__ Ray shadow_from_record_l2(const rtk::DevScene& s, const PcParams& p, unsigned owner,
                                                     float* tlim) {
    const unsigned lvp = owner / (unsigned)s.nlights;
    const int l = (int)(owner - lvp * (unsigned)s.nlights);
    const float4 a = ld4_l2(p.rec + lvp);
    const V hitp{a.x, a.y, a.z};
    return shadow_ray(s, hitp, surface_normal(s, hitp, __float_as_int(a.w)), l, tlim);
}

// Samples of workgroup blk (of G): units blk, blk+G, ... of 256 slots.
__device__ __forceinline__ unsigned group_samples(unsigned n0, unsigned G, unsigned blk) {
    const unsigned units = (n0 + 255u) / 256u;
    if (blk >= units) return 0;
    const unsigned mine = (units - 1u - blk) / G + 1u;
    const unsigned last_unit = blk + (mine - 1u) * G;
    return (mine - 1u) * 256u + min(256u, n0 - last_unit * 256u);
}

// Task index space [0, T) dealt to G workgroups in chunks of `ch`
// consecutive tasks (chunk c -> workgroup c mod G).  ch = 1 (default) spreads
// the spatially clustered heavy tasks (mirror regions) over every workgroup;
// larger chunks give a wave neighbouring tasks (more coherent fetches) at the
// price of that balance.
__device__ __forceinline__ unsigned chunk_count(unsigned T, unsigned G, unsigned blk, unsigned ch) {
    const unsigned nch = (T + ch - 1u) / ch;
    if (blk >= nch) return 0u;
    const unsigned m = (nch - 1u - blk) / G + 1u;
    const unsigned short_last = ((nch - 1u) % G == blk) ? nch * ch - T : 0u;
    return m * ch - short_last;
}
__device__ __forceinline__ unsigned chunk_task(unsigned v, unsigned G, unsigned blk, unsigned ch) {
    return (blk + (v / ch) * G) * ch + v % ch;
}

// Unsigned division by a wave-uniform divisor d > 0 with its reciprocal kept in a scalar register
// (the compiler's own 32-bit expansion: an f32 reciprocal scaled to 2^32, one Newton step, the
// quotient from a high multiply and two corrections -- exact for every 32-bit v).  The compiler
// leaves that reciprocal in a VGPR, which the leaf-queue walker then spills.
struct UDiv {
    unsigned d, rcp;
    __device__ __forceinline__ explicit UDiv(unsigned d_) : d(d_) {
        unsigned r = (unsigned)(__builtin_amdgcn_rcpf((float)d_) * 4294966784.0f);   // 0x4f7ffffe
        r += __umulhi(r, (0u - d_) * r);
        rcp = __builtin_amdgcn_readfirstlane(r);
    }
    __device__ __forceinline__ unsigned div(unsigned v) const {
        unsigned q = __umulhi(v, rcp), rem = v - q * d;
        if (rem >= d) { ++q; rem -= d; }
        if (rem >= d) ++q;
        return q;
    }
};
__device__ __forceinline__ unsigned chunk_task(unsigned v, unsigned G, unsigned blk, const UDiv& ch) {
    const unsigned q = ch.div(v);
    return (blk + q * G) * ch.d + (v - q * ch.d);
}
// Phase A's per-workgroup task regions (shadow tasks sqA / scntA, continuations cq / ccnt) read as ONE list
// in region order -- the order k_pack_a's packing gives them, without the copy: each consumer workgroup holds
// the regions' exclusive count prefix in LDS (region_prefix) and maps list index j to its region by binary
// search (region_task).  A lone frame's k_mix reads both lists so (no packing kernel between its phase A
// and phase B: -10 us per C3 frame); frame batches keep k_pack_a's packed continuations (cflat), which their
// k_mix reads 2 % faster (profiles/r06_nopack_ab.jsonl); k_fallback reads the continuations so in both.
__shared__ unsigned g_pref[kMaxChainGrid + 1];
// g_pref[0, nreg] = the exclusive prefix of cnt[0, nreg) (g_pref[nreg] = the total, returned).  Every thread
// of the workgroup; nreg <= kMaxChainGrid.  A call, not inlined: inlined at the kernels' start it still cost
// k_mix 7 VGPRs and 31-37 more SGPR spills in its walk loops.
__device__ __noinline__ unsigned region_prefix(const unsigned* cnt, unsigned nreg) {
    __shared__ unsigned s_psum[kBlock / 64];
    const int lane = lane_id(), wave = (int)(threadIdx.x >> 6);
    const unsigned per = (nreg + kBlock - 1u) / kBlock;
    const unsigned r0 = min(nreg, threadIdx.x * per), r1 = min(nreg, r0 + per);
    unsigned sum = 0;
    for (unsigned r = r0; r < r1; ++r) sum += cnt[r];
    unsigned inc = sum;
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned v = __shfl_up(inc, off, 64);
        if (lane >= off) inc += v;
    }
    if (lane == 63) s_psum[wave] = inc;
    __syncthreads();
    unsigned at = inc - sum, total = 0;
    for (int w = 0; w < kBlock / 64; ++w) {
        if (w < wave) at += s_psum[w];
        total += s_psum[w];
    }
    for (unsigned r = r0; r < r1; ++r) {
        g_pref[r] = at;
        at += cnt[r];
    }
    if (threadIdx.x == 0) g_pref[nreg] = total;
    __syncthreads();
    return total;
}
// Entry j (< g_pref[nreg]) of the region list: region r with g_pref[r] <= j < g_pref[r + 1] (the last r with
// g_pref[r] <= j: empty regions are skipped), its entry j - g_pref[r].
__device__ __forceinline__ unsigned region_of(unsigned nreg, unsigned j) {
    unsigned lo = 0, hi = nreg;
    while (hi - lo > 1u) {
        const unsigned mid = (lo + hi) >> 1;
        if (g_pref[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ unsigned region_task(const unsigned* q, unsigned cap, unsigned nreg, unsigned j) {
    const unsigned r = region_of(nreg, j);
    return q[(size_t)r * cap + (j - g_pref[r])];
}
// A shadow-task list: a packed array (REG false) or the phase-A regions through g_pref (REG true).  The shadow
// walkers take tasks in chunks of consecutive indices, so a lane's next task is nearly always in its previous
// one's region (hint): two LDS reads instead of the search's eleven.
template <bool REG>
struct TaskList {
    const unsigned* q;
    unsigned cap, nreg, hint;
    __device__ __forceinline__ unsigned operator[](unsigned j) {
        if constexpr (REG) {
            unsigned r = hint;
            if (!(g_pref[r] <= j && j < g_pref[r + 1])) hint = r = region_of(nreg, j);
            return q[(size_t)r * cap + (j - g_pref[r])];
        } else {
            return q[j];
        }
    }
};
__device__ __forceinline__ TaskList<false> flat_list(const unsigned* q) { return TaskList<false>{q, 0u, 0u, 0u}; }
__device__ __forceinline__ TaskList<true> shadow_regions_a(const PcParams& p) {
    return TaskList<true>{p.sqA, p.scapA, (unsigned)p.grid, 0u};
}

__device__ __forceinline__ unsigned cont_entry(const PcParams& p, unsigned j) {   // continuation j (region order)
    return region_task(p.cq, p.ccapA, (unsigned)p.grid, j);
}


__device__ __forceinline__ Ray shadow_from_record(const rtk::DevScene& s, const PcParams& p, unsigned owner,
                                                  float* tlim, const UDiv& nl) {
    const unsigned lvp = nl.div(owner);
    const int l = (int)(owner - lvp * nl.d);
    const float4 a = p.rec[lvp];
    const V hitp{a.x, a.y, a.z};
    return shadow_ray(s, hitp, surface_normal(s, hitp, __float_as_int(a.w)), l, tlim);
}

// Phase-B shadow tasks go to a workgroup queue in LDS (owner ids) while it has
// room; the workgroup's waves whose chains are done walk them while the other
// waves' long mirror chains still run, so those shadow rays no longer wait for
// k_occlude.  Tasks beyond the queue go to the global queue (k_pack_b +
// k_occlude) as before.  Protocol (one workgroup, no cross-workgroup waits):
// slots start kBqEmpty; a producer wave makes its hit records visible to the
// workgroup (release fence), reserves slots (LDS atomic on g_bq_tail) and
// writes the owner ids (kBqSkip for a reservation that spilled to the global
// queue); a consumer lane takes the next slot index (g_bq_head) and waits for
// it to be written, or gives up once every producer wave has finished
// (g_bq_prod == 0) and the index is past the final tail.
constexpr int kBq = kMaxBq;
constexpr unsigned kBqEmpty = 0xffffffffu, kBqSkip = 0xfffffffeu;
__shared__ unsigned g_bq[kBq > 0 ? kBq : 1];
__shared__ unsigned g_bq_tail, g_bq_head, g_bq_prod;

__device__ __forceinline__ void bq_init() {
    for (int i = threadIdx.x; i < kBq; i += kBlock) g_bq[i] = kBqEmpty;
    if (threadIdx.x == 0) {
        g_bq_tail = 0;
        g_bq_head = 0;
        g_bq_prod = kBlock / 64;
    }
}

// Walk the workgroup queue's shadow tasks (raytracer.cpp:227-280) until it is
// drained and every producer wave has finished; returns the rays walked.
template <bool COUNT>
__device__ uint32_t bq_consume(const rtk::DevScene& s, const PcParams& p, WalkStack& stk, Work& w) {
    bool active = false, have = false, out = false;   // walking / holding a slot index / no more slots
    unsigned slot = 0;
    Ray r;
    float tlim = 0.0f;
    unsigned owner = 0;
    Walk wk;
    uint32_t n = 0;
    unsigned spins = 0;      // consecutive iterations with no lane walking (spin_over)
    StepStat stat;
    while (true) {
        const unsigned long long want = __ballot(!active && !have && !out);
        if (want) {
            const unsigned base = wave_grab_lds(&g_bq_head, want);
            if (!active && !have && !out) {
                slot = base + lane_rank(want);
                if (slot < (unsigned)p.bq_cap) have = true;
                else out = true;
            }
        }
        bool idle = false;
        if (have) {
            const unsigned v = __atomic_load_n(&g_bq[slot], __ATOMIC_RELAXED);
            if (v == kBqEmpty) {
                // not written yet: wait, unless no producer is left and the slot was never reserved
                if (__atomic_load_n(&g_bq_prod, __ATOMIC_RELAXED) == 0u &&
                    slot >= __atomic_load_n(&g_bq_tail, __ATOMIC_RELAXED)) {
                    have = false;
                    out = true;
                } else {
                    idle = true;
                }
            } else {
                have = false;
                if (v != kBqSkip) {
                    owner = v;
                    r = shadow_from_record_l2(s, p, owner, &tlim);
                    ++n;
                    if (!COUNT && defer_any(s, r)) fb_shadow(p, owner);
                    else if (COUNT ? walk_begin<COUNT>(s, r, wk, w, true) : walk_begin_wide(s, r, wk, true)) active = true;
                    else p.occ[owner] = 0;
                }
            }
        }
        if (!__any(active)) {
            if (__all(out) || spin_over(s, spins)) break;
            if (__any(idle)) __builtin_amdgcn_s_sleep(2);
            continue;
        }
        spins = 0;
        stat.step(active, wk.cur >= 0, RT_STEP_STATS && active && wk.tree == nullptr && leaf_postponed(s.leaf_wait_any, wk));
        if (active) {
            const int res = occl_step_timed<COUNT>(s, r, tlim, stk, wk, w);
            if (res || walk_runaway(s, wk)) {
                p.occ[owner] = res == 2 ? 1 : 0;
                active = false;
            }
        }
    }
    stat.flush(3);
    if (COUNT) {
        wave_add_counter(&p.counters[kCntBQBytes], w.nodes);
        wave_add_counter(&p.counters[kCntBQRays], n);
    }
    return n;
}

// The u-th unit taken -> the unit id.  The slab's rows of units (tiles_x / 4 units each) are cut
// into super-rows of ublk_h tile rows (< 0: one frame of the batch), each walked in column blocks
// ublk_w units wide, so the units in flight (a launch-wide counter: the whole GPU on them at once)
// cover a column of the image instead of a full-width band (C3, 256-px columns a frame high: ~1 %
// per batched frame, ~2 % one frame).  Identity when ublk_h == 0 or the units do not tile the rows.
__device__ __forceinline__ unsigned unit_col_order(const PcParams& p, unsigned u, unsigned units) {
    return unit_col(p.tiles_x, p.ublk_h, p.ublk_w, p.nframes, u, units);
}
// The unit dealt u-th: the previous frame's heaviest units first (PcParams::uorder_on), else the column order.
__device__ __forceinline__ unsigned unit_order(const PcParams& p, unsigned u, unsigned units) {
    return p.uorder_on ? p.uorder[u] : unit_col_order(p, u, units);
}
// Sample slot of position o (0..255) of a mixed-deal virtual unit (kUidMix code; PcParams::ugrp): the
// group's G virtual units are G * 4 wave chunks of 64 positions; in chunk w, positions l < h = 64 / G hold
// samples w * h + l of the hot unit (h / 8 whole rows of one of its 8x8 tiles), the others the group's light
// units' samples in order.
__device__ __forceinline__ unsigned mix_sample(const PcParams& p, unsigned code, unsigned o) {
    const unsigned lg = (code >> 28) & 3u, sub = (code >> 24) & 7u, g = code & 0xFFFFFFu;
    const unsigned h = 64u >> lg, vv = (sub << 8) | o, w = vv >> 6, l = vv & 63u;
    const unsigned c = w * (64u - h) + (l - h);
    const unsigned slot = l < h ? 0u : 1u + (c >> 8), off = l < h ? w * h + l : (c & 255u);
    return p.ugrp[(g << lg) + slot] * 256u + off;
}

// closest-hit chains of one phase (raytracer.cpp:385-439 minus the shading):
// record each hit, queue its shadow tasks, follow (or hand on) mirrors.
// DBG (k_chain<false, true>, rt_primary_hits_production): also store each sample's level-0 hit (PcParams::dbg_t,
// dbg_m) -- the same walk, two stores added.
// nconts (phase B): the continuations.  RL (a whole lone frame, PcParams::rlists): read in region order through
// g_pref (region_prefix); otherwise k_pack_a's packed list.
template <bool COUNT, bool CONT, bool BQ = CONT, bool DBG = false, bool RL = false>
__device__ void chain_body(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, unsigned blk, unsigned G,
                           const PhaseOut& o, unsigned nconts = 0) {
    WalkStack stk;
    Work w;
    uint32_t nprim = 0, nrefl = 0, nskip = 0, nhit = 0, ncont = 0;
    const int nl = s.nlights;
    unsigned nb;
    if (CONT) nb = chunk_count(min(nconts, p.cb), G, blk, (unsigned)p.tchunk);   // the rest: k_fallback
    else nb = group_samples((unsigned)p.n0, G, blk);
    // dynamic units (phase A, p.dyn_units > 0): the workgroup's k-th 256-sample unit is not
    // blk + k*G but the next one of a launch-wide counter (p.totals[3], zeroed before the launch),
    // taken when the workgroup reaches it, so a workgroup whose samples were cheap takes more of
    // them and no workgroup waits out a fixed share.  At most p.dyn_units units per workgroup
    // (its shadow and continuation queues are sized for that many).
    const bool dyn = !CONT && p.dyn_units > 0;
    const unsigned units = ((unsigned)p.n0 + 255u) / 256u;
    if (dyn) nb = (unsigned)p.dyn_units * 256u;
    unsigned* const sq = o.sq + (size_t)blk * o.scap;
    int st = kIdle;
    bool exhausted = nb == 0;
    unsigned path = 0, cix = 0;   // sample slot; continuation index (phase B: its deeper records)
    int k = 0;
    Ray r;
    Walk wk;
    unsigned t_grab = 0, tsteps = 0, twit = 0, wit = 0;   // trace: grab time, own steps, wave steps
    unsigned ssteps = 0;     // phase A (p.urank): walk steps of the lane's current sample
    StepStat stat;
    while (true) {
        // (1) epilogue of finished walks: record, queue shadow tasks, reflect or hand on
        if (st == kDone) {
            const HitRec h = wk.best;
            const bool hit = h.prim >= 0;
            V nn{0.0f, 0.0f, 0.0f}, hitp{0.0f, 0.0f, 0.0f};
            int mat = 0, code = 0;
            const size_t lvp = rec_id(p, k, path, cix);
            if (hit) {
                hit_surface(s, r, h, &nn, &mat, &code);
                hitp = add(r.o, mul(r.d, h.t));
                rec_write(p, lvp, hitp, code, r.d, mat);
                if (COUNT) nhit++;
            }
            if (DBG && !CONT && k == 0) {
                int row, col;
                if (slab_sample_pixel(p, path, &row, &col)) {
                    p.dbg_t[(size_t)row * p.wi + col] = h.t;
                    p.dbg_m[(size_t)row * p.wi + col] = hit ? mat : 0;
                }
            }
            // one shadow task per light (:399-404) whose ray can change the pixel (light_needed; the
            // counting passes trace every one, as the reference does); light-major within the wave
            const unsigned own0 = (unsigned)(lvp * nl);
            if (CONT && BQ && kBq > 0 && __ballot(hit))
                __builtin_amdgcn_s_waitcnt(0);     // phase B: the record stores have completed before the
                                                   // owner ids are published to the workgroup (a workgroup
                                                   // fence alone does not wait for them on gfx950)
            for (int l = 0; l < nl; ++l) {
                bool want = hit;
                if (hit && s.cull_shadows && !light_needed(s, hitp, nn, l)) {
                    if (COUNT) nskip++;            // the reference traces it: counted as its shadow ray
                    if (!COUNT || s.count_prod) {
                        want = false;
                        p.occ[lvp * nl + l] = 1;   // shaded as occluded: the same sum (light_needed)
                    }
                }
                const unsigned long long m = __ballot(want);
                if (!m) continue;
                const unsigned cnt = (unsigned)__popcll(m), rank = lane_rank(m);
                bool queued = false;
                if (CONT && BQ && kBq > 0) {
                    // phase B: into the workgroup queue (walked by its finished waves)
                    const int leader = __ffsll((unsigned long long)m) - 1;
                    unsigned base = 0;
                    if (lane_id() == leader) base = atomicAdd(&g_bq_tail, cnt);
                    base = __shfl(base, leader, 64);
                    if (base + cnt <= (unsigned)p.bq_cap) {
                        if (want) __atomic_store_n(&g_bq[base + rank], own0 + (unsigned)l, __ATOMIC_RELAXED);
                        queued = true;
                    } else if (want && base + rank < (unsigned)p.bq_cap) {
                        __atomic_store_n(&g_bq[base + rank], kBqSkip, __ATOMIC_RELAXED);   // spilled: mark the slot
                    }
                }
                if (!queued) {
                    const unsigned base = wave_grab_lds(&g_scnt, m);
                    if (want) sq[base + rank] = own0 + (unsigned)l;
                }
            }
            bool ends = true;
            const int cbit = CONT ? kPathCont : 0;
            if (!hit) {                                                          // :442-449
                p.pinfo[path] = k | ((k == 0 ? kEndBg : kEndZero) << 8) | cbit;
            } else if (!s.mats[mat - 1].is_mirror) {
                p.pinfo[path] = (k + 1) | (kEndLast << 8) | cbit;
            } else if (k >= s.max_depth) {        // child beyond MaxRecursionDepth: 0 (:387-389)
                p.pinfo[path] = (k + 1) | (kEndZero << 8) | cbit;
            } else {
                ends = false;
            }
            if (CONT && !COUNT && ends && p.pdepth) p.pdepth[path] = (uint8_t)min(k + 1, 255);
            const bool handoff = !ends && k >= o.kinline;                      // deeper levels: next phase
            const unsigned long long cm = __ballot(handoff);
            if (handoff) {
                if (COUNT) ncont++;
                // a continuation the previous frame saw go deep (PcParams::pdepth): from the region's end, packed first
                const bool deep = !CONT && !COUNT && p.pdepth && p.pdepth[path] >= (uint8_t)p.deep_min;
                const unsigned long long dm = __ballot(deep);
                unsigned slot;
                if (deep) {
                    slot = o.ccap - 1u - (wave_grab_lds(&g_dcnt, dm) + lane_rank(dm));
                } else {
                    const unsigned long long sm = cm & ~dm;
                    slot = wave_grab_lds(&g_ccnt, sm) + lane_rank(sm);
                }
                o.cq[(size_t)blk * o.ccap + slot] = (unsigned)((size_t)k * p.cap + path);
                p.pinfo[path] = kPathCont;        // continued in phase B (finish_pixels' order)
                if (lvp < p.dbase) p.tail[path] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);   // reflect_from_record
            }
            if (ends || handoff) {
                st = kIdle;
                if (!CONT && !COUNT && p.urank && ssteps >= kHotSteps[kUnitClasses - 2]) atomicMax(&p.ucost[path >> 8], ssteps);
                if (kTraceBuild && p.trace && !CONT) { p.trace[2 * path] = t_grab; p.trace[2 * path + 1] = (unsigned)wall_clock64(); }
                if (kTraceBuild && p.trace && CONT) {       // phase B: {grab, end, last level, walk steps} after A's entries
                    unsigned* tb = p.trace + 2 * ((size_t)p.cap + p.trace_blocks) + 4 * (size_t)path;
                    tb[0] = t_grab; tb[1] = (unsigned)wall_clock64(); tb[2] = (unsigned)k | ((wit - twit) << 8); tb[3] = tsteps;
                }
            } else {
                const V dk = r.d;
                r = reflect_ray(s, hitp, nn, r.d);
                ++k;
                nrefl++;
                if (!COUNT && defer_closest(s, r, true)) {     // the rest of this path: k_fallback
                    if (lvp < p.dbase) p.tail[path] = make_float4(dk.x, dk.y, dk.z, 0.0f);   // reflect_from_record
                    // (k_fallback's path; fallback_chain's pinfo write clears the bit again for a phase-A path,
                    // so fin_cont's second loop still finishes its pixel)
                    if (!CONT) p.pinfo[path] = kPathCont;
                    fb_chain(p, (unsigned)lvp);
                    st = kIdle;
                } else {
                    st = (COUNT ? walk_begin<COUNT>(s, r, wk, w) : walk_begin_wide(s, r, wk)) ? kTrav : kDone;
                }
            }
        }
        // (2) refill idle lanes with this workgroup's next samples / continuations
        if (!exhausted) {
            const unsigned long long idle = __ballot(st == kIdle);
            if (idle) {
                stat.refill(idle);
                const unsigned base = wave_grab_lds(&g_head, idle);
                if (base + (unsigned)__popcll(idle) >= nb) exhausted = true;
                unsigned uid = 0;           // dyn: the unit of this lane's sample
                if (dyn) {
                    // the wave whose grab holds a unit's first sample takes that unit from the counter,
                    // once the previous unit is taken: a workgroup's units come in order, so a unit
                    // beyond the counter's end means no later one either
                    const unsigned jf = (base + 255u) >> 8;
                    if (lane_id() == 0 && jf * 256u < base + (unsigned)__popcll(idle) && jf < (unsigned)p.dyn_units) {
                        bool late = false;          // spin_over: the previous unit never came
                        unsigned n = 0;
                        if (jf > 0)
                            while (lds_load(&g_uid[jf - 1]) == kUidUnset) {
                                if (spin_over(s, n)) { late = true; break; }
                                __builtin_amdgcn_s_sleep(1);
                            }
                        const unsigned u = late ? units : atomicAdd(&p.totals[3], 1u);
                        lds_store(&g_uid[jf], u < units ? unit_order(p, u, units) : kUidNone);
                    }
                    const unsigned v = base + lane_rank(idle);
                    if (st == kIdle && v < nb) {
                        unsigned n = 0;
                        while ((uid = lds_load(&g_uid[v >> 8])) == kUidUnset) {
                            if (spin_over(s, n)) { uid = kUidNone; break; }
                            __builtin_amdgcn_s_sleep(1);
                        }
                    }
                    if (__any(st == kIdle && v < nb && uid == kUidNone)) exhausted = true;
                }
                if (st == kIdle) {
                    const unsigned v = base + lane_rank(idle);
                    if (v < nb && uid != kUidNone) {
                        if (CONT) {
                            const unsigned j = chunk_task(v, G, blk, (unsigned)p.tchunk);
                            // RL: the region-order list, and for k_finish its phase-B records' index (cid) and
                            // the packed entry; otherwise k_pack_a's list and cid
                            const unsigned lvp = RL ? cont_entry(p, j) : p.cflat[j];
                            if (RL) {
                                p.cid[lvp % (unsigned)p.cap] = j;
                                p.cflat[j] = lvp;
                            }
                            cix = j;
                            if (kTraceBuild && p.trace) { t_grab = (unsigned)wall_clock64(); tsteps = 0; twit = wit; }
                            path = lvp % (unsigned)p.cap;
                            k = (int)(lvp / (unsigned)p.cap) + 1;
                            r = reflect_from_record(s, p, lvp, path);
                            nrefl++;
                            if (!COUNT && defer_closest(s, r, true)) fb_chain(p, lvp);
                            else st = (COUNT ? walk_begin<COUNT>(s, r, wk, w) : walk_begin_wide(s, r, wk)) ? kTrav : kDone;
                        } else {
                            const unsigned idx = dyn && (uid & kUidMix) ? mix_sample(p, uid, v & 255u)
                                                 : (dyn ? uid : blk + (v >> 8) * G) * 256u + (v & 255u);
                            if (slab_sample_ray(p, idx, &r)) {
                                path = idx;
                                k = 0;
                                ssteps = 0;
                                if (kTraceBuild && p.trace) t_grab = (unsigned)wall_clock64();
                                nprim++;
                                if (s.max_depth < 0) p.pinfo[path] = 0 | (kEndZero << 8);   // depth 0 > max: black
                                else if (!COUNT && defer_closest(s, r, false)) {
                                    // (k_fallback's path; fallback_chain's pinfo write clears the bit again)
                                    p.pinfo[path] = kPathCont;
                                    fb_chain(p, kFbEye | path);
                                }
                                else st = (COUNT ? walk_begin<COUNT>(s, r, wk, w) : walk_begin_wide(s, r, wk)) ? kTrav : kDone;
                            }
                        }
                    }
                }
            }
        }
        if (!__any(st != kIdle)) {
            if (exhausted) break;
            continue;
        }
        // (3) walk until enough lanes need service
        const int thresh = exhausted ? 0 : (CONT ? p.brefill : p.refill);
        while (true) {
            if (__popcll(__ballot(st == kTrav)) <= thresh ||
                __popcll(__ballot(st == kDone)) >= (CONT ? (exhausted ? p.btail : p.bservice) : p.service))
                break;
            stat.step(st == kTrav, wk.cur >= 0, RT_STEP_STATS && st == kTrav && wk.tree == nullptr && leaf_postponed(s.leaf_wait, wk));
            if (kTraceBuild && CONT && p.trace) ++wit;
            if (st == kTrav) {
                if (kTraceBuild && CONT && p.trace) ++tsteps;
                if (!CONT) ++ssteps;
                if (closest_step_timed<COUNT, CONT>(s, r, stk, wk, w) || walk_runaway(s, wk)) st = kDone;
            }
        }
    }
    stat.flush(CONT ? 1 : 0);
    uint32_t nshadow = 0;
    if (COUNT) {
        wave_add_counter(&p.counters[CONT ? kCntBWalkBytes : kCntAWalkBytes], w.nodes);
        wave_add_counter(&p.counters[CONT ? kCntBWalks : kCntAWalks], nprim + nrefl);
        wave_add_counter(&p.counters[CONT ? kCntBHits : kCntAHits], nhit);
        if (!CONT) wave_add_counter(&p.counters[kCntConts], ncont);
    }
    if (CONT && BQ && kBq > 0) {
        if (lane_id() == 0) atomicSub(&g_bq_prod, 1u);      // this wave produces no more shadow tasks
        Work wq;                                            // the queue's walks, counted apart (kCntBQ*)
        nshadow = bq_consume<COUNT>(s, p, stk, wq);
        w.nodes += wq.nodes;
        w.tris += wq.tris;
        w.spheres += wq.spheres;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        o.scount[blk] = g_scnt;
        if (!CONT) {
            o.ccount[blk] = g_ccnt;
            if (p.ccntd) p.ccntd[blk] = g_dcnt;
        }
    }
    if (COUNT) {
        // shadow rays not traced (light_needed): counter 6; a production counting pass (count_prod)
        // skips them, and counts them among the shadow rays here so counter 1 stays the reference's
        wave_add_counter(&p.counters[1], (CONT ? nshadow : 0u) + (s.count_prod ? nskip : 0u));
        wave_add_counter(&p.counters[6], nskip);
        wave_add_counter(&p.counters[0], nprim);
        wave_add_counter(&p.counters[2], nrefl);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// any-hit of the packed shadow tasks j = blk, blk+G, ... < total
// (raytracer.cpp:227-280).
template <bool COUNT, class TL>
__device__ void occlude_body(const rtk::DevScene& s, const PcParams& p, unsigned blk, unsigned G,
                             TL tasks, unsigned total, int role) {   // role 0: A's tasks, 1: B's overflow
    WalkStack stk;
    Work w;
    uint32_t nrays = 0;
    const unsigned t_start = kTraceBuild && p.trace ? (unsigned)wall_clock64() : 0u;
    const unsigned n = chunk_count(total, G, blk, (unsigned)p.ochunk);
    bool active = false, exhausted = n == 0;
    Ray r;
    float tlim = 0.0f;
    unsigned owner = 0;
    Walk wk;
    StepStat stat;
    while (true) {
        if (!exhausted) {
            const unsigned long long idle = __ballot(!active);
            if (idle) {
                stat.refill(idle);
                const unsigned base = wave_grab_lds(&g_head, idle);
                if (base + (unsigned)__popcll(idle) >= n) exhausted = true;
                if (!active) {
                    const unsigned idx = base + lane_rank(idle);
                    if (idx < n) {
                        const unsigned j = chunk_task(idx, G, blk, (unsigned)p.ochunk);
                        owner = tasks[j];
                        r = shadow_from_record(s, p, owner, &tlim);
                        nrays++;
                        if (!COUNT && defer_any(s, r)) fb_shadow(p, owner);
                        else if (COUNT ? walk_begin<COUNT>(s, r, wk, w, true) : walk_begin_wide(s, r, wk, true)) active = true;
                        else p.occ[owner] = 0;
                    }
                }
            }
        }
        if (!__any(active)) {
            if (exhausted) break;
            continue;
        }
        const int thresh = exhausted ? 0 : p.orefill;
        while (__popcll(__ballot(active)) > thresh) {
            stat.step(active, wk.cur >= 0, RT_STEP_STATS && active && wk.tree == nullptr && leaf_postponed(s.leaf_wait_any, wk));
            if (active) {
                const int res = occl_step_timed<COUNT>(s, r, tlim, stk, wk, w);
                if (res || walk_runaway(s, wk)) {
                    p.occ[owner] = res == 2 ? 1 : 0;
                    active = false;
                }
            }
        }
    }
    stat.flush(2);
    if (kTraceBuild && p.trace && threadIdx.x == 0 && blk < (unsigned)p.ogrid) {
        p.trace[2 * ((size_t)p.cap + blk)] = t_start;
        p.trace[2 * ((size_t)p.cap + blk) + 1] = (unsigned)wall_clock64();
    }
    if (COUNT) {
        wave_add_counter(&p.counters[role ? kCntBOBytes : kCntASBytes], w.nodes);
        wave_add_counter(&p.counters[role ? kCntBORays : kCntASRays], nrays);
        wave_add_counter(&p.counters[1], nrays);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// Any-hit walks with a wave leaf queue (A's shadow rays: k_occlude, and k_mix's shadow role).
// Any hit is order-free (raytracer.cpp:227-280: the answer is whether SOME reachable leaf -- its
// exact box hit -- holds a primitive with t < dist), so a lane that reaches a leaf record does not
// test it: it appends (lane, record) to its wave's LDS queue and walks on.  Interior steps then run
// with every walking lane (no lane waits at a leaf, no step issues both kinds), and once 64 records
// are queued (or no lane walks) the whole wave tests 64 of them at once, each lane one record
// against its owner lane's ray (fetched by lane shuffles).  A hit marks the owner occluded, which
// ends its walk; a lane's ray is unoccluded when its walk is over and none of its queued records
// hit.  A lane takes its next task only once its queued records are all tested.  The same leaves
// are tested with the same arithmetic as wide_any_step, so the answer is the same; an occluded ray
// may walk a few more nodes before its record is tested.
// LDS: the walk-stack array g_lstk, re-cut as ints (this role has no closest-hit walks): per lane
// kOStk stack entries + one sink entry, per wave a kLq-entry queue, per lane its queued count.
// ---------------------------------------------------------------------------
constexpr int kOStk = 22;                 // LDS stack entries per lane (deeper ones in scratch)
constexpr int kLq = 128;                  // queued leaf records per wave (tested 64 at a time)
constexpr int kLqSrcShift = 25;           // queue entry: leaf-record offset | owner lane << 25
static_assert(2 * (kLdsStackEntries + 1) * kBlock >= (kOStk + 1) * kBlock + (kBlock / 64) * kLq + kBlock,
              "the occlusion walker's stack, queues and counts must fit in g_lstk");
__shared__ unsigned g_lqn[kBlock / 64];            // per wave: queued records
__shared__ unsigned long long g_lhit[kBlock / 64]; // per wave: lanes whose ray a tested record occludes

__device__ __forceinline__ int* oq_base() { return reinterpret_cast<int*>(g_lstk); }
__device__ __forceinline__ void ostk_lds_put(int i, int v) { oq_base()[i * kBlock + threadIdx.x] = v; }
__device__ __forceinline__ int ostk_lds_at(int i) { return oq_base()[i * kBlock + threadIdx.x]; }
__device__ __forceinline__ unsigned* lq_base() {
    return reinterpret_cast<unsigned*>(oq_base() + (kOStk + 1) * kBlock) + (threadIdx.x >> 6) * kLq;
}
__device__ __forceinline__ int* lpend_base() { return oq_base() + (kOStk + 1) * kBlock + (kBlock / 64) * kLq; }

struct OStack {   // int entries: [0, kOStk) in LDS, deeper in scratch
    int d[dl::kMaxStack > kOStk ? dl::kMaxStack - kOStk : 1];
    __device__ __forceinline__ void put(int i, int v) {
        if (i < kOStk) ostk_lds_put(i, v);
        else d[i - kOStk] = v;
    }
    __device__ __forceinline__ int at(int i) { return i < kOStk ? ostk_lds_at(i) : d[i - kOStk]; }
};

// Test 64 queued records of this wave (lane j: entry j < n), mark the owners they occlude, retire
// the entries and shift the rest down.
__device__ __forceinline__ void lq_flush(const rtk::DevScene& s, const Ray& r, float tlim, unsigned nq) {
    const int lane = lane_id(), wave = (int)(threadIdx.x >> 6);
    unsigned* const q = lq_base();
    const unsigned n = min(nq, 64u);
    const unsigned e = (unsigned)lane < n ? q[lane] : 0u;
    const int src = (int)(e >> kLqSrcShift);
    // a record of a ray already found occluded is retired untested
    const bool valid = (unsigned)lane < n &&
                       !((__atomic_load_n(&g_lhit[wave], __ATOMIC_RELAXED) >> src) & 1ull);
    // the owner lane's ray (every lane takes part in the shuffles)
    Ray o;
    o.o = V{__shfl(r.o.x, src, 64), __shfl(r.o.y, src, 64), __shfl(r.o.z, src, 64)};
    o.d = V{__shfl(r.d.x, src, 64), __shfl(r.d.y, src, 64), __shfl(r.d.z, src, 64)};
    o.inv = V{__shfl(r.inv.x, src, 64), __shfl(r.inv.y, src, 64), __shfl(r.inv.z, src, 64)};
    const float olim = __shfl(tlim, src, 64);
    // the rest of the queue moves down (all reads before any write: one wave, LDS in order)
    const unsigned rest = nq - n;
    const unsigned mv = (unsigned)lane < rest ? q[n + lane] : 0u;
    if (valid) {
        const float4* L = s.lrec + (e & ((1u << kLqSrcShift) - 1u));
        const float4 h0 = L[0], h1 = L[1], c0 = L[2], c1 = L[3], c2 = L[4];
        float bt;
        bool hit = false;
        if (box_hit_fast(o, h0, h1, &bt)) {          // the reference leaf's exact box (NaN-free ray)
            const int cnt = __float_as_int(h0.w), slot0 = __float_as_int(h1.w);
            hit = for_leaf_prims(L, slot0, cnt, c0, c1, c2, [&](int, const float4& p0, const float4& p1, const float4& p2) {
                float t;
                const bool h = __float_as_int(p0.w) >= 0 ? tri_hit(o, p0, p1, p2, &t) : sphere_hit(o, p0, p1, &t);
                return h && t < olim;
            });
        }
        if (hit) atomicOr(&g_lhit[wave], 1ull << src);
    }
    if ((unsigned)lane < n) atomicSub(&lpend_base()[(wave << 6) + src], 1);
    if ((unsigned)lane < rest) q[lane] = mv;
    if (lane == 0) __atomic_store_n(&g_lqn[wave], rest, __ATOMIC_RELAXED);
}

// The shadow tasks tasks[j] of this workgroup (as occlude_body) with the leaf queue; production only.
template <class TL>
__device__ void occlude_queue_body(const rtk::DevScene& s, const PcParams& p, unsigned blk, unsigned G,
                                   TL tasks, unsigned total) {
    const int lane = lane_id(), wave = (int)(threadIdx.x >> 6);
    const unsigned n = chunk_count(total, G, blk, (unsigned)p.ochunk);
    const UDiv och((unsigned)p.ochunk), nld((unsigned)s.nlights);
    // the queue count, the hit mask and the queued counts are written by other lanes of the wave:
    // every read is an atomic load (no value kept in a register across the loop)
    if (lane == 0) {
        __atomic_store_n(&g_lqn[wave], 0u, __ATOMIC_RELAXED);
        __atomic_store_n(&g_lhit[wave], 0ull, __ATOMIC_RELAXED);
    }
    int* const pend = lpend_base() + threadIdx.x;
    __atomic_store_n(pend, 0, __ATOMIC_RELAXED);
    OStack stk;
    bool exhausted = n == 0;
    bool have = false, trav = false, done = false;   // a task; walking it; its answer written
    Ray r;
    r.o = r.d = r.inv = V{0.0f, 0.0f, 0.0f};
    float tlim = 0.0f;
    unsigned owner = 0;
    int cur = 0, sp = 0, steps = 0;
    unsigned spins = 0;      // consecutive iterations without a step, a test, a retired task or a grab (spin_over)
    while (true) {
        bool prog = false;   // this iteration made progress (wave-uniform)
        // (1) retire finished tasks: occluded (a record hit), or walked with every record tested
        {
            const unsigned long long hm = __atomic_load_n(&g_lhit[wave], __ATOMIC_RELAXED);
            if (have && !done && ((hm >> lane) & 1ull)) {
                p.occ[owner] = 1;
                done = true;
                trav = false;
            }
            const bool retire = have && !trav && __atomic_load_n(pend, __ATOMIC_RELAXED) == 0;
            if (retire) {
                if (!done) p.occ[owner] = 0;
                have = false;
            }
            prog = __any(retire);
            const unsigned long long freed = __ballot(!have) & hm;
            if (freed && lane == 0) atomicAnd(&g_lhit[wave], ~freed);   // the next task starts unmarked
        }
        // (2) refill lanes without a task
        if (!exhausted) {
            const unsigned long long idle = __ballot(!have);
            if (idle && __popcll(idle) >= 64 - p.orefill) {
                prog = true;
                const unsigned base = wave_grab_lds(&g_head, idle);
                if (base + (unsigned)__popcll(idle) >= n) exhausted = true;
                if (!have) {
                    const unsigned idx = base + lane_rank(idle);
                    if (idx < n) {
                        owner = tasks[chunk_task(idx, G, blk, och)];
                        r = shadow_from_record(s, p, owner, &tlim, nld);
                        if (defer_any(s, r)) {
                            fb_shadow(p, owner);
                        } else if (s.nnodes <= 0) {   // nothing to hit (walk_begin)
                            p.occ[owner] = 0;
                        } else {
                            have = true;
                            trav = true;
                            done = false;
                            cur = s.swroot;
                            sp = 0;
                            steps = 0;
                        }
                    }
                }
            }
        }
        if (!__any(have)) {
            if (exhausted) break;
            continue;
        }
        // (3) walk: queue the leaf records reached, step the interior nodes, until 64 records wait
        //     or no lane walks (or, with tasks left, too few lanes walk)
        while (true) {
            // drain leaf codes into the queue (each pass adds at most one record per lane)
            while (true) {
                const bool atleaf = trav && cur < 0;
                const unsigned long long lm = __ballot(atleaf);
                if (!lm) break;
                const unsigned nq = __atomic_load_n(&g_lqn[wave], __ATOMIC_RELAXED);
                if (nq + (unsigned)__popcll(lm) > (unsigned)kLq) break;
                if (atleaf) {
                    lq_base()[nq + lane_rank(lm)] = ((unsigned)cur & ~dl::kLeafBit) | ((unsigned)lane << kLqSrcShift);
                    atomicAdd(pend, 1);
                    if (sp > 0) cur = stk.at(--sp);
                    else trav = false;
                }
                if (lane == 0) __atomic_store_n(&g_lqn[wave], nq + (unsigned)__popcll(lm), __ATOMIC_RELAXED);
            }
            const unsigned long long im = __ballot(trav && cur >= 0);
            if (__atomic_load_n(&g_lqn[wave], __ATOMIC_RELAXED) >= 64u || !im) break;
            if (__popcll(__ballot(have && !trav)) >= p.lq_wait) break;
            if (!exhausted && __popcll(__ballot(have)) <= p.orefill) break;
            prog = true;
            if (trav && cur >= 0) {
                constexpr int W = dl::kWideSlots;
                WideNode nd;
                wide_load(s.swnodes, cur, nd);
                float tmn[W], tmx[W];
                wide_slabs(nd, r, tmn, tmx);
                uint32_t vs = 0;                  // empty slots: +inf / -inf planes, never hit
#pragma unroll
                for (int c = 0; c < W; ++c) vs |= (uint32_t)any_slot_valid(tmn[c], tmx[c]) << c;
                if (vs) {
                    if (__all(!(trav && cur >= 0) || sp + W <= kOStk)) {
                        // every hit slot written unconditionally (misses to the sink entry), the
                        // first on top, which is the next node
#pragma unroll
                        for (int c = 0; c < W; ++c)
                            ostk_lds_put(((vs >> c) & 1u) ? sp + __builtin_popcount(vs >> (c + 1)) : kOStk, wide_code(nd, c));
                        sp += __builtin_popcount(vs) - 1;
                        cur = ostk_lds_at(sp);
                    } else {
                        const uint32_t first = (uint32_t)__builtin_ctz(vs), pm = vs & (vs - 1u);
                        int next = 0;
#pragma unroll
                        for (int c = 0; c < W; ++c) {
                            next = (uint32_t)c == first ? wide_code(nd, c) : next;
                            if ((pm >> c) & 1u) stk.put(sp + __builtin_popcount(pm & ((1u << c) - 1u)), wide_code(nd, c));
                        }
                        sp += __builtin_popcount(pm);
                        cur = next;
                    }
                } else if (sp > 0) {
                    cur = stk.at(--sp);
                } else {
                    trav = false;
                }
                if (trav && ++steps > s.walk_cap) {          // walk_runaway: ended as unoccluded
                    __hip_atomic_fetch_or(s.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    trav = false;
                }
            }
        }
        // (4) test queued records: 64 at a time, or what is left once no lane walks
        const unsigned nq = __atomic_load_n(&g_lqn[wave], __ATOMIC_RELAXED);
        if (nq >= 64u || (nq > 0u && (!__any(trav) || __popcll(__ballot(have && !trav)) >= p.lq_wait))) {
            lq_flush(s, r, tlim, nq);
            prog = true;
        }
        if (prog) spins = 0;
        else if (spin_over(s, spins)) break;
    }
}

__device__ __forceinline__ PhaseOut phase_a(const PcParams& p) {
    return PhaseOut{p.sqA, p.scapA, p.scntA, p.cq, p.ccapA, p.ccnt, p.kinline};
}
__device__ __forceinline__ PhaseOut phase_b(const PcParams& p) {
    return PhaseOut{p.sqB, p.scapB, p.scntB, nullptr, 0u, nullptr, 1 << 30};
}

// Phase A: every sample, levels [0, kinline].
template <bool COUNT, bool DBG = false>
__global__ __launch_bounds__(kBlock, COUNT ? 4 : RT_WAVES_PER_EU) void k_chain(rtk::DevScene s, rtk::Eye e, PcParams p) {
    if (threadIdx.x == 0) g_ccnt = g_dcnt = 0;
    if (threadIdx.x < kDynUnits) g_uid[threadIdx.x] = kUidUnset;
    block_init(s);
    chain_body<COUNT, false, false, DBG>(s, e, p, blockIdx.x, gridDim.x, phase_a(p));
}

// Region b of a per-workgroup queue (q[b*cap ..], cnt[b] entries) copied to
// its place in the packed array: the consumers then index tasks directly.
// Workgroup 0 stores the total.  cid (continuations): cid[sample] = the packed index of its continuation
// (its phase-B records).
__device__ unsigned pack_region(const unsigned* q, unsigned cap, const unsigned* cnt, int nreg, unsigned* flat,
                                unsigned* total, unsigned b, unsigned* cid = nullptr, unsigned ncap = 1,
                                bool top = false, unsigned base = 0) {
    // (top: the region's entries are at its end, q[b * cap + cap - 1 - k]; base: the packed array's offset)
    __shared__ unsigned s_before, s_all;
    if (threadIdx.x == 0) { s_before = 0; s_all = 0; }
    __syncthreads();
    unsigned before = 0, all = 0;
#pragma unroll 8
    for (int i = threadIdx.x; i < nreg; i += kBlock) {
        const unsigned c = cnt[i];
        all += c;
        if ((unsigned)i < b) before += c;
    }
    if (all) atomicAdd(&s_all, all);
    if (before) atomicAdd(&s_before, before);
    __syncthreads();
    const unsigned off = base + s_before, n = cnt[b];
    const unsigned* src = q + (size_t)b * cap;
    auto at = [&](unsigned k) { return top ? src[cap - 1u - k] : src[k]; };
    unsigned k = threadIdx.x;
    for (; k + 3 * kBlock < n; k += 4 * kBlock) {          // four loads in flight per lane
        const unsigned v0 = at(k), v1 = at(k + kBlock), v2 = at(k + 2 * kBlock), v3 = at(k + 3 * kBlock);
        flat[off + k] = v0; flat[off + k + kBlock] = v1; flat[off + k + 2 * kBlock] = v2; flat[off + k + 3 * kBlock] = v3;
        if (cid) {
            cid[(v0 & ~kFbEye) % ncap] = off + k; cid[(v1 & ~kFbEye) % ncap] = off + k + kBlock;
            cid[(v2 & ~kFbEye) % ncap] = off + k + 2 * kBlock; cid[(v3 & ~kFbEye) % ncap] = off + k + 3 * kBlock;
        }
    }
    for (; k < n; k += kBlock) {
        const unsigned v = at(k);
        flat[off + k] = v;
        if (cid) cid[(v & ~kFbEye) % ncap] = off + k;
    }
    const unsigned tot = s_all;
    if (total && b == 0 && threadIdx.x == 0) *total = tot;
    __syncthreads();
    return tot;
}

// The next frame's phase-A unit order (PcParams::uorder, k_mix's last shadow-role workgroup in lone frames):
// the units by cost class (kHotSteps, the heaviest class first; seven classes: 9 us less per repeated C3
// frame than three, profiles/r05_ab_rank.txt), each class in the column order (the table ucol, made on the
// host); ucost cleared for the next frame's marks.  One workgroup: thread t takes a contiguous run of the
// column order; the per-class offsets come from block-wide exclusive scans of the runs' class counts.
__device__ __forceinline__ int unit_class(unsigned c) {
#pragma unroll
    for (int i = 0; i < kUnitClasses - 1; ++i)
        if (c >= kHotSteps[i]) return i;
    return kUnitClasses - 1;
}
// The mixed deal pays where the heavy units' lockstep waves are phase A's tail, not where the launch's bulk
// outlasts them: C3 (6.3 units per k_chain workgroup) one frame -4 %, C3 at SSAA 2 (25 per workgroup) +1 %,
// 1024^2 scenes (3.2) +-1.5 % (profiles/r06_mix_*.jsonl).
constexpr unsigned kMixRounds = 12;
__device__ void rank_units(const PcParams& p) {
    __shared__ unsigned s_wave[kBlock / 64][kUnitClasses];
    const unsigned units = ((unsigned)p.n0 + 255u) / 256u;
    const unsigned per = (units + kBlock - 1) / kBlock, j0 = min(units, threadIdx.x * per), j1 = min(units, j0 + per);
    unsigned mine[kUnitClasses] = {};          // class counts of this thread's run
    for (unsigned j = j0; j < j1; ++j) {
        const int cls = unit_class(p.ucost[p.ucol[j]]);
#pragma unroll
        for (int c = 0; c < kUnitClasses; ++c) mine[c] += c == cls ? 1u : 0u;
    }
    const int lane = lane_id(), wave = (int)(threadIdx.x >> 6);
    unsigned inc[kUnitClasses];                // inclusive scans in the wave, then over the waves
#pragma unroll
    for (int c = 0; c < kUnitClasses; ++c) {
        inc[c] = mine[c];
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned v = __shfl_up(inc[c], off, 64);
            if (lane >= off) inc[c] += v;
        }
        if (lane == 63) s_wave[wave][c] = inc[c];
    }
    __syncthreads();
    unsigned at[kUnitClasses], base = 0, nhot = 0;
    const int mcls = p.mix_cls & 0xff;
#pragma unroll
    for (int c = 0; c < kUnitClasses; ++c) {
        unsigned before = 0, total = 0;
        for (int w = 0; w < kBlock / 64; ++w) {
            if (w < wave) before += s_wave[w][c];
            total += s_wave[w][c];
        }
        at[c] = base + before + inc[c] - mine[c];
        base += total;
        if (c < mcls) nhot += total;
    }
    // the mixed deal (PcParams::ugrp): groups of G = 2^lg units, all in the resident workgroups' first units
    // (so every hot unit starts at once; with more hot units than that, the heaviest grid / G), and only in
    // launches of at most kMixRounds units per workgroup
    unsigned lg = (unsigned)(p.mix_cls >> 8) & 3u;
    if (lg == 0) {
        lg = 3;
        while (lg > 1 && (nhot << lg) > (unsigned)p.grid) --lg;
    }
    nhot = min(nhot, (unsigned)p.grid >> lg);
    if (nhot == 0 || (nhot << lg) > units || units > kMixRounds * (unsigned)p.grid) lg = 0, nhot = 0;
    const unsigned nlight = nhot * ((1u << lg) - 1u);
    for (unsigned j = j0; j < j1; ++j) {
        const unsigned u = p.ucol[j];
        const int cls = unit_class(p.ucost[u]);
        unsigned pos = 0;
#pragma unroll
        for (int c = 0; c < kUnitClasses; ++c)     // (no dynamic index into at[]: it would live in scratch)
            if (c == cls) pos = at[c]++;
        // heaviest-first position pos -> a group's hot unit, a group's light unit (the lightest nlight),
        // or a plain unit after the groups' virtual units
        if (pos < nhot) {
            p.ugrp[pos << lg] = u;
        } else if (pos >= units - nlight) {
            const unsigned q = units - 1u - pos, g = q / ((1u << lg) - 1u);
            p.ugrp[(g << lg) + 1u + (q - g * ((1u << lg) - 1u))] = u;
        } else {
            p.uorder[pos + nlight] = u;
        }
        p.ucost[u] = 0;
    }
    for (unsigned v = threadIdx.x; v < (nhot << lg); v += kBlock)
        p.uorder[v] = kUidMix | lg << 28 | (v & ((1u << lg) - 1u)) << 24 | v >> lg;
}

// After phase A (frame batches, the chunks of a larger lone frame): the continuations packed, and A's shadow
// tasks where they are not walked in place (p.sflatA: a lone frame's chunks).
__global__ __launch_bounds__(kBlock) void k_pack_a(PcParams p) {
    if (p.sflatA) pack_region(p.sqA, p.scapA, p.scntA, p.grid, p.sflatA, &p.totals[0], blockIdx.x);
    // the continuations the previous frame saw go deep first (PcParams::pdepth; k_chain queued them at their
    // regions' ends), then the rest
    unsigned nd = 0;
    if (p.ccntd) nd = pack_region(p.cq, p.ccapA, p.ccntd, p.grid, p.cflat, nullptr, blockIdx.x, p.cid, (unsigned)p.cap,
                                  true);
    const unsigned ns = pack_region(p.cq, p.ccapA, p.ccnt, p.grid, p.cflat, nullptr, blockIdx.x, p.cid,
                                    (unsigned)p.cap, false, nd);
    if (blockIdx.x == 0 && threadIdx.x == 0) p.totals[1] = nd + ns;
    if (p.cont_peak && blockIdx.x == 0 && threadIdx.x == 0) atomicMax(p.cont_peak, p.totals[1]);   // (its own write)
}
__global__ __launch_bounds__(kBlock) void k_pack_b(PcParams p) {
    pack_region(p.sqB, p.scapB, p.scntB, p.gb, p.sflatB, &p.totals[2], blockIdx.x);
}

// Workgroups [0, gb): phase B chains (continuations); the rest: phase A's shadow tasks.
// BQ: phase B's shadow tasks go to the workgroup LDS queue first (a lone frame: its waves whose
// chains are done walk them during the deep-chain tail); without it (frame batches) they all go to
// k_pack_b + k_occlude, and the kernel needs 26.7 instead of 32.8 KB of LDS and 96 VGPRs: 5 waves.
#ifndef RT_MIX_WAVES
#define RT_MIX_WAVES 4           // 4 waves/SIMD: no VGPR spills (5: 29 spilled); single frame 1.17-1.19 vs 1.22-1.24 ms
#endif
#ifndef RT_MIX_NOBQ_WAVES
#define RT_MIX_NOBQ_WAVES 5      // without the LDS queue: 96 VGPRs, no spills
#endif
// Shadow tasks where their phase left them (p.occ_inplace / occ_inplace_b): region r (phase workgroup
// r's queue) to workgroup w + k W, one region at a time -- no packed copy of 4 B in and out per task.
// which = 0: A's (k_occlude in frame batches, k_mix's shadow role in a lone frame), 1: B's overflow.
__device__ __forceinline__ void occlude_regions(const rtk::DevScene& s, const PcParams& p, int which, unsigned w,
                                                unsigned W) {
    const unsigned nreg = which ? (unsigned)p.gb : (unsigned)p.grid;
    const unsigned* const q = which ? p.sqB : p.sqA;
    const unsigned* const cnt = which ? p.scntB : p.scntA;
    const size_t qcap = which ? p.scapB : p.scapA;
    for (unsigned r = w; r < nreg; r += W) {
        if (r != w) {
            __syncthreads();                    // every wave is done with the previous region
            if (threadIdx.x == 0) g_head = 0;
            __syncthreads();
        }
        occlude_queue_body(s, p, 0, 1, flat_list(q + (size_t)r * qcap), cnt[r]);
    }
}

// RL (a whole lone frame, PcParams::rlists): phase A's lists read in their regions (g_pref) -- a separate
// instantiation, since the region code alone, never run, cost the packed variant 5 % in C5's big launches.
template <bool COUNT, bool BQ, bool RL = false>
__global__ __launch_bounds__(kBlock, BQ || COUNT ? RT_MIX_WAVES : RT_MIX_NOBQ_WAVES) void k_mix(rtk::DevScene s,
                                                                                                  rtk::Eye e, PcParams p) {
    const bool chain = blockIdx.x < (unsigned)p.gb;
    if (threadIdx.x == 0) g_ccnt = 0;
    if (BQ && chain && kBq > 0) bq_init();
    block_init(s);
    // the role's phase-A list: a whole lone frame's (p.rlists) continuations or A's shadow tasks in region order
    // (g_pref); otherwise packed by k_pack_a (which also stored their counts)
    unsigned total;
    if constexpr (RL) total = region_prefix(chain ? p.ccnt : p.scntA, (unsigned)p.grid);
    else total = chain ? p.totals[1] : p.totals[0];
    if (chain) {
        if (RL && blockIdx.x == 0 && threadIdx.x == 0) {
            p.totals[1] = total;                       // the launch's continuations (k_fallback, the host)
            if (p.cont_peak) atomicMax(p.cont_peak, total);
        }
        if (p.bprio) __builtin_amdgcn_s_setprio(3);    // the deep chains are the frame's critical path
        chain_body<COUNT, true, BQ, false, RL>(s, e, p, blockIdx.x, (unsigned)p.gb, phase_b(p), total);
    } else if constexpr (BQ) {                          // (the shadow role: lone frames only)
        const auto tl = [&] {
            if constexpr (RL) return shadow_regions_a(p);
            else return flat_list(p.sflatA);
        }();
        if constexpr (!COUNT && RT_LEAF_QUEUE) occlude_queue_body(s, p, blockIdx.x - p.gb, gridDim.x - p.gb, tl, total);
        else occlude_body<COUNT>(s, p, blockIdx.x - p.gb, gridDim.x - p.gb, tl, total, 0);
    }
    // a lone frame's next unit order, by the last shadow-role workgroup once its shadow rays are done:
    // beside phase B's deep chains, off the frame's critical path (in a packing pass it cost 30 us there)
    if (!COUNT && !chain && p.urank && blockIdx.x == gridDim.x - 1) rank_units(p);
}

// Phase B's shadow tasks (which = 1), or phase A's (which = 0: p.split_occ, frame batches).
template <bool COUNT>
__global__ __launch_bounds__(kBlock, RT_OCC_WAVES_PER_EU) void k_occlude(rtk::DevScene s, PcParams p, int which) {
    block_init(s);
    if constexpr (!COUNT && RT_LEAF_QUEUE) {
        // tasks where their phase left them: region r (phase workgroup r's queue) to workgroup r mod G,
        // one region at a time (no packed copy of 4 B in and out per task): A's in frame batches, B's
        // LDS-queue overflow in lone frames (few tasks; no k_pack_b launch on the frame's critical path)
        const bool inplace = which ? p.occ_inplace_b != 0 : p.occ_inplace != 0;
        // (production A's tasks here are always in place: p.occ_inplace with p.split_occ; no g_pref in this
        // kernel, whose 6 waves per SIMD need its LDS)
        if (inplace || !which) occlude_regions(s, p, which, blockIdx.x, gridDim.x);
        else occlude_queue_body(s, p, blockIdx.x, gridDim.x, flat_list(p.sflatB), p.totals[2]);
        // a lone frame without phase B walks A's shadow tasks here (no k_mix): the next frame's unit order
        if (!which && p.urank && blockIdx.x == gridDim.x - 1) rank_units(p);
    } else {
        if (which) occlude_body<COUNT>(s, p, blockIdx.x, gridDim.x, flat_list(p.sflatB), p.totals[2], 1);
        else occlude_body<COUNT>(s, p, blockIdx.x, gridDim.x, shadow_regions_a(p), region_prefix(p.scntA, (unsigned)p.grid), 0);
    }
}

// Output row of slab row lr.  A frame split into out_k interleaved sub-frames
// (rt_api.cpp render_frame) renders sub-frame out_j's stripes; its stripe m is
// stripe m*out_k + out_j of the caller's slab.
__device__ __forceinline__ int out_row(const PcParams& p, int lr) {
    const int m = lr / p.stripe_rows;
    return (m * p.out_k + p.out_j) * p.stripe_rows + (lr - m * p.stripe_rows);
}

// Small scenes (<= kFinishMats materials, <= kFinishLights lights): k_finish
// keeps the materials and lights in LDS (their loads
// then wait on lgkmcnt, not on the prefetched records' vmcnt).
constexpr int kFinishMats = 64, kFinishLights = 4;
__shared__ dl::Material g_fmats[kFinishMats];
__shared__ dl::Light g_flights[kFinishLights];

template <bool LDS>
__device__ __forceinline__ const dl::Material& fin_mat(const rtk::DevScene& s, int i) {
    if (LDS) return g_fmats[i];
    return s.mats[i];
}
template <bool LDS>
__device__ __forceinline__ const dl::Light& fin_light(const rtk::DevScene& s, int i) {
    if (LDS) return g_flights[i];
    return s.lights[i];
}

// Blinn-Phong of one hit (raytracer.cpp:391-425): hit point, ray direction, normal, material words;
// occluded(l): light l's shadow ray found an occluder.  The one shading arithmetic of the chain path
// (k_finish from records, k_fallback inline).
template <bool LDS, class OCC>
__device__ __forceinline__ V shade_core(const rtk::DevScene& s, const V hitp, const V d, const V n_, const float4 mA,
                                        const float4 mD, const float4 mS, OCC&& occluded_fn) {
    V L{0.0f, 0.0f, 0.0f};
    L = add(L, V{mA.x, mA.y, mA.z});                                                  // :394-395
    const V pnt = add(hitp, mul(n_, s.eps));                                           // :397
    // LDS (small scenes): <= kFinishLights lights, a fully unrolled loop and no byte loads
    const int nl = LDS ? kFinishLights : s.nlights;
#pragma unroll 1
    for (int l = 0; l < nl; ++l) {
        if (LDS && l >= s.nlights) break;
        if (occluded_fn(l)) continue;
        const dl::Light& Lt = fin_light<LDS>(s, l);
        const float4 lp = ld4(&Lt.px), li4 = ld4(&Lt.ix);
        const V lpos{lp.x, lp.y, lp.z};
        const float dist = len(sub(lpos, pnt));
        const V ldir = nrm(sub(lpos, pnt));
        const V ldir_real = nrm(sub(lpos, hitp));
        const float cos_t = dot(ldir_real, n_);
        const V E = divs(V{li4.x, li4.y, li4.z}, dist * dist);
        if (cos_t >= s.cos_thr && cos_t <= 1.0f) {
            const V hh = nrm(add(ldir, neg(nrm(d))));
            const float base = smax(0.0f, dot(nrm(n_), hh));
            const float ca = phong_pow(base, mA.w);
            L = add(L, had(mul(V{mS.x, mS.y, mS.z}, ca), E));
        }
        const float cl = smax(0.0f, smin(1.0f, cos_t));
        L = add(L, had(mul(V{mD.x, mD.y, mD.z}, cl), E));
    }
    return L;
}

// The same for record rid from its already-loaded words (hit point a.xyz, ray direction dir): occ bit
// l set = light l occluded (lights >= 32 read their byte directly).
template <bool LDS>
__device__ __forceinline__ V shade_words(const rtk::DevScene& s, const PcParams& p, unsigned rid, const float4 a,
                                         const V n_, const V dir, const float4 mA, const float4 mD,
                                         const float4 mS, uint32_t occ32) {
    return shade_core<LDS>(s, V{a.x, a.y, a.z}, dir, n_, mA, mD, mS, [&](int l) {
        return (LDS || l < 32) ? ((occ32 >> l) & 1u) != 0 : p.occ[(size_t)rid * s.nlights + l] != 0;
    });
}

// Occlusion bytes of record rid.  Up to four lights: the two aligned dwords
// covering them, loaded together and decoded only where the bits are used, so
// the loads stay in flight with the prefetched record (a byte loop waits for
// every outstanding load).  The occlusion array is padded by 8 bytes for the
// second dword.  More lights: decoded from the bytes at use.
struct OccRaw {
    uint32_t w0, w1;
    unsigned off;     // byte offset of the record's first light (owner id of light 0, < 2^31)
};
template <bool SMALL>
__device__ __forceinline__ OccRaw occ_load(const PcParams& p, unsigned rid, int nl) {
    OccRaw o;
    o.off = rid * (unsigned)nl;
    if (SMALL) {
        const uint32_t* wd = reinterpret_cast<const uint32_t*>(p.occ) + (o.off >> 2);
        o.w0 = wd[0];
        // the second dword only when the record's bytes cross into it (never for 1, 2 or 4 lights)
        o.w1 = (o.off & 3u) + (unsigned)nl > 4u ? wd[1] : 0u;
    } else {
        o.w0 = o.w1 = 0;
    }
    return o;
}
template <bool SMALL>
__device__ __forceinline__ uint32_t occ_bits(const PcParams& p, const OccRaw& o, int nl) {
    uint32_t m = 0;
    if (SMALL) {
        const uint64_t v = ((uint64_t)o.w0 | ((uint64_t)o.w1 << 32)) >> ((o.off & 3u) * 8u);
#pragma unroll
        for (int l = 0; l < 4; ++l)
            if (l < nl && ((v >> (8 * l)) & 0xffu)) m |= 1u << l;
    } else {
        for (int l = 0; l < nl && l < 32; ++l) m |= (p.occ[o.off + l] ? 1u : 0u) << l;
    }
    return m;
}

// Shade and fold one sample's recorded levels deepest-first, the next
// (shallower) level's record and occlusion bytes in flight while the current
// one is shaded: c_k = clamp(L_k + c_{k+1} (x) km_k) (raytracer.cpp:436-451).
// Compact phase-A levels (k < ca <= kCompactLevels, PcParams::dbase) get their
// direction words when they come up: level 0's direction is the sample's eye
// ray's, level 1's its reflection at level 0 (the chain's own arithmetic
// on the same values), their materials the surfaces' (surface_mat).
template <bool LDS, bool CMP>
__device__ __forceinline__ V path_shade_fold(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p,
                                             unsigned path) {
    const int info = p.pinfo[path];
    const int nlev = info & 0xff, kind = (info >> 8) & 0xff;
    V c = kind == kEndBg ? V{s.bgx, s.bgy, s.bgz} : V{0.0f, 0.0f, 0.0f};
    if (kind == kEndTail) {                    // levels >= nlev: k_fallback's folded colour
        const float4 t = p.tail[path];
        c = V{t.x, t.y, t.z};
    }
    if (nlev == 0) return c;
    const int nl = s.nlights;
    const int ca = CMP ? min(nlev, p.clevels) : 0;   // (k_finish<.., false>: launches without compact records)
    auto compact_d = [&](int k, const float4 ak) {   // {direction, material} of compact level k (record ak)
        Ray r0;
        slab_sample_ray(p, path, &r0);      // the sample's eye ray, from the slot (nothing held for it)
        V dk = r0.d;
        if (kCompactLevels > 1 && k == 1) {
            const float4 a0 = p.rec[path];
            const V h0{a0.x, a0.y, a0.z};
            dk = reflect_ray(s, h0, surface_normal(s, h0, __float_as_int(a0.w)), dk).d;
        }
        return make_float4(dk.x, dk.y, dk.z, __int_as_float(surface_mat(s, __float_as_int(ak.w))));
    };
    const unsigned cx = nlev > p.la ? p.cid[path] : 0u;   // continued paths: their phase-B records
    unsigned rid = rec_id(p, nlev - 1, path, cx);
    float4 a = p.rec[rid], ds = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (nlev - 1 >= ca) ds = p.recd[rid - p.dbase];
    OccRaw oc = occ_load<LDS>(p, rid, nl);
    for (int k = nlev - 1; k >= 0; --k) {
        const float4 d = k < ca ? compact_d(k, a) : ds;
        const dl::Material& M = fin_mat<LDS>(s, __float_as_int(d.w) - 1);   // before the prefetch (vmcnt order)
        const float4 mA = ld4(&M.kax), mD = ld4(&M.kdx), mS = ld4(&M.ksx), km = ld4(&M.kmx);
        const V n_ = surface_normal(s, V{a.x, a.y, a.z}, __float_as_int(a.w));
        // the next (shallower) record: phase-B ids step down by cb, phase-A ids are (k-1) * cap + path
        const unsigned rn = k - 1 >= p.la ? rid - p.cb : (unsigned)max(k - 1, 0) * (unsigned)p.cap + path;
        const bool stored = !CMP || k - 1 >= ca;   // the next level's record has its direction word
#if RT_FINISH_PREFETCH
        const float4 na = p.rec[rn];
        float4 nd = ds;
        if (stored) nd = p.recd[rn - p.dbase];
        const OccRaw noc = occ_load<LDS>(p, rn, nl);
#endif
        const V L = shade_words<LDS>(s, p, rid, a, n_, V{d.x, d.y, d.z}, mA, mD, mS, occ_bits<LDS>(p, oc, nl));
        if (kind == kEndLast && k == nlev - 1) c = vclamp(L, 0.0f, FLT_MAX);
        else c = vclamp(add(L, had(c, V{km.x, km.y, km.z})), 0.0f, FLT_MAX);
#if RT_FINISH_PREFETCH
        rid = rn; a = na; ds = nd; oc = noc;
#else
        if (k > 0) {
            rid = rn; a = p.rec[rn];
            if (stored) ds = p.recd[rn - p.dbase];
            oc = occ_load<LDS>(p, rn, nl);
        }
#endif
    }
    return c;
}

// One output pixel (rr, ocol) of the chunk: its F x F samples shaded, folded, quantised and averaged.
template <bool LDS, bool CMP>
__device__ __forceinline__ void finish_pixel(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, int rr,
                                             int ocol) {
    const int F = p.aa;
    const int lr = p.chunk_row0 / p.aa + rr;
    if (lr >= p.slab_rows) return;
    int lf = lr;
    const int fr = batch_frame(p, &lf);
    const int stripe = lf / p.stripe_rows;
    const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lf - stripe * p.stripe_rows);
    if (g >= p.height) return;
    uint32_t sr = 0, sg = 0, sb = 0;
    for (int k = 0; k < F; ++k)
        for (int l = 0; l < F; ++l) {
            const V c = path_shade_fold<LDS, CMP>(s, e, p, slab_slot(p.tiles_x, ocol * F + l, rr * F + k));
            sr += quantise(c.x); sg += quantise(c.y); sb += quantise(c.z);
        }
    const uint32_t ff = (uint32_t)(F * F);
    uint8_t* o = (p.nframes > 1 ? p.fouts[fr] : p.out) + ((size_t)out_row(p, lf) * p.width + ocol) * 3;
    o[0] = (uint8_t)(sr / ff); o[1] = (uint8_t)(sg / ff); o[2] = (uint8_t)(sb / ff);
}

// Output pixel (rr, ocol) of the chunk: does any of its samples continue in phase B (pinfo's kPathCont)?
__device__ __forceinline__ bool pixel_cont(const PcParams& p, int rr, int ocol) {
    bool cont = false;
    for (int k = 0; k < p.aa; ++k)
        for (int l = 0; l < p.aa; ++l)
            cont |= (p.pinfo[slab_slot(p.tiles_x, ocol * p.aa + l, rr * p.aa + k)] & kPathCont) != 0;
    return cont;
}

// p.fin_cont (chain path): the pixels of the paths continued in phase B first (the packed continuations,
// cflat: k_pack_a's, or a lone frame's k_mix / k_fallback stored them at their grab; each pixel once, by the
// lane holding its first continued sample), so their long folds
// overlap the rest; then every pixel without a continued sample (pinfo's kPathCont bit).
template <bool LDS, bool CMP>
__device__ __forceinline__ void finish_pixels(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p) {
    const int F = p.aa;
    const unsigned gtid = blockIdx.x * kBlock + threadIdx.x, gstride = gridDim.x * kBlock;
    if (p.fin_cont) {
        const unsigned n = p.totals[1];
        for (unsigned j = gtid; j < n; j += gstride) {
            const unsigned path = (p.cflat[j] & ~kFbEye) % (unsigned)p.cap;
            const unsigned tile = path >> 6, lane = path & 63u;
            const int ix = (int)(tile % (unsigned)p.tiles_x) * 8 + (int)(lane & 7u);
            const int iyc = (int)(tile / (unsigned)p.tiles_x) * 8 + (int)(lane >> 3);
            const int ocol = ix / F, rr = iyc / F;
            unsigned first = path;
            for (int k = F - 1; k >= 0; --k)
                for (int l = F - 1; l >= 0; --l) {
                    const unsigned sl = slab_slot(p.tiles_x, ocol * F + l, rr * F + k);
                    if (p.pinfo[sl] & kPathCont) first = sl;
                }
            if (first == path) finish_pixel<LDS, CMP>(s, e, p, rr, ocol);
        }
    }
    if (F == 1) {   // one sample a pixel: a wave per 8x8 tile, the records' own order (C3 -0.5 to -1 %)
        for (unsigned q = gtid; q < (unsigned)p.n0; q += gstride) {
            const unsigned tile = q >> 6, lane = q & 63u;
            const unsigned ty = tile / (unsigned)p.tiles_x, tx = tile - ty * (unsigned)p.tiles_x;
            const int ocol = (int)(tx * 8u + (lane & 7u)), rr = (int)(ty * 8u + (lane >> 3));
            if (ocol >= p.width || rr >= p.chunk_rows) continue;
            if (p.fin_cont && (p.pinfo[q] & kPathCont)) continue;
            int lf = p.chunk_row0 + rr;                         // finish_pixel at F = 1: sample q is the pixel
            if (lf >= p.slab_rows) continue;
            const int fr = batch_frame(p, &lf);
            const int stripe = lf / p.stripe_rows;
            if ((stripe * p.nranks + p.rank) * p.stripe_rows + (lf - stripe * p.stripe_rows) >= p.height) continue;
            const V c = path_shade_fold<LDS, CMP>(s, e, p, q);
            uint8_t* o = (p.nframes > 1 ? p.fouts[fr] : p.out) + ((size_t)out_row(p, lf) * p.width + ocol) * 3;
            o[0] = (uint8_t)quantise(c.x); o[1] = (uint8_t)quantise(c.y); o[2] = (uint8_t)quantise(c.z);
        }
        return;
    }
    const int npix = (p.chunk_rows / p.aa) * p.width;
    for (int q = (int)gtid; q < npix; q += (int)gstride) {
        const int rr = q / p.width, ocol = q - rr * p.width;
        if (p.fin_cont && pixel_cont(p, rr, ocol)) continue;
        finish_pixel<LDS, CMP>(s, e, p, rr, ocol);
    }
}

// k_finish: k_shade + k_compose in one pass, one lane per output pixel, with
// the scene's materials and lights in LDS (host checks they fit);
// k_finish_any: the same for larger scenes, tables read from global memory.
template <bool CMP>
__global__ __launch_bounds__(kBlock, CMP ? RT_FINISH_CMP_WAVES : RT_FINISH_WAVES) void k_finish(rtk::DevScene s,
                                                                                                 rtk::Eye e, PcParams p) {
    float4* dm = reinterpret_cast<float4*>(g_fmats);
    const float4* sm = reinterpret_cast<const float4*>(s.mats);
    for (int i = threadIdx.x; i < s.nmats * 4; i += kBlock) dm[i] = sm[i];
    float4* dl_ = reinterpret_cast<float4*>(g_flights);
    const float4* sl = reinterpret_cast<const float4*>(s.lights);
    for (int i = threadIdx.x; i < s.nlights * 2; i += kBlock) dl_[i] = sl[i];
    __syncthreads();
    finish_pixels<true, CMP>(s, e, p);
}
template <bool CMP>
__global__ __launch_bounds__(kBlock, RT_FINISH_ANY_WAVES) void k_finish_any(rtk::DevScene s, rtk::Eye e, PcParams p) {
    finish_pixels<false, CMP>(s, e, p);
}

// ---------------------------------------------------------------------------
// k_fallback: what the timed walks leave (rare): rays the wide trees' fused
// slab test does not take (defer_closest / defer_any: NaN, or a direction
// component of 0) and continuations beyond the phase-B record capacity.  Each
// lane runs the general walks (wide or binary trees, the reference's NaN
// semantics) one item at a time:
//   * a chain entry: the path from the deferred ray to its end, closest hit,
//     shadow rays inline, shading (shade_core) and the deepest-first fold
//     (raytracer.cpp:385-452) -> tail[path], pinfo = nlev | kEndTail;
//   * a shadow task: its any-hit walk -> occ[owner];
//   * after a full shadow queue: every occlusion byte marked kOccDeferred.
// Launched after the shadow kernels and before k_finish; with nothing to do it
// exits at once.
// ---------------------------------------------------------------------------
constexpr int kFbMaxLevels = 66;      // max_recursion_depth <= 64 (rt_scene_set_max_depth) + 1

__device__ __forceinline__ bool fallback_any(const rtk::DevScene& s, const Ray& r, float tlim, WalkStack& stk,
                                             Work& w) {
    Walk wk;
    if (!walk_begin<false>(s, r, wk, w, true)) return false;
    while (true) {
        const int res = occl_step<false, FetchTop>(s, r, tlim, stk, wk, w);
        if (res) return res == 2;
        if (walk_runaway(s, wk)) return false;
    }
}

__device__ void fallback_chain(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, unsigned entry,
                               WalkStack& stk, Work& w, bool cont = false) {   // cont: a continuation (cont_entry)
    const unsigned cap = (unsigned)p.cap;
    unsigned path;
    int k;
    Ray r;
    if (entry & kFbEye) {                          // a deferred eye ray
        path = entry & ~kFbEye;
        k = 0;
        if (!slab_sample_ray(p, path, &r)) return;
    } else {                                       // the reflection of record `entry`
        const size_t aspace = (size_t)p.la * cap;
        int kprev;
        if (entry < aspace) {
            kprev = (int)(entry / cap);
            path = entry % cap;
        } else {
            const size_t q = entry - aspace;
            kprev = p.la + (int)(q / p.cb);
            path = cont_entry(p, (unsigned)(q % p.cb)) % cap;   // (k_fallback: g_pref holds the continuations)
        }
        k = kprev + 1;
        r = reflect_from_record(s, p, entry, path);
    }
    const int k0 = k;
    V Ls[kFbMaxLevels], Km[kFbMaxLevels];          // the mirror levels' shading and km, k0 onward
    int n = 0;
    V c{0.0f, 0.0f, 0.0f};                         // the deepest level's value (before the fold)
    while (true) {
        if (k > s.max_depth) break;                // beyond MaxRecursionDepth: 0 (:387-389)
        Walk wk;
        if (walk_begin<false>(s, r, wk, w)) {
            while (!closest_step<false, FetchTop, WalkStack>(s, r, stk, wk, w) && !walk_runaway(s, wk)) {
            }
        }
        const HitRec h = wk.best;
        if (p.dbg_t && k == 0) {                   // diagnostics: a deferred eye ray's hit (PcParams::dbg_t)
            int row, col, mat = 0;
            if (h.prim >= 0) {
                V nn;
                int code;
                hit_surface(s, r, h, &nn, &mat, &code);
            }
            if (slab_sample_pixel(p, path, &row, &col)) {
                p.dbg_t[(size_t)row * p.wi + col] = h.t;
                p.dbg_m[(size_t)row * p.wi + col] = mat;
            }
        }
        if (h.prim < 0) {                          // miss: background at depth 0, else 0 (:442-449)
            if (k == 0) c = V{s.bgx, s.bgy, s.bgz};
            break;
        }
        V nn;
        int mat, code;
        hit_surface(s, r, h, &nn, &mat, &code);
        const V hitp = add(r.o, mul(r.d, h.t));
        const dl::Material& M = s.mats[mat - 1];
        const float4 mA = ld4(&M.kax), mD = ld4(&M.kdx), mS = ld4(&M.ksx), km = ld4(&M.kmx);
        const V L = shade_core<false>(s, hitp, r.d, nn, mA, mD, mS, [&](int l) {
            if (s.cull_shadows && !light_needed(s, hitp, nn, l)) return true;   // the same sum (light_needed)
            float tlim;
            const Ray sr = shadow_ray(s, hitp, nn, l, &tlim);
            return fallback_any(s, sr, tlim, stk, w);
        });
        if (!M.is_mirror) {                        // the last level: its own clamp (:451)
            c = vclamp(L, 0.0f, FLT_MAX);
            break;
        }
        Ls[n] = L;
        Km[n] = V{km.x, km.y, km.z};
        ++n;
        if (k >= s.max_depth || n >= kFbMaxLevels) break;   // the child beyond the depth returns 0
        r = reflect_ray(s, hitp, nn, r.d);
        ++k;
    }
    for (int i = n - 1; i >= 0; --i) c = vclamp(add(Ls[i], had(c, Km[i])), 0.0f, FLT_MAX);   // :436-451
    p.tail[path] = make_float4(c.x, c.y, c.z, 0.0f);
    p.pinfo[path] = k0 | (kEndTail << 8) | (k0 >= p.la || cont ? kPathCont : 0);
}

__global__ __launch_bounds__(kBlock) void k_fallback(rtk::DevScene s, rtk::Eye e, PcParams p) {
    block_init(s);
    const unsigned ncont = region_prefix(p.ccnt, (unsigned)p.grid);   // the continuation list (cont_entry)
    WalkStack stk;
    Work w;
    const unsigned gt = blockIdx.x * kBlock + threadIdx.x, gs = gridDim.x * kBlock;
    const unsigned nfc = min(p.totals[4], p.fbc_cap);
    const unsigned novf = ncont > p.cb ? ncont - p.cb : 0u;
    if (gt == 0 && p.counters) {                   // what this launch left to k_fallback (rt_counters_read_raw)
        atomicAdd(&p.counters[kCntFbLaunches], 1ull);
        atomicAdd(&p.counters[kCntFbConts], (unsigned long long)ncont);
        atomicAdd(&p.counters[kCntFbContOvf], (unsigned long long)novf);
        atomicAdd(&p.counters[kCntFbChains], (unsigned long long)p.totals[4]);
        atomicAdd(&p.counters[kCntFbShadows], (unsigned long long)p.totals[5]);
        if (p.totals[6]) atomicAdd(&p.counters[kCntFbOvfScans], 1ull);
        if (p.clevels) atomicAdd(&p.counters[kCntCompactLaunches], 1ull);
    }
    for (unsigned i = gt; i < nfc + novf; i += gs) {
        unsigned entry;
        if (i < nfc) {
            entry = p.fbc[i];
        } else {                                   // a continuation beyond cb (packed for k_finish: a lone frame)
            entry = cont_entry(p, p.cb + (i - nfc));
            p.cflat[p.cb + (i - nfc)] = entry;
        }
        fallback_chain(s, e, p, entry, stk, w, i >= nfc);
    }
    const unsigned nfs = min(p.totals[5], p.fbs_cap);
    for (unsigned i = gt; i < nfs; i += gs) {
        const unsigned owner = p.fbs[i];
        float tlim;
        const Ray r = shadow_from_record(s, p, owner, &tlim);
        p.occ[owner] = fallback_any(s, r, tlim, stk, w) ? 1 : 0;
    }
    if (p.totals[6]) {                             // the shadow queue overflowed: the marked bytes
        const size_t nocc = ((size_t)p.la * (unsigned)p.cap + (size_t)(p.levels - p.la) * p.cb) * s.nlights;
        for (size_t i = gt; i < nocc; i += gs)
            if (p.occ[i] == kOccDeferred) {
                float tlim;
                const Ray r = shadow_from_record(s, p, (unsigned)i, &tlim);
                p.occ[i] = fallback_any(s, r, tlim, stk, w) ? 1 : 0;
            }
    }
}

// Diagnostics (rt_walk_timing): wave 0 of one workgroup walks ray i with
// lanes [0, lanes) (the same ray in every lane), reps times; lane 0 records
// the last rep's shader cycles (s_memtime), the steps and the winner.  mode 0:
// the production closest-hit walk (the reference-order wide tree), 1: the binary
// reference tree.  Measures the dependent-step latency of one walk.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_walk_timing(rtk::DevScene s, const float* rays, int n, int lanes, int reps,
                                                        unsigned long long* out) {
    constexpr int mode = MODE;
    block_init(s);
    if (threadIdx.x >= 64) return;
    WalkStack stk;
    Work w;
    for (int i = 0; i < n; ++i) {
        const Ray r = make_ray(V{rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]},
                               V{rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]});
        unsigned long long t0 = 0, t1 = 0, first = 0;
        int steps = 0;
        HitRec h{-1.0f, -1};
#pragma unroll 1
        for (int rep = 0; rep < reps; ++rep) {
            t0 = __builtin_amdgcn_s_memtime();
            steps = 0;
            if (mode == 3) {                     // memory only: dependent wide-node fetches (first child) from the root
                if (threadIdx.x == 0 && s.swnodes) {
                    int cur = s.swroot;
#pragma unroll 1
                    for (int hop = 0; hop < 64; ++hop) {
                        if (cur < 0) cur = s.swroot;
                        if (cur < 0) break;
                        const float4* Q = reinterpret_cast<const float4*>(&s.swnodes[cur]);
                        const float4 q5 = Q[5];
                        cur = __float_as_int(q5.z) ^ (int)(rays[0] * 0.0f);
                        ++steps;
                    }
                    h = HitRec{0.0f, cur};
                }
            } else if (mode == 4) {              // memory only: the same with all seven loads of a node
                if (threadIdx.x == 0 && s.swnodes) {
                    int cur = s.swroot;
#pragma unroll 1
                    for (int hop = 0; hop < 64; ++hop) {
                        if (cur < 0) cur = s.swroot;
                        if (cur < 0) break;
                        WideNode nd;
                        wide_load(s.swnodes, cur, nd);
                        int pick = 0;
#pragma unroll
                        for (int j = 0; j < 7; ++j) pick ^= __float_as_int(nd.q[j].x);
                        cur = wide_code(nd, 0) + (pick & 0);
                        ++steps;
                    }
                    h = HitRec{0.0f, cur};
                }
            } else if ((int)threadIdx.x < lanes) {
                Walk wk;
                bool go = mode == 0 ? walk_begin<false>(s, r, wk, w) : walk_begin<true>(s, r, wk, w);
#pragma unroll 1
                while (go) {
                    ++steps;
                    const bool done = mode == 0 ? closest_step<false, FetchTop, WalkStack>(s, r, stk, wk, w)
                                                : closest_step<true, FetchTop, WalkStack>(s, r, stk, wk, w);
                    if (done) break;
                }
                h = wk.best;
            }
            t1 = __builtin_amdgcn_s_memtime();
            if (rep == 0) first = t1 - t0;
        }
        if (threadIdx.x == 0) {
            out[4 * i] = t1 - t0;
            out[4 * i + 1] = (unsigned long long)steps;
            out[4 * i + 2] = (unsigned long long)(long long)h.prim;
            out[4 * i + 3] = first;
        }
    }
}

}  // namespace

// A kernel launch; with a KTimer, through hipExtLaunchKernel with the timer's next start / stop events.
#define RT_LAUNCH(KT, KIND, KERN, GRID, BLK, ST, ...)                                                       \
    do {                                                                                                 \
        hipEvent_t e0_ = nullptr, e1_ = nullptr;                                                         \
        if (KT) (KT)->take(KIND, &e0_, &e1_);                                                            \
        if (e0_) hipExtLaunchKernelGGL(KERN, GRID, BLK, 0, ST, e0_, e1_, 0, __VA_ARGS__);                \
        else hipLaunchKernelGGL(KERN, GRID, BLK, 0, ST, __VA_ARGS__);                                    \
    } while (0)

// Shading + fold + SSAA: k_finish (a lane per pixel; materials and lights in LDS), or k_finish_any for
// larger scenes.
void launch_finish(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, hipStream_t st, KTimer* kt) {
    const int npix = (p.chunk_rows / p.aa) * p.width;
    const dim3 pgrid(std::max(1, std::min((npix + kBlock - 1) / kBlock, p.fin_grid > 0 ? p.fin_grid : INT32_MAX)));
    const dim3 blk(kBlock);
    if (s.nmats <= kFinishMats && s.nlights <= kFinishLights) {
        if (p.clevels) RT_LAUNCH(kt, kKFinish, (k_finish<true>), pgrid, blk, st, s, e, p);
        else RT_LAUNCH(kt, kKFinish, (k_finish<false>), pgrid, blk, st, s, e, p);
    } else {
        if (p.clevels) RT_LAUNCH(kt, kKFinish, (k_finish_any<true>), pgrid, blk, st, s, e, p);
        else RT_LAUNCH(kt, kKFinish, (k_finish_any<false>), pgrid, blk, st, s, e, p);
    }
}

hipError_t chain_occupancy(int* chain_blocks_per_cu, int* mix_blocks_per_cu, int* occlude_blocks_per_cu) {
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(chain_blocks_per_cu, k_chain<false>, kBlock, 0);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(mix_blocks_per_cu, k_mix<false, true, true>, kBlock, 0);
    if (e == hipSuccess)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occlude_blocks_per_cu, k_occlude<false>, kBlock, 0);
    return e;
}

hipError_t launch_walk_timing(const rtk::DevScene& s, const float* rays, int n, int lanes, int reps, int mode,
                              unsigned long long* out, hipStream_t st) {
    if (mode == 0) hipLaunchKernelGGL(k_walk_timing<0>, dim3(1), dim3(kBlock), 0, st, s, rays, n, lanes, reps, out);
    else if (mode == 1) hipLaunchKernelGGL(k_walk_timing<1>, dim3(1), dim3(kBlock), 0, st, s, rays, n, lanes, reps, out);
    else if (mode == 3) hipLaunchKernelGGL(k_walk_timing<3>, dim3(1), dim3(kBlock), 0, st, s, rays, n, lanes, reps, out);
    else hipLaunchKernelGGL(k_walk_timing<4>, dim3(1), dim3(kBlock), 0, st, s, rays, n, lanes, reps, out);
    return hipGetLastError();
}

// Diagnostics (rt_phong_pow): the specular power term exactly as the shading
// kernels evaluate it (phong_pow: integer fast path, double-double fallback).
__global__ __launch_bounds__(kBlock) void k_phong_pow(const float* base, const float* expo, float* out, int n) {
    const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (i < n) out[i] = phong_pow(base[i], expo[i]);
}

hipError_t launch_phong_pow(const float* base, const float* expo, float* out, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_phong_pow, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, base, expo, out, n);
    return hipGetLastError();
}

// Diagnostics (rt_cramer_div): the triangle test's three quotients exactly as tri_hit evaluates
// them (cramer_div3: one shared reciprocal, IEEE divisions for the lanes outside its range).
__global__ __launch_bounds__(kBlock) void k_cramer_div(const float* den, const float* num, float* out, int n) {
    const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
    if (i < n) rtd::cramer_div3(den[i], num[3 * i], num[3 * i + 1], num[3 * i + 2], out[3 * i], out[3 * i + 1], out[3 * i + 2]);
}

hipError_t launch_cramer_div(const float* den, const float* num, float* out, int n, hipStream_t st) {
    hipLaunchKernelGGL(k_cramer_div, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, den, num, out, n);
    return hipGetLastError();
}

// Diagnostics (rt_udiv): the walkers' uniform-divisor division (UDiv), one divisor per workgroup
// (it must be wave-uniform): q[j * nv + i] = v[i] / d[j].
__global__ __launch_bounds__(kBlock) void k_udiv(const unsigned* v, int nv, const unsigned* d, unsigned* q) {
    const UDiv u(d[blockIdx.x]);
    for (int i = threadIdx.x; i < nv; i += kBlock) q[(size_t)blockIdx.x * nv + i] = u.div(v[i]);
}

hipError_t launch_udiv(const unsigned* v, int nv, const unsigned* d, int nd, unsigned* q, hipStream_t st) {
    hipLaunchKernelGGL(k_udiv, dim3(nd), dim3(kBlock), 0, st, v, nv, d, q);
    return hipGetLastError();
}

// Diagnostics (RT_STEP_STATS builds): read (and optionally clear) g_step_stat.
extern "C" int rt_debug_step_stats(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_step_stat), sizeof(g_step_stat)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_step_stat), z, sizeof(z)) != hipSuccess) return -1;
    }
    return RT_STEP_STATS;
}

unsigned chain_block_units(int n0, int grid) {
    const unsigned units = ((unsigned)n0 + 255u) / 256u;
    return (units + (unsigned)grid - 1u) / (unsigned)grid;
}

unsigned chain_block_scap(int n0, int grid, int levels, int nlights) {
    return chain_block_units(n0, grid) * 256u * (unsigned)levels * (unsigned)nlights;
}

hipError_t launch_chain_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, bool count,
                              hipStream_t st, KTimer* kt) {
    const dim3 blk(kBlock);
    const bool phase_b = p.kinline < s.max_depth;     // any continuation possible
    {   // the task counts (k_mix stores the continuations'), the dynamic unit counter, k_fallback's counts
        const hipError_t me = hipMemsetAsync(p.totals, 0, kTotalsWords * sizeof(unsigned), st);
        if (me != hipSuccess) return me;
    }
    if (count) RT_LAUNCH(kt, kKChain, k_chain<true>, dim3(p.grid), blk, st, s, e, p);
    else if (p.dbg_t) RT_LAUNCH(kt, kKChain, (k_chain<false, true>), dim3(p.grid), blk, st, s, e, p);
    else RT_LAUNCH(kt, kKChain, k_chain<false>, dim3(p.grid), blk, st, s, e, p);
    // phase A's lists packed, except a whole lone frame's: its k_mix reads them in their regions (region_prefix)
    if (!p.rlists) RT_LAUNCH(kt, kKPackA, k_pack_a, dim3(p.grid), blk, st, p);
    PcParams q = p;
    if (!phase_b) q.gb = 0;
    // p.split_occ (frame batches): k_mix only walks the chains, A's shadow tasks go to k_occlude (5 waves
    // per SIMD; in place, p.occ_inplace); otherwise k_mix's other
    // workgroups walk them beside the chains.  Without phase B (depth 0): no k_mix at all, A's shadow tasks
    // in k_occlude, a lone frame's too
    const bool split = p.split_occ != 0;
    // a lone frame without phase B (depth 0): A's shadow tasks in place by the 6-wave k_occlude instead of
    // k_mix's 4-wave shadow role (C2 one frame 0.146 -> 0.140 ms, profiles/r06_d0_ab.jsonl)
    const bool occ_a = split || (!phase_b && !count);
    const int mgrid = occ_a ? (split ? q.gb : 0) : q.gb + p.ogrid;
    // frame batches (split): phase B's shadow tasks all through k_pack_b + k_occlude (no LDS queue)
    if (mgrid == 0) {
    } else if (count) {
        if (split) RT_LAUNCH(kt, kKMix, (k_mix<true, false>), dim3(mgrid), blk, st, s, e, q);
        else if (p.rlists) RT_LAUNCH(kt, kKMix, (k_mix<true, true, true>), dim3(mgrid), blk, st, s, e, q);
        else RT_LAUNCH(kt, kKMix, (k_mix<true, true>), dim3(mgrid), blk, st, s, e, q);
    } else {
        if (split) RT_LAUNCH(kt, kKMix, (k_mix<false, false>), dim3(mgrid), blk, st, s, e, q);
        else if (p.rlists) RT_LAUNCH(kt, kKMix, (k_mix<false, true, true>), dim3(mgrid), blk, st, s, e, q);
        else RT_LAUNCH(kt, kKMix, (k_mix<false, true>), dim3(mgrid), blk, st, s, e, q);
    }
    if (occ_a) {
        if (count) RT_LAUNCH(kt, kKOccA, k_occlude<true>, dim3(p.occ_grid), blk, st, s, p, 0);
        else RT_LAUNCH(kt, kKOccA, k_occlude<false>, dim3(p.occ_grid), blk, st, s, p, 0);
    }
    if (phase_b) {
        if (count || !p.occ_inplace_b) RT_LAUNCH(kt, kKPackB, k_pack_b, dim3(p.gb), blk, st, p);
        const int og = split ? p.occ_grid : p.ogrid;
        if (count) RT_LAUNCH(kt, kKOccB, k_occlude<true>, dim3(og), blk, st, s, p, 1);
        else RT_LAUNCH(kt, kKOccB, k_occlude<false>, dim3(og), blk, st, s, p, 1);
    }
    RT_LAUNCH(kt, kKFallback, k_fallback, dim3(p.fb_grid), blk, st, s, e, p);
    // continued pixels first only where they are few and deep (one sample per pixel): with 16 samples
    // a pixel (C5: 130 vs 106 ms) and without phase B (C2: +5 %) the extra pinfo reads cost more
    PcParams f = p;
    f.fin_cont = phase_b && p.aa == 1;
    launch_finish(s, e, f, st, kt);
    return hipGetLastError();
}

}  // namespace rtc
