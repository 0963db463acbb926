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

#include "pathchain.hpp"
#include "traverse2.hpp"
#include "wave_util.hpp"

using namespace rtd;

namespace rtc {

namespace {

constexpr int kBlock = 256;
#ifndef RT_WAVES_PER_EU
#define RT_WAVES_PER_EU 1
#endif
constexpr int kLdsStack = 8;     // stack entries kept in LDS (deeper ones in private memory)

enum LaneState : int { kIdle = 0, kTrav = 1, kDone = 2 };

// LDS, named directly so every access is a ds_read/ds_write (a generic
// pointer to them would compile to flat loads that wait on vmcnt + lgkmcnt).
__shared__ float4 g_top[4 * dl::kTopPairs];   // top BVH pairs, 16 KiB
__shared__ int2 g_stk[kLdsStack * kBlock];     // first stack entries, [entry][thread], 16 KiB
__shared__ unsigned g_head;                    // block-local work queue head
__shared__ unsigned g_scnt;                    // block-local shadow-ray count (hit lanes)
__shared__ unsigned g_pref[kMaxChainGrid + 1]; // k_occlude: shadow-queue region prefix

struct FetchTop {
    __device__ static __forceinline__ void pair(const rtk::DevScene& s, int p, float4& l0, float4& l1, float4& r0,
                                                float4& r1) {
        if (p < s.top_pairs) {
            l0 = g_top[4 * p]; l1 = g_top[4 * p + 1]; r0 = g_top[4 * p + 2]; r1 = g_top[4 * p + 3];
        } else {
            FetchGlobal::pair(s, p, l0, l1, r0, r1);
        }
    }
};

struct StackTwoTier {        // entries [0, kLdsStack) in LDS, deeper ones private
    int2 deep[dl::kMaxStack - kLdsStack];
    __device__ __forceinline__ void put(int i, int2 v) {
        if (i < kLdsStack) g_stk[i * kBlock + threadIdx.x] = v;
        else deep[i - kLdsStack] = v;
    }
    __device__ __forceinline__ int2 at(int i) const {
        if (i < kLdsStack) return g_stk[i * kBlock + threadIdx.x];
        return deep[i - kLdsStack];
    }
};

template <bool PRIV>
struct StackSel {
    using type = StackTwoTier;
};
template <>
struct StackSel<true> {
    using type = StackPriv;
};

__device__ __forceinline__ void block_init(const rtk::DevScene& s) {
    if (threadIdx.x == 0) {
        g_head = 0;
        g_scnt = 0;
    }
    const float4* src = reinterpret_cast<const float4*>(s.pairs);
    for (int i = threadIdx.x; i < 4 * s.top_pairs; i += kBlock) g_top[i] = src[i];
    __syncthreads();
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

typedef float nt4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float4* p, float4 v) {
    const nt4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<nt4*>(p));
}
__device__ __forceinline__ float4 ld_nt(const float4* p) {
    const nt4 x = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}

// Block b's samples: units b, b+G, b+2G, ... of 256 consecutive slots.
__device__ __forceinline__ unsigned block_samples(unsigned n0, unsigned G) {
    const unsigned units = (n0 + 255u) / 256u;
    if (blockIdx.x >= units) return 0;
    const unsigned mine = (units - 1u - blockIdx.x) / G + 1u;
    const unsigned last_unit = blockIdx.x + (mine - 1u) * G;
    return (mine - 1u) * 256u + min(256u, n0 - last_unit * 256u);
}
// Within a full unit, `spread` > 1 interleaves its 4 tiles over consecutive
// v (a wave takes 64/spread-sample strips of `spread` tiles), so one heavy
// 8x8 tile is shared by several waves instead of serialising one.
__device__ __forceinline__ unsigned block_sample(unsigned v, unsigned G, unsigned n0, unsigned spread) {
    const unsigned unit = blockIdx.x + (v >> 8) * G;
    unsigned u = v & 255u;
    if (spread > 1u && (unit + 1u) * 256u <= n0) {
        const unsigned grp = u / (64u * spread), j = u % (64u * spread);
        u = (grp * spread + j % spread) * 64u + j / spread;
    }
    return unit * 256u + u;
}

// ---------------------------------------------------------------------------
// k_chain: closest-hit chain of every sample (raytracer.cpp:385-439 minus the
// shading): record each hit, queue its shadow rays, follow mirrors.
// ---------------------------------------------------------------------------
template <bool COUNT, bool PRIV>
__global__ __launch_bounds__(kBlock, RT_WAVES_PER_EU) void k_chain(rtk::DevScene s, rtk::Eye e, PcParams p) {
    block_init(s);
    typename StackSel<PRIV>::type stk;
    Work w;
    uint32_t nprim = 0, nrefl = 0;
    const unsigned G = gridDim.x;
    const unsigned nb = block_samples((unsigned)p.n0, G);
    const int nl = s.nlights;
    float4* sray = p.sray + 2 * (size_t)blockIdx.x * p.block_scap;
    int st = kIdle;
    bool exhausted = nb == 0;
    unsigned path = 0;
    int k = 0;
    Ray r;
    Walk wk;
    unsigned t_grab = 0;
    while (true) {
        // (1) epilogue of finished walks: record, queue shadow rays, reflect
        if (st == kDone) {
            const HitRec h = wk.best;
            const bool hit = h.prim >= 0;
            V nn{0.0f, 0.0f, 0.0f}, hitp{0.0f, 0.0f, 0.0f}, pnt{0.0f, 0.0f, 0.0f};
            int mat = 0;
            if (hit) {
                hit_surface(s, r, h, &nn, &mat);
                hitp = add(r.o, mul(r.d, h.t));
                float4* rc = p.rec + ((size_t)k * p.cap + path) * 3;
                st_nt(rc + 0, make_float4(hitp.x, hitp.y, hitp.z, __int_as_float(mat)));
                st_nt(rc + 1, make_float4(nn.x, nn.y, nn.z, h.t));
                st_nt(rc + 2, make_float4(r.d.x, r.d.y, r.d.z, 0.0f));
                pnt = add(hitp, mul(nn, s.eps));                                 // :397
            }
            // one shadow ray per light (:399-404), light-major within the wave
            const unsigned long long hm = __ballot(hit);
            if (hit) {
                const unsigned cnt = (unsigned)__popcll(hm);
                const unsigned base = wave_grab_lds(&g_scnt, hm);
                const unsigned rank = lane_rank(hm);
                for (int l = 0; l < nl; ++l) {
                    const float4 lp = ld4(&s.lights[l].px);
                    const V lpos{lp.x, lp.y, lp.z};
                    const float dist = len(sub(lpos, pnt));
                    const V ldir = nrm(sub(lpos, pnt));
                    const int owner = (int)(((size_t)k * p.cap + path) * nl + l);
                    const unsigned slot = base * nl + l * cnt + rank;
                    st_nt(sray + 2 * slot, make_float4(pnt.x, pnt.y, pnt.z, __int_as_float(owner)));
                    st_nt(sray + 2 * slot + 1, make_float4(ldir.x, ldir.y, ldir.z, dist));
                }
            }
            if (!hit) {                                                          // :442-449
                p.pinfo[path] = k | ((k == 0 ? kEndBg : kEndZero) << 8);
                st = kIdle;
                if (p.trace) { p.trace[2 * path] = t_grab; p.trace[2 * path + 1] = (unsigned)wall_clock64(); }
            } else if (!s.mats[mat - 1].is_mirror) {
                p.pinfo[path] = (k + 1) | (kEndLast << 8);
                st = kIdle;
                if (p.trace) { p.trace[2 * path] = t_grab; p.trace[2 * path + 1] = (unsigned)wall_clock64(); }
            } else if (k >= s.max_depth) {        // child beyond MaxRecursionDepth: 0 (:387-389)
                p.pinfo[path] = (k + 1) | (kEndZero << 8);
                st = kIdle;
                if (p.trace) { p.trace[2 * path] = t_grab; p.trace[2 * path + 1] = (unsigned)wall_clock64(); }
            } else {
                const V d2 = nrm(r.d);                                         // :431-435
                const V n2 = nrm(nn);
                const float rcos = dot(neg(d2), n2);
                r = make_ray(pnt, add(d2, mul(mul(n2, 2.0f), rcos)));
                ++k;
                nrefl++;
                st = walk_begin<COUNT>(s, r, wk, w) ? kTrav : kDone;
            }
        }
        // (2) refill idle lanes with this block's next samples
        if (!exhausted) {
            const unsigned long long idle = __ballot(st == kIdle);
            if (idle) {
                const unsigned base = wave_grab_lds(&g_head, idle);
                if (base + (unsigned)__popcll(idle) >= nb) exhausted = true;
                if (st == kIdle) {
                    const unsigned v = base + lane_rank(idle);
                    if (v < nb) {
                        const unsigned idx = block_sample(v, G, (unsigned)p.n0, (unsigned)p.spread);
                        if (slab_sample_ray(e, p, idx, &r)) {
                            path = idx;
                            k = 0;
                            if (p.trace) t_grab = (unsigned)wall_clock64();
                            nprim++;
                            if (s.max_depth < 0) p.pinfo[path] = 0 | (kEndZero << 8);   // depth 0 > max: black
                            else st = walk_begin<COUNT>(s, r, wk, w) ? kTrav : kDone;
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
        if (s.prio) wave_priority(st == kTrav ? k : 0);
        const int thresh = exhausted ? 0 : p.refill;
        while (__popcll(__ballot(st == kTrav)) > thresh && __popcll(__ballot(st == kDone)) < p.service) {
            if (st == kTrav && closest_step<COUNT, FetchTop>(s, r, stk, wk, w)) st = kDone;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) p.bcount[blockIdx.x] = g_scnt * (unsigned)nl;
    if (COUNT) {
        wave_add_counter(&p.counters[0], nprim);
        wave_add_counter(&p.counters[2], nrefl);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// k_scan: exclusive prefix of the per-block shadow counts (one workgroup).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan(PcParams p) {
    __shared__ unsigned part[1024];
    const int G = p.grid;
    const int per = (G + 1023) / 1024;
    const int b0 = threadIdx.x * per;
    unsigned sum = 0;
    for (int i = b0; i < min(G, b0 + per); ++i) sum += p.bcount[i];
    part[threadIdx.x] = sum;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {            // Hillis-Steele inclusive scan
        const unsigned v = threadIdx.x >= (unsigned)off ? part[threadIdx.x - off] : 0u;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    unsigned run = threadIdx.x == 0 ? 0u : part[threadIdx.x - 1];
    for (int i = b0; i < min(G, b0 + per); ++i) {
        p.bprefix[i] = run;
        run += p.bcount[i];
    }
    if (threadIdx.x == 1023) p.bprefix[G] = part[1023];
}

// ---------------------------------------------------------------------------
// k_occlude: any-hit of every queued shadow ray (raytracer.cpp:227-280).
// The rays of all k_chain regions form one index space (prefix sums); each
// workgroup takes an equal slice of it, so a region full of mirror bounces
// is spread over the whole grid.
// ---------------------------------------------------------------------------
template <bool COUNT, bool PRIV>
__global__ __launch_bounds__(kBlock, RT_WAVES_PER_EU) void k_occlude(rtk::DevScene s, PcParams p) {
    const int GC = p.grid;
    for (int i = threadIdx.x; i <= GC; i += kBlock) g_pref[i] = p.bprefix[i];
    block_init(s);                                   // (its barrier also publishes g_pref)
    typename StackSel<PRIV>::type stk;
    Work w;
    uint32_t nrays = 0;
    const unsigned t_start = p.trace ? (unsigned)wall_clock64() : 0u;
    const unsigned total = g_pref[GC];
    const unsigned G = gridDim.x, b = blockIdx.x;
    const unsigned n = b < total ? (total - b + G - 1u) / G : 0u;   // rays j = b, b+G, b+2G, ...
    bool active = false, exhausted = n == 0;
    Ray r;
    float tlim = 0.0f;
    int owner = 0;
    Walk wk;
    while (true) {
        if (!exhausted) {
            const unsigned long long idle = __ballot(!active);
            if (idle) {
                const unsigned base = wave_grab_lds(&g_head, idle);
                if (base + (unsigned)__popcll(idle) >= n) exhausted = true;
                if (!active) {
                    const unsigned idx = base + lane_rank(idle);
                    if (idx < n) {
                        const unsigned j = b + idx * G;
                        int lo = 0, hi = GC;                       // g_pref[lo] <= j < g_pref[hi]
                        while (hi - lo > 1) {
                            const int m = (lo + hi) >> 1;
                            if (g_pref[m] <= j) lo = m; else hi = m;
                        }
                        const float4* sray = p.sray + 2 * ((size_t)lo * p.block_scap + (j - g_pref[lo]));
                        const float4 a = ld_nt(sray), c = ld_nt(sray + 1);
                        r = make_ray(V{a.x, a.y, a.z}, V{c.x, c.y, c.z});
                        tlim = c.w;
                        owner = __float_as_int(a.w);
                        nrays++;
                        if (walk_begin<COUNT>(s, r, wk, w, true)) active = true;
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
            if (active) {
                const int res = any_step<COUNT, FetchTop>(s, r, tlim, stk, wk, w);
                if (res) {
                    p.occ[owner] = res == 2 ? 1 : 0;
                    active = false;
                }
            }
        }
    }
    if (p.trace && threadIdx.x == 0) {
        p.trace[2 * ((size_t)p.cap + blockIdx.x)] = t_start;
        p.trace[2 * ((size_t)p.cap + blockIdx.x) + 1] = (unsigned)wall_clock64();
    }
    if (COUNT) {
        wave_add_counter(&p.counters[1], nrays);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// k_fused: chains and shadow rays in ONE persistent kernel, by wave role.
// Waves [0, P) of a workgroup are producers: exactly k_chain's loop (closest-
// hit chains, uninterrupted by shadow work), except that each finished hit
// appends one u32 task per light (owner id) to the wave's own queue and
// publishes the new tail with a workgroup-scope release.  The other waves are
// consumers from the start, and producers turn into consumers once the
// workgroup's samples are gone: they take published tasks from any producer
// queue (LDS CAS on the taken count), re-derive the shadow ray from the hit
// record and walk it (any-hit).  Shadow work thus overlaps the chains instead
// of waiting for the slowest chain of the frame (k_chain -> k_occlude).
// Queue capacity is the worst case (every sample of the workgroup recording
// every level), so no queue can overflow.
// ---------------------------------------------------------------------------
__shared__ unsigned g_pub[kBlock / 64];    // per producer wave: tasks published
__shared__ unsigned g_take[kBlock / 64];   // per producer wave: tasks taken
__shared__ unsigned g_live;                // producer waves still producing

__device__ __forceinline__ unsigned lds_acquire(unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_release(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool COUNT>
__global__ __launch_bounds__(kBlock, RT_WAVES_PER_EU) void k_fused(rtk::DevScene s, rtk::Eye e, PcParams p) {
    const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
    const int P = p.producers;
    if (threadIdx.x < kBlock / 64) {
        g_pub[threadIdx.x] = 0;
        g_take[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) g_live = (unsigned)P;
    block_init(s);
    StackPriv stk;
    Work w;
    uint32_t nprim = 0, nrefl = 0, nshadow = 0;
    const int nl = s.nlights;
    unsigned* const qbase = p.wq + (size_t)blockIdx.x * (kBlock / 64) * p.wq_cap;
    Ray r;
    Walk wk;
    if (wave < P) {
        // ---- producer: k_chain's loop ----
        const unsigned G = gridDim.x;
        const unsigned nb = block_samples((unsigned)p.n0, G);
        unsigned* q = qbase + (size_t)wave * p.wq_cap;
        unsigned pub = 0;                                   // wave-uniform
        int st = kIdle;
        bool exhausted = nb == 0;
        unsigned path = 0;
        int k = 0;
        unsigned t_grab = 0;
        while (true) {
            const bool done = st == kDone;
            const bool hit = done && wk.best.prim >= 0;
            const unsigned long long hm = __ballot(hit);
            const unsigned hcnt = (unsigned)__popcll(hm);
            const unsigned base = pub;
            pub += hcnt * (unsigned)nl;
            if (done) {
                const HitRec h = wk.best;
                V nn{0.0f, 0.0f, 0.0f}, pnt{0.0f, 0.0f, 0.0f};
                int mat = 0;
                if (hit) {
                    hit_surface(s, r, h, &nn, &mat);
                    const V hitp = add(r.o, mul(r.d, h.t));
                    float4* rc = p.rec + ((size_t)k * p.cap + path) * 3;
                    rc[0] = make_float4(hitp.x, hitp.y, hitp.z, __int_as_float(mat));
                    rc[1] = make_float4(nn.x, nn.y, nn.z, h.t);
                    rc[2] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);
                    pnt = add(hitp, mul(nn, s.eps));                              // :397
                    const unsigned rank = lane_rank(hm);
                    const unsigned own0 = (unsigned)(((size_t)k * p.cap + path) * nl);
                    for (int l = 0; l < nl; ++l) q[base + (unsigned)l * hcnt + rank] = own0 + (unsigned)l;
                }
                if (!hit) {                                                       // :442-449
                    p.pinfo[path] = k | ((k == 0 ? kEndBg : kEndZero) << 8);
                    st = kIdle;
                } else if (!s.mats[mat - 1].is_mirror) {
                    p.pinfo[path] = (k + 1) | (kEndLast << 8);
                    st = kIdle;
                } else if (k >= s.max_depth) {      // child beyond MaxRecursionDepth: 0 (:387-389)
                    p.pinfo[path] = (k + 1) | (kEndZero << 8);
                    st = kIdle;
                } else {
                    const V d2 = nrm(r.d);                                       // :431-435
                    const V n2 = nrm(nn);
                    const float rcos = dot(neg(d2), n2);
                    r = make_ray(pnt, add(d2, mul(mul(n2, 2.0f), rcos)));
                    ++k;
                    nrefl++;
                    st = walk_begin<COUNT>(s, r, wk, w) ? kTrav : kDone;
                }
                if (p.trace && st == kIdle) {
                    p.trace[2 * path] = t_grab;
                    p.trace[2 * path + 1] = (unsigned)wall_clock64();
                }
            }
            if (hcnt && lane == 0) lds_release(&g_pub[wave], pub);   // records + tasks before the tail
            if (!exhausted) {
                const unsigned long long idle = __ballot(st == kIdle);
                if (idle) {
                    const unsigned gb = wave_grab_lds(&g_head, idle);
                    if (gb + (unsigned)__popcll(idle) >= nb) exhausted = true;
                    if (st == kIdle) {
                        const unsigned v = gb + lane_rank(idle);
                        if (v < nb) {
                            const unsigned idx = block_sample(v, G, (unsigned)p.n0, (unsigned)p.spread);
                            if (slab_sample_ray(e, p, idx, &r)) {
                                path = idx;
                                k = 0;
                                nprim++;
                                if (p.trace) t_grab = (unsigned)wall_clock64();
                                if (s.max_depth < 0) p.pinfo[path] = 0 | (kEndZero << 8);   // depth 0 > max: black
                                else st = walk_begin<COUNT>(s, r, wk, w) ? kTrav : kDone;
                            }
                        }
                    }
                }
            }
            if (!__any(st != kIdle)) {
                if (exhausted) break;
                continue;
            }
            const int thresh = exhausted ? 0 : p.refill;
            while (__popcll(__ballot(st == kTrav)) > thresh && __popcll(__ballot(st == kDone)) < p.service) {
                if (st == kTrav && closest_step<COUNT, FetchTop>(s, r, stk, wk, w)) st = kDone;
            }
        }
        if (lane == 0) __hip_atomic_fetch_add(&g_live, -1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // ---- consumer: shadow tasks from every producer queue ----
    {
        bool active = false;
        float tlim = 0.0f;
        unsigned owner = 0;
        int spin = 0;
        while (true) {
            const unsigned long long idle = __ballot(!active);
            unsigned gq = 0, gt = 0, gn = 0;
            bool live = true;
            if (idle) {
                const unsigned ni = (unsigned)__popcll(idle);
                if (lane == __ffsll((unsigned long long)idle) - 1) {
                    live = lds_acquire(&g_live) != 0;    // read before the queues: a 0 here means every tail is final
                    for (int i = 0; i < P && gn == 0; ++i) {
                        const int qq = (wave + i) % P;
                        while (true) {
                            const unsigned t = __hip_atomic_load(&g_take[qq], __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
                            const unsigned pb = lds_acquire(&g_pub[qq]);
                            if (pb <= t) break;
                            const unsigned n = min(ni, pb - t);
                            unsigned expect = t;
                            if (__hip_atomic_compare_exchange_strong(&g_take[qq], &expect, t + n, __ATOMIC_RELAXED,
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
                                gq = (unsigned)qq; gt = t; gn = n;
                                break;
                            }
                        }
                    }
                }
                const int leader = __ffsll((unsigned long long)idle) - 1;
                gq = __shfl(gq, leader, 64);
                gt = __shfl(gt, leader, 64);
                gn = __shfl(gn, leader, 64);
                live = __shfl((int)live, leader, 64) != 0;
                if (!active) {
                    const unsigned rank = lane_rank(idle);
                    if (rank < gn) {
                        owner = qbase[(size_t)gq * p.wq_cap + gt + rank];
                        const unsigned lvp = owner / (unsigned)nl;
                        const int l = (int)(owner - lvp * (unsigned)nl);
                        const float4* rc = p.rec + (size_t)lvp * 3;
                        const float4 a = rc[0], b = rc[1];
                        const V pnt = add(V{a.x, a.y, a.z}, mul(V{b.x, b.y, b.z}, s.eps));   // :397
                        const float4 lp = ld4(&s.lights[l].px);
                        const V lpos{lp.x, lp.y, lp.z};
                        tlim = len(sub(lpos, pnt));                                          // :400-404
                        r = make_ray(pnt, nrm(sub(lpos, pnt)));
                        nshadow++;
                        if (walk_begin<COUNT>(s, r, wk, w, true)) active = true;
                        else p.occ[owner] = 0;
                    }
                }
            }
            if (!__any(active)) {
                if (gn == 0) {
                    if (!live) break;                 // producers done and every queue drained
                    __builtin_amdgcn_s_sleep(2);
                    ++spin;
                }
                continue;
            }
            // walk until enough lanes are free (all of them once nothing is queued)
            const int thresh = (gn > 0 || live) ? p.crefill : 0;
            while (__popcll(__ballot(active)) > thresh) {
                if (active) {
                    const int res = any_step<COUNT, FetchTop>(s, r, tlim, stk, wk, w);
                    if (res) {
                        p.occ[owner] = res == 2 ? 1 : 0;
                        active = false;
                    }
                }
            }
        }
        (void)spin;
    }
    if (COUNT) {
        wave_add_counter(&p.counters[0], nprim);
        wave_add_counter(&p.counters[1], nshadow);
        wave_add_counter(&p.counters[2], nrefl);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// Blinn-Phong of recorded level k of a path (raytracer.cpp:392-427).
__device__ __forceinline__ V shade_level(const rtk::DevScene& s, const PcParams& p, unsigned path, int k,
                                         int* mat_out) {
    const float4* rc = p.rec + ((size_t)k * p.cap + path) * 3;
    const float4 a = ld_nt(rc), b = ld_nt(rc + 1), c = ld_nt(rc + 2);
    const int mat = __float_as_int(a.w);
    *mat_out = mat;
    const V hitp{a.x, a.y, a.z}, n_{b.x, b.y, b.z}, d{c.x, c.y, c.z};
    const dl::Material& M = s.mats[mat - 1];
    const float4 mA = ld4(&M.kax), mD = ld4(&M.kdx);
    V L{0.0f, 0.0f, 0.0f};
    L = add(L, V{mA.x, mA.y, mA.z});                                                  // :394-395
    const V pnt = add(hitp, mul(n_, s.eps));                                           // :397
    const uint8_t* occ = p.occ + ((size_t)k * p.cap + path) * s.nlights;
    for (int l = 0; l < s.nlights; ++l) {
        if (occ[l]) continue;
        const float4 lp = ld4(&s.lights[l].px), li4 = ld4(&s.lights[l].ix);
        const V lpos{lp.x, lp.y, lp.z};
        const float dist = len(sub(lpos, pnt));
        const V ldir = nrm(sub(lpos, pnt));
        const V ldir_real = nrm(sub(lpos, hitp));
        const float cos_t = dot(ldir_real, n_);
        const V E = divs(V{li4.x, li4.y, li4.z}, dist * dist);
        // theta = acos(cos)*180/3.1415 <= 90.01  <=>  cos in [cos_thr, 1]
        if (cos_t >= s.cos_thr && cos_t <= 1.0f) {
            const V hh = nrm(add(ldir, neg(nrm(d))));
            const float base = smax(0.0f, dot(nrm(n_), hh));
            const float ca = (float)pow((double)base, (double)mA.w);
            const float4 mS = ld4(&M.ksx);
            L = add(L, had(mul(V{mS.x, mS.y, mS.z}, ca), E));
        }
        const float cl = smax(0.0f, smin(1.0f, cos_t));                               // clampFloat(cos, 0, 1)
        L = add(L, had(mul(V{mD.x, mD.y, mD.z}, cl), E));
    }
    return L;
}

// Recursive clamp-and-add evaluated deepest-first (raytracer.cpp:436-451).
__device__ __forceinline__ V path_color(const rtk::DevScene& s, const PcParams& p, unsigned path) {
    const int info = p.pinfo[path];
    const int nlev = info & 0xff, kind = info >> 8;
    V c = kind == kEndBg ? V{s.bgx, s.bgy, s.bgz} : V{0.0f, 0.0f, 0.0f};
    int k = nlev - 1;
    int mat;
    if (kind == kEndLast) {
        c = vclamp(shade_level(s, p, path, k, &mat), 0.0f, FLT_MAX);
        --k;
    }
    for (; k >= 0; --k) {
        const V L = shade_level(s, p, path, k, &mat);
        const float4 km = ld4(&s.mats[mat - 1].kmx);
        c = vclamp(add(L, had(c, V{km.x, km.y, km.z})), 0.0f, FLT_MAX);
    }
    return c;
}

// k_compose: shading + fold + toPixel + ImageProcessor::downSample per output pixel
__global__ __launch_bounds__(kBlock) void k_compose(rtk::DevScene s, PcParams p) {
    const int lr0 = p.chunk_row0 / p.aa;
    const int nrows = p.chunk_rows / p.aa;
    const int npix = nrows * p.width;
    const int F = p.aa;
    for (int q = blockIdx.x * kBlock + threadIdx.x; q < npix; q += gridDim.x * kBlock) {
        const int rr = q / p.width, ocol = q - rr * p.width;
        const int lr = lr0 + rr;
        if (lr >= p.slab_rows) continue;
        const int stripe = lr / p.stripe_rows;
        const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows);
        if (g >= p.height) continue;
        uint32_t sr = 0, sg = 0, sb = 0;
        for (int k = 0; k < F; ++k)
            for (int l = 0; l < F; ++l) {
                const V c = path_color(s, p, slab_slot(p.tiles_x, ocol * F + l, rr * F + k));
                sr += quantise(c.x); sg += quantise(c.y); sb += quantise(c.z);
            }
        const uint32_t ff = (uint32_t)(F * F);
        uint8_t* o = p.out + ((size_t)lr * p.width + ocol) * 3;
        o[0] = (uint8_t)(sr / ff); o[1] = (uint8_t)(sg / ff); o[2] = (uint8_t)(sb / ff);
    }
}

}  // namespace

hipError_t chain_occupancy(bool priv_stack, int* chain_blocks_per_cu, int* occlude_blocks_per_cu) {
    hipError_t e;
    if (priv_stack) {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(chain_blocks_per_cu, k_chain<false, true>, kBlock, 0);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occlude_blocks_per_cu, k_occlude<false, true>, kBlock, 0);
    } else {
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(chain_blocks_per_cu, k_chain<false, false>, kBlock, 0);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(occlude_blocks_per_cu, k_occlude<false, false>, kBlock, 0);
    }
    return e;
}

hipError_t fused_occupancy(int* blocks_per_cu) {
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_fused<false>, kBlock, 0);
}

unsigned fused_wave_qcap(int n0, int grid, int levels, int nlights) {
    return chain_block_scap(n0, grid, levels, nlights);   // a producer wave may take all of its block's samples
}

hipError_t launch_fused_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, bool count,
                              hipStream_t st) {
    if (count)
        hipLaunchKernelGGL(k_fused<true>, dim3(p.grid), dim3(kBlock), 0, st, s, e, p);
    else
        hipLaunchKernelGGL(k_fused<false>, dim3(p.grid), dim3(kBlock), 0, st, s, e, p);
    const int npix = (p.chunk_rows / p.aa) * p.width;
    hipLaunchKernelGGL(k_compose, dim3(std::max(1, std::min(p.grid, (npix + kBlock - 1) / kBlock))), dim3(kBlock),
                       0, st, s, p);
    return hipGetLastError();
}

unsigned chain_block_scap(int n0, int grid, int levels, int nlights) {
    const unsigned units = ((unsigned)n0 + 255u) / 256u;
    const unsigned per_block = (units + (unsigned)grid - 1u) / (unsigned)grid;
    return per_block * 256u * (unsigned)levels * (unsigned)nlights;
}

hipError_t launch_chain_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, bool count,
                              hipStream_t st) {
    const dim3 blk(kBlock), grid(p.grid);
#define RT_CHAIN_LAUNCH(C, P)                                                        \
    do {                                                                             \
        hipLaunchKernelGGL((k_chain<C, P>), grid, blk, 0, st, s, e, p);               \
        hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, st, p);                     \
        hipLaunchKernelGGL((k_occlude<C, P>), dim3(p.ogrid), blk, 0, st, s, p);        \
    } while (0)
    if (count) {
        if (p.priv_stack) RT_CHAIN_LAUNCH(true, true); else RT_CHAIN_LAUNCH(true, false);
    } else {
        if (p.priv_stack) RT_CHAIN_LAUNCH(false, true); else RT_CHAIN_LAUNCH(false, false);
    }
#undef RT_CHAIN_LAUNCH
    const int npix = (p.chunk_rows / p.aa) * p.width;
    hipLaunchKernelGGL(k_compose, dim3(std::max(1, std::min(p.grid, (npix + kBlock - 1) / kBlock))), blk, 0, st, s,
                       p);
    return hipGetLastError();
}

}  // namespace rtc
