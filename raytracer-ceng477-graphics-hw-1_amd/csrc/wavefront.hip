// Wavefront renderer kernels (see wavefront.hpp for the pipeline).
#include <hip/hip_runtime.h>

#include "traverse.hpp"
#include "wavefront.hpp"

using namespace rtd;

namespace rtw {

namespace {

constexpr int kBlock = 256;

// Wave-aggregated append: one atomic per wave, lanes get consecutive slots
// (`mult` slots per lane with pred set).  Must be reached by every lane.
__device__ __forceinline__ unsigned wave_append(unsigned* counter, bool pred, unsigned mult) {
    const unsigned long long m = __ballot(pred);
    if (m == 0) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m) * mult);
    base = __shfl(base, leader, 64);
    return base + (unsigned)__popcll(m & ((1ull << lane) - 1ull)) * mult;
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void add_counter(unsigned long long* c, unsigned long long v) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(c, v);
}

// Level-0 sample slot -> eye ray.  Slots are ordered 8x8 internal-pixel tile
// by tile (one tile per wave) for coherence; rows are slab-local and mapped
// to global rows through the stripe round-robin (raytracer.cpp:353 analogue).
__device__ __forceinline__ bool sample_ray(const rtk::Eye& e, const WfParams& p, unsigned s, Ray* r) {
    const unsigned tile = s >> 6, lane = s & 63;
    const int tx = (int)(tile % (unsigned)p.tiles_x), ty = (int)(tile / (unsigned)p.tiles_x);
    const int ix = tx * 8 + (int)(lane & 7);
    const int iyc = ty * 8 + (int)(lane >> 3);
    if (ix >= p.wi || iyc >= p.chunk_rows) return false;
    const int iy = p.chunk_row0 + iyc;
    const int lr = iy / p.aa, sub = iy - lr * p.aa;
    if (lr >= p.slab_rows) return false;
    const int stripe = lr / p.stripe_rows;
    const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows);
    if (g >= p.height) return false;
    *r = eye_ray(e, g * p.aa + sub, ix);
    return true;
}

__device__ __forceinline__ Ray queue_ray(const float4* q, unsigned i) {
    const float4 o = q[2 * i], d = q[2 * i + 1];
    return make_ray(V{o.x, o.y, o.z}, V{d.x, d.y, d.z});
}

// ---------------------------------------------------------------------------
// closest hit of level `level` + hit epilogue + shadow-ray generation
// ---------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_trace(rtk::DevScene s, rtk::Eye e, WfParams p, int level) {
    extern __shared__ int lds[];
    int* stk = lds + threadIdx.x;
    const unsigned n = level == 0 ? (unsigned)p.n0 : p.qcount[level];
    const float4* qin = p.q[level & 1];
    float4* R = p.R + (size_t)level * p.cap;
    int* child = p.child + (size_t)level * p.cap;
    const bool beyond = level > s.max_depth;
    Work w;
    uint32_t nrays = 0;
    for (unsigned i0 = blockIdx.x * kBlock; i0 < n; i0 += gridDim.x * kBlock) {
        const unsigned i = i0 + threadIdx.x;
        bool valid = i < n;
        Ray r;
        if (valid) {
            if (level == 0) valid = sample_ray(e, p, i, &r);
            else r = queue_ray(qin, i);
        }
        HitRec h{-1.0f, -1};
        if (valid) {
            nrays++;
            if (!beyond) h = closest_hit<COUNT, kBlock>(s, r, stk, w);           // :390
        }
        const bool hit = h.prim >= 0;
        V pnt{0.0f, 0.0f, 0.0f};
        if (hit) {
            V nrm_;
            int mat;
            hit_surface(s, r, h, &nrm_, &mat);
            pnt = add(add(r.o, mul(r.d, h.t)), mul(nrm_, s.eps));              // :397
            p.hit[2 * i] = make_float4(pnt.x, pnt.y, pnt.z, __int_as_float(mat));
            p.hit[2 * i + 1] = make_float4(nrm_.x, nrm_.y, nrm_.z, h.t);
        } else if (i < n) {
            p.hit[2 * i] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(0));
            // miss: background at depth 0, black deeper (:442-449); beyond max depth: black (:387-389)
            const bool bg = valid && level == 0 && !beyond;
            R[i] = make_float4(bg ? s.bgx : 0.0f, bg ? s.bgy : 0.0f, bg ? s.bgz : 0.0f, __int_as_float(0));
            child[i] = -1;
        }
        // one shadow ray per light (:399-404)
        const unsigned slot = wave_append(&p.scount[level], hit, (unsigned)s.nlights);
        if (hit) {
            for (int l = 0; l < s.nlights; ++l) {
                const float4 lp = ld4(&s.lights[l].px);
                const V lpos{lp.x, lp.y, lp.z};
                const float dist = len(sub(lpos, pnt));
                const V ldir = nrm(sub(lpos, pnt));
                p.sray[2 * (slot + l)] = make_float4(pnt.x, pnt.y, pnt.z, __int_as_float((int)(i * s.nlights + l)));
                p.sray[2 * (slot + l) + 1] = make_float4(ldir.x, ldir.y, ldir.z, dist);
            }
        }
    }
    if (COUNT) {
        add_counter(&p.counters[level == 0 ? 0 : 2], nrays);
        add_counter(&p.counters[3], w.nodes);
        add_counter(&p.counters[4], w.tris);
        add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// any-hit of the shadow queue (raytracer.cpp:227-280)
// ---------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_shadow(rtk::DevScene s, WfParams p, int level) {
    extern __shared__ int lds[];
    int* stk = lds + threadIdx.x;
    const unsigned n = p.scount[level];
    Work w;
    uint32_t nrays = 0;
    for (unsigned i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 a = p.sray[2 * i], b = p.sray[2 * i + 1];
        const Ray r = make_ray(V{a.x, a.y, a.z}, V{b.x, b.y, b.z});
        nrays++;
        p.occ[__float_as_int(a.w)] = any_hit<COUNT, kBlock>(s, r, b.w, stk, w) ? 1 : 0;
    }
    if (COUNT) {
        add_counter(&p.counters[1], nrays);
        add_counter(&p.counters[3], w.nodes);
        add_counter(&p.counters[4], w.tris);
        add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// Blinn-Phong shading + mirror spawn (raytracer.cpp:392-439)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_shade(rtk::DevScene s, rtk::Eye e, WfParams p, int level) {
    const unsigned n = level == 0 ? (unsigned)p.n0 : p.qcount[level];
    const float4* qin = p.q[level & 1];
    float4* qout = p.q[(level + 1) & 1];
    float4* R = p.R + (size_t)level * p.cap;
    int* child = p.child + (size_t)level * p.cap;
    for (unsigned i0 = blockIdx.x * kBlock; i0 < n; i0 += gridDim.x * kBlock) {
        const unsigned i = i0 + threadIdx.x;
        int mat = 0;
        float4 h0 = make_float4(0, 0, 0, 0);
        if (i < n) {
            h0 = p.hit[2 * i];
            mat = __float_as_int(h0.w);
        }
        bool spawn = false;
        V pnt{h0.x, h0.y, h0.z}, refl{0.0f, 0.0f, 0.0f};
        if (mat != 0) {
            Ray r;
            if (level == 0) sample_ray(e, p, i, &r);
            else r = queue_ray(qin, i);
            const float4 h1 = p.hit[2 * i + 1];
            const V n_{h1.x, h1.y, h1.z};
            const float t = h1.w;
            const dl::Material& M = s.mats[mat - 1];
            const float4 mA = ld4(&M.kax), mD = ld4(&M.kdx);
            V L{0.0f, 0.0f, 0.0f};
            L = add(L, V{mA.x, mA.y, mA.z});                                         // :394-395
            const V hitp = add(r.o, mul(r.d, t));
            for (int l = 0; l < s.nlights; ++l) {                                     // :399-427
                if (p.occ[i * s.nlights + l]) continue;
                const float4 lp = ld4(&s.lights[l].px), li4 = ld4(&s.lights[l].ix);
                const V lpos{lp.x, lp.y, lp.z};
                const float dist = len(sub(lpos, pnt));
                const V ldir = nrm(sub(lpos, pnt));
                const V ldir_real = nrm(sub(lpos, hitp));
                const float cos_t = dot(ldir_real, n_);
                const V E = divs(V{li4.x, li4.y, li4.z}, dist * dist);
                // theta = acos(cos)*180/3.1415 <= 90.01  <=>  cos in [cos_thr, 1]
                if (cos_t >= s.cos_thr && cos_t <= 1.0f) {
                    const V hh = nrm(add(ldir, neg(nrm(r.d))));
                    const float base = smax(0.0f, dot(nrm(n_), hh));
                    const float ca = phong_pow(base, mA.w);
                    const float4 mS = ld4(&M.ksx);
                    L = add(L, had(mul(V{mS.x, mS.y, mS.z}, ca), E));
                }
                const float cl = smax(0.0f, smin(1.0f, cos_t));                      // clampFloat(cos, 0, 1)
                L = add(L, had(mul(V{mD.x, mD.y, mD.z}, cl), E));
            }
            if (__float_as_int(mD.w)) {                                              // :430-439
                R[i] = make_float4(L.x, L.y, L.z, __int_as_float(mat));
                const V d2 = nrm(r.d);
                const V n2 = nrm(n_);
                const float rc = dot(neg(d2), n2);
                refl = add(d2, mul(mul(n2, 2.0f), rc));
                spawn = level < s.max_depth;
                if (!spawn) child[i] = -2;                                           // depth > max: 0
            } else {
                const V cl = vclamp(L, 0.0f, FLT_MAX);                                // :451
                R[i] = make_float4(cl.x, cl.y, cl.z, __int_as_float(0));
                child[i] = -1;
            }
        }
        const unsigned slot = wave_append(&p.qcount[level + 1], spawn, 1u);
        if (spawn) {
            qout[2 * slot] = make_float4(pnt.x, pnt.y, pnt.z, 0.0f);
            qout[2 * slot + 1] = make_float4(refl.x, refl.y, refl.z, 0.0f);
            child[i] = (int)slot;
        }
    }
}

// c_k = clamp(L_k + c_{k+1} (x) km_k, 0, FLT_MAX), deepest level first.
__device__ __forceinline__ V fold_value(const rtk::DevScene& s, const float4 r, int ch, const float4* Rnext) {
    const int mat = __float_as_int(r.w);
    if (mat == 0) return V{r.x, r.y, r.z};
    V rec{0.0f, 0.0f, 0.0f};
    if (ch >= 0) {
        const float4 c = Rnext[ch];
        rec = V{c.x, c.y, c.z};
    }
    const float4 km = ld4(&s.mats[mat - 1].kmx);
    return vclamp(add(V{r.x, r.y, r.z}, had(rec, V{km.x, km.y, km.z})), 0.0f, FLT_MAX);
}

__global__ __launch_bounds__(kBlock) void k_fold(rtk::DevScene s, WfParams p, int level) {
    const unsigned n = p.qcount[level];
    float4* R = p.R + (size_t)level * p.cap;
    const float4* Rn = p.R + (size_t)(level + 1) * p.cap;
    const int* child = p.child + (size_t)level * p.cap;
    for (unsigned i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 r = R[i];
        if (__float_as_int(r.w) == 0) continue;
        const V c = fold_value(s, r, child[i], Rn);
        R[i] = make_float4(c.x, c.y, c.z, r.w);
    }
}

// level-0 fold + toPixel + ImageProcessor::downSample, one output pixel per thread
__global__ __launch_bounds__(kBlock) void k_resolve(rtk::DevScene s, WfParams p) {
    const int lr0 = p.chunk_row0 / p.aa;
    const int nrows = p.chunk_rows / p.aa;
    const int npix = nrows * p.width;
    const float4* R0 = p.R;
    const float4* R1 = p.R + p.cap;
    const int* child0 = p.child;
    const int F = p.aa;
    for (int q = blockIdx.x * kBlock + threadIdx.x; q < npix; q += gridDim.x * kBlock) {
        const int rr = q / p.width, ocol = q - rr * p.width;
        const int lr = lr0 + rr;
        if (lr >= p.slab_rows) continue;
        const int stripe = lr / p.stripe_rows;
        const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows);
        if (g >= p.height) continue;
        uint32_t sr = 0, sg = 0, sb = 0;
        for (int k = 0; k < F; ++k) {
            const int iyc = rr * F + k;
            for (int l = 0; l < F; ++l) {
                const int ix = ocol * F + l;
                const unsigned sidx = ((unsigned)((iyc >> 3) * p.tiles_x + (ix >> 3)) << 6) |
                                      (unsigned)((iyc & 7) * 8 + (ix & 7));
                const V c = fold_value(s, R0[sidx], child0[sidx], R1);
                sr += quantise(c.x); sg += quantise(c.y); sb += quantise(c.z);
            }
        }
        const uint32_t ff = (uint32_t)(F * F);
        uint8_t* o = p.out + ((size_t)lr * p.width + ocol) * 3;
        o[0] = (uint8_t)(sr / ff); o[1] = (uint8_t)(sg / ff); o[2] = (uint8_t)(sb / ff);
    }
}

}  // namespace

hipError_t launch_frame_chunk(const rtk::DevScene& s, const rtk::Eye& e, const WfParams& p, int grid_blocks,
                              bool count, hipStream_t st) {
    const int levels = (s.max_depth > 0 ? s.max_depth : 0) + 1;
    const size_t stack_lds = (size_t)s.stack_entries * kBlock * sizeof(int);
    const dim3 blk(kBlock);
    hipError_t err = hipMemsetAsync(p.qcount, 0, sizeof(unsigned) * (2 * levels + 2), st);
    if (err != hipSuccess) return err;
    const int g0 = std::min(grid_blocks, (p.n0 + kBlock - 1) / kBlock);
    for (int k = 0; k < levels; ++k) {
        const int g = k == 0 ? g0 : grid_blocks;
        if (count) hipLaunchKernelGGL(k_trace<true>, dim3(g), blk, stack_lds, st, s, e, p, k);
        else hipLaunchKernelGGL(k_trace<false>, dim3(g), blk, stack_lds, st, s, e, p, k);
        if (count) hipLaunchKernelGGL(k_shadow<true>, dim3(grid_blocks), blk, stack_lds, st, s, p, k);
        else hipLaunchKernelGGL(k_shadow<false>, dim3(grid_blocks), blk, stack_lds, st, s, p, k);
        hipLaunchKernelGGL(k_shade, dim3(g), blk, 0, st, s, e, p, k);
    }
    // deepest level first; the deepest level's mirrors fold with a zero child (:387-389)
    for (int k = levels - 1; k >= 1; --k) hipLaunchKernelGGL(k_fold, dim3(grid_blocks), blk, 0, st, s, p, k);
    const int npix = (p.chunk_rows / p.aa) * p.width;
    hipLaunchKernelGGL(k_resolve, dim3(std::min(grid_blocks, (npix + kBlock - 1) / kBlock)), blk, 0, st, s, p);
    return hipGetLastError();
}

}  // namespace rtw
