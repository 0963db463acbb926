// Chain renderer kernels (see pathchain.hpp).
#include <hip/hip_runtime.h>

#include "pathchain.hpp"
#include "traverse2.hpp"
#include "wave_util.hpp"

using namespace rtd;

namespace rtc {

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// k_chain: closest-hit chain of every sample (raytracer.cpp:385-439 minus the
// shading): record each hit, queue its shadow rays, follow mirrors.
// ---------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_chain(rtk::DevScene s, rtk::Eye e, PcParams p) {
    extern __shared__ int2 stk_lds[];
    int2* stk = stk_lds + threadIdx.x;
    Work w;
    uint32_t nprim = 0, nrefl = 0;
    const unsigned n = (unsigned)p.n0;
    const int nl = s.nlights;
    for (unsigned i0 = blockIdx.x * kBlock; i0 < n; i0 += gridDim.x * kBlock) {
        const unsigned path = i0 + threadIdx.x;
        Ray r;
        const bool valid = path < n && slab_sample_ray(e, p, path, &r);
        int nlev = 0, kind = kEndZero;
        if (valid) {
            nprim++;
            for (int k = 0; k <= s.max_depth; ++k) {                        // :387-389
                if (k > 0) nrefl++;
                const HitRec h = closest_hit2<COUNT, kBlock>(s, r, stk, w);  // :390
                if (h.prim < 0) {                                          // :442-449
                    kind = k == 0 ? kEndBg : kEndZero;
                    break;
                }
                V nn;
                int mat;
                hit_surface(s, r, h, &nn, &mat);
                const V hitp = add(r.o, mul(r.d, h.t));
                float4* rc = p.rec + ((size_t)k * p.cap + path) * 3;
                rc[0] = make_float4(hitp.x, hitp.y, hitp.z, __int_as_float(mat));
                rc[1] = make_float4(nn.x, nn.y, nn.z, h.t);
                rc[2] = make_float4(r.d.x, r.d.y, r.d.z, 0.0f);
                nlev = k + 1;
                const V pnt = add(hitp, mul(nn, s.eps));                    // :397
                // one shadow ray per light (:399-404), traced by k_occlude
                const unsigned slot = atomicAdd(p.scount, (unsigned)nl);
                for (int l = 0; l < nl; ++l) {
                    const float4 lp = ld4(&s.lights[l].px);
                    const V lpos{lp.x, lp.y, lp.z};
                    const float dist = len(sub(lpos, pnt));
                    const V ldir = nrm(sub(lpos, pnt));
                    const int owner = (int)(((size_t)k * p.cap + path) * nl + l);
                    if (slot + l < p.scap) {
                        p.sray[2 * (slot + l)] = make_float4(pnt.x, pnt.y, pnt.z, __int_as_float(owner));
                        p.sray[2 * (slot + l) + 1] = make_float4(ldir.x, ldir.y, ldir.z, dist);
                    }
                }
                if (!s.mats[mat - 1].is_mirror) {
                    kind = kEndLast;
                    break;
                }
                if (k >= s.max_depth) {            // child would be beyond MaxRecursionDepth: 0
                    kind = kEndZero;
                    break;
                }
                const V d2 = nrm(r.d);                                     // :431-435
                const V n2 = nrm(nn);
                const float rcos = dot(neg(d2), n2);
                r = make_ray(pnt, add(d2, mul(mul(n2, 2.0f), rcos)));
            }
        }
        if (path < n) p.pinfo[path] = nlev | (kind << 8);
    }
    if (COUNT) {
        wave_add_counter(&p.counters[0], nprim);
        wave_add_counter(&p.counters[2], nrefl);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// ---------------------------------------------------------------------------
// k_occlude: any-hit of every queued shadow ray (raytracer.cpp:227-280)
// ---------------------------------------------------------------------------
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_occlude(rtk::DevScene s, PcParams p) {
    extern __shared__ int2 stk_lds[];
    int2* stk = stk_lds + threadIdx.x;
    Work w;
    uint32_t nrays = 0;
    const unsigned n = min(*p.scount, p.scap);
    for (unsigned i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 a = p.sray[2 * i], b = p.sray[2 * i + 1];
        const Ray r = make_ray(V{a.x, a.y, a.z}, V{b.x, b.y, b.z});
        nrays++;
        p.occ[__float_as_int(a.w)] = any_hit2<COUNT, kBlock>(s, r, b.w, stk, w) ? 1 : 0;
    }
    if (COUNT) {
        wave_add_counter(&p.counters[1], nrays);
        wave_add_counter(&p.counters[3], w.nodes);
        wave_add_counter(&p.counters[4], w.tris);
        wave_add_counter(&p.counters[5], w.spheres);
    }
}

// Blinn-Phong of recorded level k of a path (raytracer.cpp:392-427).
__device__ __forceinline__ V shade_level(const rtk::DevScene& s, const PcParams& p, unsigned path, int k,
                                         int* mat_out) {
    const float4* rc = p.rec + ((size_t)k * p.cap + path) * 3;
    const float4 a = rc[0], b = rc[1], c = rc[2];
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

hipError_t launch_chain_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, int grid_blocks,
                              bool count, hipStream_t st) {
    const size_t lds = (size_t)s.pair_stack * kBlock * sizeof(int2);
    const dim3 blk(kBlock);
    hipError_t err = hipMemsetAsync(p.scount, 0, sizeof(unsigned), st);
    if (err != hipSuccess) return err;
    const int g0 = std::min(grid_blocks, (p.n0 + kBlock - 1) / kBlock);
    if (count) hipLaunchKernelGGL(k_chain<true>, dim3(g0), blk, lds, st, s, e, p);
    else hipLaunchKernelGGL(k_chain<false>, dim3(g0), blk, lds, st, s, e, p);
    if (count) hipLaunchKernelGGL(k_occlude<true>, dim3(grid_blocks), blk, lds, st, s, p);
    else hipLaunchKernelGGL(k_occlude<false>, dim3(grid_blocks), blk, lds, st, s, p);
    const int npix = (p.chunk_rows / p.aa) * p.width;
    hipLaunchKernelGGL(k_compose, dim3(std::min(grid_blocks, (npix + kBlock - 1) / kBlock)), blk, 0, st, s, p);
    return hipGetLastError();
}

}  // namespace rtc
