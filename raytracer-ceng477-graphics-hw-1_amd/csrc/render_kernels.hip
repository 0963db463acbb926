// HIP kernels (gfx950) for the hot path: primary raygen -> ordered-DFS
// closest-hit -> Blinn-Phong + any-hit shadow rays -> mirror recursion ->
// quantise -> SSAA box filter, one megakernel per frame.
//
// Mapping: 256-thread workgroup = 4 waves; each wave owns an 8x8 tile of
// OUTPUT pixels (lane = 8*ty + tx) and loops over the F*F SSAA samples of its
// pixel.  Traversal stacks live in LDS, laid out [entry][thread] so a wave's
// 64 lanes always touch 64 distinct banks whatever their stack depths.  The
// per-level {local colour, material} records needed to fold the recursion
// back-to-front (raytracer.cpp:436-451) also live in LDS.
#include <hip/hip_runtime.h>

#include "render_kernels.hpp"
#include "rt_device.hpp"

using namespace rtd;

namespace rtk {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float4 ldg4(const void* p) { return *reinterpret_cast<const float4*>(p); }

struct Counts {
    uint32_t primary, shadow, reflection, nodes, tris, spheres;
};

struct Hit {
    float t;
    int prim;   // leaf prim index of the winner, -1 = none
};

// Ray::getFirstIntersection (raytracer.cpp:177-225).
template <bool COUNT>
__device__ Hit closest_hit(const DevScene& s, const Ray& r, int* stk, Counts& cnt) {
    Hit best{-1.0f, -1};
    float tmax = FLT_MAX;
    int sp = 0;
    if (s.nnodes > 0) { stk[0] = 0; sp = 1; }
    while (sp > 0) {
        --sp;
        const int ni = stk[sp * kBlock];
        const float4 lo = ldg4(&s.nodes[ni].minx);
        const float4 hi = ldg4(&s.nodes[ni].maxx);
        if (COUNT) cnt.nodes++;
        float bt;
        if (!(box_hit(r, lo, hi, &bt) && bt <= tmax)) continue;
        const int b = __float_as_int(hi.w);
        const int a = __float_as_int(lo.w);
        if (b >= 0) {   // interior: b = axis, a = right child index
            if (comp(r.d, b) > 0) { stk[sp * kBlock] = a; stk[(sp + 1) * kBlock] = ni + 1; }
            else { stk[sp * kBlock] = ni + 1; stk[(sp + 1) * kBlock] = a; }
            sp += 2;
            continue;
        }
        const int ntri = b & dl::kNtriMask;
        const int nsph = (b >> dl::kNtriBits) & dl::kMaxLeafSpheres;
        for (int i = a; i < a + ntri; ++i) {
            const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
            if (COUNT) cnt.tris++;
            float t;
            if (tri_hit(r, pr[0], pr[1], pr[2], &t) && (t < best.t || best.t == -1.0f)) {
                best.t = t; best.prim = i; tmax = t;
            }
        }
        for (int i = a + ntri; i < a + ntri + nsph; ++i) {
            const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
            if (COUNT) cnt.spheres++;
            float t;
            if (sphere_hit(r, pr[0], pr[1], &t) && (t < best.t || best.t == -1.0f)) {
                best.t = t; best.prim = i; tmax = t;
            }
        }
    }
    return best;
}

// Ray::getAnyIntersectionUntilT + traverse (raytracer.cpp:227-280).
template <bool COUNT>
__device__ bool any_hit(const DevScene& s, const Ray& r, float tlim, int* stk, Counts& cnt) {
    int sp = 0;
    if (s.nnodes > 0) { stk[0] = 0; sp = 1; }
    while (sp > 0) {
        --sp;
        const int ni = stk[sp * kBlock];
        const float4 lo = ldg4(&s.nodes[ni].minx);
        const float4 hi = ldg4(&s.nodes[ni].maxx);
        if (COUNT) cnt.nodes++;
        float bt;
        if (!box_hit(r, lo, hi, &bt)) continue;
        const int b = __float_as_int(hi.w);
        const int a = __float_as_int(lo.w);
        if (b >= 0) {
            if (comp(r.d, b) > 0) { stk[sp * kBlock] = a; stk[(sp + 1) * kBlock] = ni + 1; }
            else { stk[sp * kBlock] = ni + 1; stk[(sp + 1) * kBlock] = a; }
            sp += 2;
            continue;
        }
        const int ntri = b & dl::kNtriMask;
        const int nsph = (b >> dl::kNtriBits) & dl::kMaxLeafSpheres;
        for (int i = a; i < a + ntri; ++i) {
            const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
            if (COUNT) cnt.tris++;
            float t;
            if (tri_hit(r, pr[0], pr[1], pr[2], &t) && t < tlim) return true;
        }
        for (int i = a + ntri; i < a + ntri + nsph; ++i) {
            const float4* pr = reinterpret_cast<const float4*>(&s.prims[i]);
            if (COUNT) cnt.spheres++;
            float t;
            if (sphere_hit(r, pr[0], pr[1], &t) && t < tlim) return true;
        }
    }
    return false;
}

// EyeRayGenerator::generate (raytracer.cpp:319-324).  (col+0.5)*su is a
// double expression in the reference whose value is the exact product of
// two floats, so the correctly rounded fp32 product is bit-identical.
__device__ __forceinline__ Ray eye_ray(const Eye& e, int row, int col) {
    const float su = ((float)col + 0.5f) * e.su;
    const float sv = ((float)row + 0.5f) * e.sv;
    const V q{e.qx, e.qy, e.qz}, u{e.ux, e.uy, e.uz}, v{e.vx, e.vy, e.vz}, eye{e.ex, e.ey, e.ez};
    const V sp = sub(add(q, mul(u, su)), mul(v, sv));
    return make_ray(eye, sub(sp, eye));
}

// RayTracer::rayTrace (raytracer.cpp:385-452) unrolled into a loop over
// recursion depth; mirror levels park {L_k, material_k} in LDS and the
// clamp-and-add recursion c_k = clamp(L_k + c_{k+1} (x) km_k) is folded
// deepest-first afterwards, which reproduces the recursive evaluation order.
template <bool COUNT>
__device__ V trace_path(const DevScene& s, Ray ray, int* stk, float* fold, Counts& cnt) {
    int depth = 0;
    int nlev = 0;
    V c{0.0f, 0.0f, 0.0f};
    while (true) {
        if (depth > s.max_depth) { c = V{0.0f, 0.0f, 0.0f}; break; }          // :387-389
        if (COUNT && depth > 0) cnt.reflection++;
        const Hit h = closest_hit<COUNT>(s, ray, stk, cnt);                    // :390
        if (h.prim < 0) {                                                      // :442-449
            c = depth > 0 ? V{0.0f, 0.0f, 0.0f} : V{s.bgx, s.bgy, s.bgz};
            break;
        }
        // Winner's normal and material (Intersection::normal / material_id).
        const float4* pr = reinterpret_cast<const float4*>(&s.prims[h.prim]);
        const float4 p0 = pr[0];
        V n;
        int mat;
        if (s.prim_is_sphere(h.prim, p0)) {
            const float4 p1 = pr[1];
            n = sphere_normal(ray, p0, p1.x, h.t);
            mat = __float_as_int(pr[2].w);
        } else {
            const dl::TriShade ts = s.tri_shade[__float_as_int(p0.w)];
            n = V{ts.nx, ts.ny, ts.nz};
            mat = ts.material;
        }
        const dl::Material& M = s.mats[mat - 1];
        const float4 mA = ldg4(&M.kax), mD = ldg4(&M.kdx);
        V L = V{0.0f, 0.0f, 0.0f};
        L = add(L, V{mA.x, mA.y, mA.z});                                       // :394-395
        const V hitp = add(ray.o, mul(ray.d, h.t));                            // getPoint
        const V p = add(hitp, mul(n, s.eps));                                  // :397
        for (int li = 0; li < s.nlights; ++li) {                               // :399-427
            const float4 lp = ldg4(&s.lights[li].px), li4 = ldg4(&s.lights[li].ix);
            const V lpos{lp.x, lp.y, lp.z};
            const float dist = len(sub(lpos, p));
            const V ldir = nrm(sub(lpos, p));
            const V ldir_real = nrm(sub(lpos, add(ray.o, mul(ray.d, h.t))));
            const Ray lray = make_ray(p, ldir);
            if (COUNT) cnt.shadow++;
            if (any_hit<COUNT>(s, lray, dist, stk, cnt)) continue;
            const float cos_t = dot(ldir_real, n);
            const V E = divs(V{li4.x, li4.y, li4.z}, dist * dist);
            // theta = acos(cos)*180/3.1415 <= 90.01  <=>  cos in [cos_thr, 1]
            if (cos_t >= s.cos_thr && cos_t <= 1.0f) {
                const V hh = nrm(add(lray.d, neg(nrm(ray.d))));
                const float base = smax(0.0f, dot(nrm(n), hh));
                const float ca = phong_pow(base, mA.w);
                const float4 mS = ldg4(&M.ksx);
                L = add(L, had(mul(V{mS.x, mS.y, mS.z}, ca), E));
            }
            const float cl = smax(0.0f, smin(1.0f, cos_t));                   // clampFloat(cos, 0, 1)
            L = add(L, had(mul(V{mD.x, mD.y, mD.z}, cl), E));
        }
        if (__float_as_int(mD.w)) {                                            // :430-439
            fold[(nlev * 4 + 0) * kBlock] = L.x;
            fold[(nlev * 4 + 1) * kBlock] = L.y;
            fold[(nlev * 4 + 2) * kBlock] = L.z;
            fold[(nlev * 4 + 3) * kBlock] = __int_as_float(mat);
            ++nlev;
            const V d2 = nrm(ray.d);
            const V n2 = nrm(n);
            const float rc = dot(neg(d2), n2);
            ray = make_ray(p, add(d2, mul(mul(n2, 2.0f), rc)));
            ++depth;
            if (s.prio) wave_priority(depth);
            continue;
        }
        c = vclamp(L, 0.0f, FLT_MAX);                                          // :451
        break;
    }
    for (int k = nlev - 1; k >= 0; --k) {
        const V Lk{fold[(k * 4 + 0) * kBlock], fold[(k * 4 + 1) * kBlock], fold[(k * 4 + 2) * kBlock]};
        const int mk = __float_as_int(fold[(k * 4 + 3) * kBlock]);
        const float4 km = ldg4(&s.mats[mk - 1].kmx);
        c = vclamp(add(Lk, had(c, V{km.x, km.y, km.z})), 0.0f, FLT_MAX);     // :438, :451
    }
    return c;
}

__device__ __forceinline__ uint32_t quantise(float x) {                    // toPixel parser.h:88-93
    const float k = smax(0.0f, smin(x, 255.0f));
    return (uint32_t)__builtin_roundf(k);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_render(DevScene s, Eye e, FrameParams p) {
    extern __shared__ int lds[];
    const int tid = threadIdx.x;
    int* stk = lds + tid;
    float* fold = reinterpret_cast<float*>(lds + s.stack_entries * kBlock) + tid;
    const int wave = tid >> 6, lane = tid & 63;
    const int ocol = (blockIdx.x * 2 + (wave & 1)) * 8 + (lane & 7);
    const int lrow = (blockIdx.y * 2 + (wave >> 1)) * 8 + (lane >> 3);
    Counts cnt{0, 0, 0, 0, 0, 0};
    const unsigned t_start = p.trace ? (unsigned)wall_clock64() : 0u;
    bool active = ocol < p.width && lrow < p.slab_rows;
    int grow = 0;
    if (active) {
        const int stripe = lrow / p.stripe_rows;
        grow = (stripe * p.nranks + p.rank) * p.stripe_rows + lrow % p.stripe_rows;
        active = grow < p.height;
    }
    if (active) {
        const int F = p.aa;
        uint32_t sr = 0, sg = 0, sb = 0;
        for (int k = 0; k < F; ++k)
            for (int l = 0; l < F; ++l) {
                const Ray r = eye_ray(e, grow * F + k, ocol * F + l);
                if (COUNT) cnt.primary++;
                const V c = trace_path<COUNT>(s, r, stk, fold, cnt);
                sr += quantise(c.x); sg += quantise(c.y); sb += quantise(c.z);
            }
        const uint32_t ff = (uint32_t)(F * F);                               // downSample :459-484
        uint8_t* o = p.out + ((size_t)lrow * p.width + ocol) * 3;
        o[0] = (uint8_t)(sr / ff); o[1] = (uint8_t)(sg / ff); o[2] = (uint8_t)(sb / ff);
        if (p.trace) {
            const size_t q = (size_t)lrow * p.width + ocol;
            p.trace[2 * q] = t_start;
            p.trace[2 * q + 1] = (unsigned)wall_clock64();
        }
    }
    if (COUNT) {
        const unsigned long long v[6] = {cnt.primary, cnt.shadow, cnt.reflection, cnt.nodes, cnt.tris, cnt.spheres};
        for (int i = 0; i < 6; ++i) {
            const unsigned long long w = wave_sum(v[i]);
            if (lane == 0 && w) atomicAdd(&p.counters[i], w);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_primary_hits(DevScene s, Eye e, int W, int H, float* t_out, int* m_out) {
    extern __shared__ int lds[];
    int* stk = lds + threadIdx.x;
    const int idx = blockIdx.x * kBlock + threadIdx.x;
    if (idx >= W * H) return;
    const int row = idx / W, col = idx % W;
    Counts cnt{};
    const Ray r = eye_ray(e, row, col);
    const Hit h = closest_hit<false>(s, r, stk, cnt);
    int mat = 0;
    if (h.prim >= 0) {
        const float4 p0 = reinterpret_cast<const float4*>(&s.prims[h.prim])[0];
        mat = s.prim_is_sphere(h.prim, p0) ? __float_as_int(reinterpret_cast<const float4*>(&s.prims[h.prim])[2].w)
                                           : s.tri_shade[__float_as_int(p0.w)].material;
    }
    t_out[idx] = h.t;
    m_out[idx] = mat;
}

// Rank-0 reassembly of round-robin stripes (inverse of the k_render mapping).
__global__ void k_unshuffle(const uint8_t* slabs, uint8_t* img, int row_bytes, int height, int stripe_rows,
                            int nranks, int slab_rows) {
    const int y = blockIdx.y;
    if (y >= height) return;
    const int stripe = y / stripe_rows;
    const int owner = stripe % nranks;
    const int lrow = (stripe / nranks) * stripe_rows + y % stripe_rows;
    const uint8_t* src = slabs + ((size_t)owner * slab_rows + lrow) * row_bytes;
    uint8_t* dst = img + (size_t)y * row_bytes;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < row_bytes; i += gridDim.x * blockDim.x) dst[i] = src[i];
}

}  // namespace

size_t render_lds_bytes(const DevScene& s) {
    return (size_t)(s.stack_entries + 4 * (s.max_depth + 1)) * kBlock * sizeof(int);
}

hipError_t launch_render(const DevScene& s, const Eye& e, const FrameParams& p, bool count, hipStream_t stream) {
    const dim3 grid((p.width + 15) / 16, (p.slab_rows + 15) / 16);
    const size_t lds = render_lds_bytes(s);
    if (count)
        hipLaunchKernelGGL(k_render<true>, grid, dim3(kBlock), lds, stream, s, e, p);
    else
        hipLaunchKernelGGL(k_render<false>, grid, dim3(kBlock), lds, stream, s, e, p);
    return hipGetLastError();
}

hipError_t launch_primary_hits(const DevScene& s, const Eye& e, int W, int H, float* t, int* m, hipStream_t stream) {
    const int n = W * H;
    hipLaunchKernelGGL(k_primary_hits, dim3((n + kBlock - 1) / kBlock), dim3(kBlock),
                       (size_t)s.stack_entries * kBlock * sizeof(int), stream, s, e, W, H, t, m);
    return hipGetLastError();
}

hipError_t launch_unshuffle(const uint8_t* slabs, uint8_t* img, int width, int height, int stripe_rows, int nranks,
                            int slab_rows, hipStream_t stream) {
    const int row_bytes = width * 3;
    const dim3 grid((row_bytes + 255) / 256, height);
    hipLaunchKernelGGL(k_unshuffle, grid, dim3(256), 0, stream, slabs, img, row_bytes, height, stripe_rows, nranks,
                       slab_rows);
    return hipGetLastError();
}

}  // namespace rtk
