// Small HIP kernels beside the chain renderer (pathchain.hip): the primary-hit
// dump of the parity surface (rt_primary_hits: the reference's own binary-tree
// walk, raytracer.cpp:177-225, one lane per internal pixel, stack in LDS laid
// out [entry][thread] so a wave's lanes touch distinct banks) and the rank-0
// reassembly of row stripes (rt_unshuffle_stripes).
#include <hip/hip_runtime.h>

#include "render_kernels.hpp"
#include "rt_device.hpp"

using namespace rtd;

namespace rtk {

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ float4 ldg4(const void* p) { return *reinterpret_cast<const float4*>(p); }

struct Counts {
    uint32_t nodes, tris, spheres;
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
