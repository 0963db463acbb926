// Measured roofline denominators on the device the renderer runs on
// (rt_measure_peaks, include/rt/rt.h; SURVEY.md §8(d): "Fraction = that /
// measured HBM peak, where the peak comes from a streaming-copy kernel on the
// box").  Three kernels:
//   * k_copy: streaming float4 copy of a buffer far larger than the Infinity
//     Cache (read + write bytes over time) -- the HBM peak;
//   * k_read: the same buffer read only (a running XOR) -- the HBM read peak;
//   * k_walk: the walks' own fetch shape -- one dependent 128-B line per lane
//     per step (eight dwordx4, each lane its own line: 64 distinct lines per
//     wave instruction), best of 8..20 waves per CU (~10 TB/s);
//   * k_gather (8 lanes per line): the same bytes as full-line fetches, 8
//     distinct lines per wave instruction, many in flight -- what the L2
//     delivers (~25 TB/s).
//   Both over a table that fits one XCD's 4 MiB L2 and over a table the size
//   of the scene's walk hot set (lines beyond L2 come from the Infinity Cache).
// Times are best-of-N HIP event intervals on a private stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "rt/rt.h"
#include "rt_internal.hpp"

namespace {

constexpr int kBlk = 256;

// U 16-B loads in flight per lane before their stores (plain or nontemporal); n: a multiple of U x the
// grid's threads.  rt_measure_peaks keeps the best variant and grid (MI355X_MICROARCH.md: ~6.3 TB/s).
typedef float f4v __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ __launch_bounds__(kBlk) void k_copy(const float4* __restrict__ src_, float4* __restrict__ dst_, size_t n) {
    const f4v* src = reinterpret_cast<const f4v*>(src_);
    f4v* dst = reinterpret_cast<f4v*>(dst_);
    const size_t stride = (size_t)gridDim.x * kBlk;
    for (size_t i = (size_t)blockIdx.x * kBlk + threadIdx.x; i + (U - 1) * stride < n; i += U * stride) {
        f4v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
}

__global__ __launch_bounds__(kBlk) void k_read(const float4* __restrict__ src, size_t n, unsigned* sink) {
    const size_t stride = (size_t)gridDim.x * kBlk;
    unsigned acc = 0;
    size_t i = (size_t)blockIdx.x * kBlk + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {      // four loads in flight per lane
        const float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
        acc ^= __float_as_uint(a.x) ^ __float_as_uint(a.y) ^ __float_as_uint(a.z) ^ __float_as_uint(a.w) ^
               __float_as_uint(b.x) ^ __float_as_uint(b.y) ^ __float_as_uint(b.z) ^ __float_as_uint(b.w) ^
               __float_as_uint(c.x) ^ __float_as_uint(c.y) ^ __float_as_uint(c.z) ^ __float_as_uint(c.w) ^
               __float_as_uint(d.x) ^ __float_as_uint(d.y) ^ __float_as_uint(d.z) ^ __float_as_uint(d.w);
    }
    for (; i < n; i += stride) {
        const float4 a = src[i];
        acc ^= __float_as_uint(a.x) ^ __float_as_uint(a.y) ^ __float_as_uint(a.z) ^ __float_as_uint(a.w);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;            // never true in practice; keeps the loads
}

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned pick(unsigned h, unsigned n) { return (unsigned)(((unsigned long long)h * n) >> 32); }

// ITER iterations per lane, UNROLL independent random lines in flight per lane.  COOP = false: every
// lane reads its own line (eight dwordx4, 64 distinct lines per wave instruction: the walks'
// divergent fetch); COOP = true: the same bytes with the 8 lanes of each group reading the 8 pieces
// of one line (8 distinct lines per wave instruction: what the L2 delivers to full-line fetches).
template <int UNROLL, bool COOP>
__global__ __launch_bounds__(kBlk) void k_gather(const float4* __restrict__ tab, unsigned nlines, int iters,
                                                 unsigned seed, unsigned* sink) {
    const unsigned gtid = blockIdx.x * kBlk + threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (int it = 0; it < iters; it += UNROLL) {
        float4 v[UNROLL][8];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (!COOP) {
                const unsigned line = pick(mix32(gtid * 0x9e3779b1u + (unsigned)(it + u) * 0x85ebca6bu + seed), nlines);
                const float4* q = tab + (size_t)line * 8;
#pragma unroll
                for (int j = 0; j < 8; ++j) v[u][j] = q[j];
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const unsigned owner = (gtid & ~63u) + (lane >> 3) + 8u * (unsigned)j;
                    const unsigned line = pick(mix32(owner * 0x9e3779b1u + (unsigned)(it + u) * 0x85ebca6bu + seed), nlines);
                    v[u][j] = tab[(size_t)line * 8 + (lane & 7)];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j)
                acc ^= __float_as_uint(v[u][j].x) ^ __float_as_uint(v[u][j].y) ^ __float_as_uint(v[u][j].z) ^
                       __float_as_uint(v[u][j].w);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

// The walks' own shape: one dependent 128-B line per lane per step (the next line from the data), each
// lane its own line (eight dwordx4: 64 distinct lines per wave instruction), STEPS steps.
__global__ __launch_bounds__(kBlk) void k_walk(const float4* __restrict__ tab, unsigned nlines, int steps,
                                              unsigned* sink) {
    unsigned line = pick(mix32(blockIdx.x * kBlk + threadIdx.x), nlines);
    unsigned acc = 0;
    for (int st = 0; st < steps; ++st) {
        const float4* q = tab + (size_t)line * 8;
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = q[j];
        unsigned h = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            h ^= __float_as_uint(v[j].x) ^ __float_as_uint(v[j].y) ^ __float_as_uint(v[j].z) ^ __float_as_uint(v[j].w);
        acc ^= h;
        line = pick(mix32(h ^ (unsigned)st ^ ((blockIdx.x * kBlk + threadIdx.x) * 0x9e3779b1u)), nlines);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

#define PK_TRY(expr)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) {                                                                      \
            err = std::string(#expr) + ": " + hipGetErrorName(e_);                                   \
            goto done;                                                                               \
        }                                                                                            \
    } while (0)

}  // namespace

extern "C" int rt_measure_peaks(int device, uint64_t scene_table_bytes, rt_peaks* out) {
    if (!out) return rt_internal_set_error(RT_ERR_ARG, "peaks: out is NULL");
    *out = rt_peaks{};
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return rt_internal_set_error(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (device >= ndev) return rt_internal_set_error(RT_ERR_ARG, "peaks: device ordinal out of range");
    std::string err;
    float4 *big = nullptr, *big2 = nullptr, *tab = nullptr;
    unsigned* sink = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const size_t big_bytes = size_t(2) << 30;                    // 2 GiB: 8x the 256 MiB Infinity Cache
    const size_t nbig = big_bytes / sizeof(float4);
    const size_t small_table = size_t(2) << 20;                   // 2 MiB: inside one XCD's 4 MiB L2
    const size_t scene_table = std::max<size_t>(128, std::min<size_t>(scene_table_bytes, size_t(64) << 20)) & ~size_t(127);
    const size_t tab_bytes = std::max(small_table, scene_table);
    int cus = 256;
    int caller_dev = -1;                                           // restored on exit (the caller's current device)
    (void)hipGetDevice(&caller_dev);
    {
        if (device >= 0) PK_TRY(hipSetDevice(device));
        hipDeviceProp_t prop;
        int cur = 0;
        PK_TRY(hipGetDevice(&cur));
        PK_TRY(hipGetDeviceProperties(&prop, cur));
        cus = std::max(1, prop.multiProcessorCount);
        PK_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        PK_TRY(hipEventCreate(&e0));
        PK_TRY(hipEventCreate(&e1));
        PK_TRY(hipMalloc(reinterpret_cast<void**>(&big), big_bytes));
        PK_TRY(hipMalloc(reinterpret_cast<void**>(&big2), big_bytes));
        PK_TRY(hipMalloc(reinterpret_cast<void**>(&tab), tab_bytes));
        PK_TRY(hipMalloc(reinterpret_cast<void**>(&sink), 64));
        PK_TRY(hipMemsetAsync(big, 0x3c, big_bytes, st));
        PK_TRY(hipMemsetAsync(big2, 0, big_bytes, st));
        PK_TRY(hipMemsetAsync(tab, 0x41, tab_bytes, st));
        auto best_ms = [&](auto launch, int reps) -> float {
            float best = 1e30f;
            launch();                                           // warm (and the caches, for the gather)
            for (int r = 0; r < reps; ++r) {
                if (hipEventRecord(e0, st) != hipSuccess) return -1.0f;
                launch();
                if (hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return -1.0f;
                float ms = 0;
                if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return -1.0f;
                best = std::min(best, ms);
            }
            return best;
        };
        const dim3 grid(cus * 8), blk(kBlk);
        float ms = 0;
        for (int wpc : {4, 8, 16, 32})             // best over the grid size and the copy variant (2 GiB divides
            for (int var = 0; var < 4; ++var) {     // every grid's 8 x threads)
                const dim3 cg(cus * wpc / 4);
                ms = best_ms([&] {
                    if (var == 0) hipLaunchKernelGGL((k_copy<4, true>), cg, blk, 0, st, big, big2, nbig);
                    else if (var == 1) hipLaunchKernelGGL((k_copy<4, false>), cg, blk, 0, st, big, big2, nbig);
                    else if (var == 2) hipLaunchKernelGGL((k_copy<8, true>), cg, blk, 0, st, big, big2, nbig);
                    else hipLaunchKernelGGL((k_copy<8, false>), cg, blk, 0, st, big, big2, nbig);
                }, 4);
                if (ms <= 0) { err = "peaks: copy timing failed"; goto done; }
                out->hbm_copy_gbps = std::max(out->hbm_copy_gbps, 2.0 * (double)big_bytes / (ms * 1e-3) / 1e9);
            }
        for (int wpc : {8, 16, 32}) {
            const dim3 rg(cus * wpc / 4);
            ms = best_ms([&] { hipLaunchKernelGGL(k_read, rg, blk, 0, st, big, nbig, sink); }, 4);
            if (ms <= 0) { err = "peaks: read timing failed"; goto done; }
            out->hbm_read_gbps = std::max(out->hbm_read_gbps, (double)big_bytes / (ms * 1e-3) / 1e9);
        }
        const int iters = 64;
        PK_TRY(hipMemcpyAsync(tab, big, tab_bytes, hipMemcpyDeviceToDevice, st));   // varied words (the walk's hash)
        for (int which = 0; which < 4; ++which) {
            const size_t tb = (which & 1) == 0 ? small_table : scene_table;
            const unsigned nlines = (unsigned)(tb / 128);
            double gbps = 0;
            if (which < 2) {           // the divergent walk shape, best of 8..20 waves per CU
                const int wsteps = 128;
                for (int wpc : {8, 12, 16, 20}) {
                    const dim3 wg(cus * wpc / 4);
                    ms = best_ms([&] { hipLaunchKernelGGL(k_walk, wg, blk, 0, st, tab, nlines, wsteps, sink); }, 3);
                    if (ms <= 0) { err = "peaks: walk timing failed"; goto done; }
                    gbps = std::max(gbps, (double)wg.x * kBlk * wsteps * 128.0 / (ms * 1e-3) / 1e9);
                }
            } else {                   // full-line fetches: 8 lanes per line
                for (int var = 0; var < 4; ++var) {     // 2 or 4 lines in flight per lane; 16 or 32 waves per CU
                    const dim3 gg(var & 2 ? cus * 4 : cus * 8);
                    const double gb = (double)gg.x * kBlk * iters * 128.0;
                    ms = best_ms([&] {
                        if (var & 1) hipLaunchKernelGGL((k_gather<4, true>), gg, blk, 0, st, tab, nlines, iters, 17u + which, sink);
                        else hipLaunchKernelGGL((k_gather<2, true>), gg, blk, 0, st, tab, nlines, iters, 17u + which, sink);
                    }, 4);
                    if (ms <= 0) { err = "peaks: gather timing failed"; goto done; }
                    gbps = std::max(gbps, gb / (ms * 1e-3) / 1e9);
                }
            }
            if (which == 0) { out->l2_gather_gbps = gbps; out->l2_table_bytes = (double)tb; }
            else if (which == 1) { out->scene_gather_gbps = gbps; out->scene_table_bytes = (double)tb; }
            else if (which == 2) out->l2_line_gbps = gbps;
            else out->scene_line_gbps = gbps;
        }
        PK_TRY(hipGetLastError());
    }
done:
    if (st) (void)hipStreamSynchronize(st);
    (void)hipFree(big); (void)hipFree(big2); (void)hipFree(tab); (void)hipFree(sink);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (caller_dev >= 0) (void)hipSetDevice(caller_dev);
    if (!err.empty()) return rt_internal_set_error(RT_ERR_HIP, err.c_str());
    return RT_OK;
}
