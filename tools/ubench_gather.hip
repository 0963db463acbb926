// Microbenchmark: gathers of random 128-B lines from a shared table (the BVH
// walks' fetch shape), per-lane lines vs lines shared by 8 lanes, to see what
// bounds a divergent node fetch (the texture-address path processes the
// distinct lines of each wave instruction).
//   hipcc --offload-arch=gfx950 -O3 -o ubench_gather ubench_gather.hip && ./ubench_gather
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ unsigned pick(unsigned h, unsigned n) { return (unsigned)(((unsigned long long)h * n) >> 32); }

// MODE 0: every lane its own random line, NLD dwordx4 loads of it (a divergent wide-node fetch)
// MODE 1: lanes 8j..8j+7 share one random line, lane l loads 16-B piece l%8 (a cooperative fetch:
//         8 distinct lines per wave instruction instead of 64); NLD loads = NLD different lines
template <int MODE, int NLD, int UNROLL>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ tab, unsigned nlines, int iters, unsigned* sink) {
    const unsigned gtid = blockIdx.x * 256 + threadIdx.x;
    const unsigned lane = threadIdx.x & 63;
    unsigned acc = 0;
    for (int it = 0; it < iters; it += UNROLL) {
        float4 v[UNROLL][NLD];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            if (MODE == 0) {
                const unsigned line = pick(mix32(gtid * 0x9e3779b1u + (unsigned)(it + u) * 0x85ebca6bu), nlines);
                const float4* q = tab + (size_t)line * 8;
#pragma unroll
                for (int j = 0; j < NLD; ++j) v[u][j] = q[j];
            } else {
#pragma unroll
                for (int j = 0; j < NLD; ++j) {
                    const unsigned owner = (gtid & ~63u) + ((lane >> 3) + 8u * (unsigned)j) % 64u;
                    const unsigned line = pick(mix32(owner * 0x9e3779b1u + (unsigned)(it + u) * 0x85ebca6bu), nlines);
                    v[u][j] = tab[(size_t)line * 8 + (lane & 7)];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
#pragma unroll
            for (int j = 0; j < NLD; ++j)
                acc ^= __float_as_uint(v[u][j].x) ^ __float_as_uint(v[u][j].y) ^ __float_as_uint(v[u][j].z) ^
                       __float_as_uint(v[u][j].w);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main() {
    const size_t max_bytes = size_t(64) << 20;
    float4* tab;
    unsigned* sink;
    CHECK(hipMalloc(&tab, max_bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(tab, 0x41, max_bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int iters = 64;
    for (size_t tb : {size_t(2) << 20, size_t(5) << 20, size_t(32) << 20}) {
        const unsigned nlines = (unsigned)(tb / 128);
        for (int wpc : {8, 16, 32}) {
            const int blocks = cus * wpc / 4;
            auto run = [&](int mode) {
                if (mode == 0) hipLaunchKernelGGL((gather<0, 8, 2>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, sink);
                else if (mode == 1) hipLaunchKernelGGL((gather<1, 8, 2>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, sink);
                else hipLaunchKernelGGL((gather<0, 4, 4>), dim3(blocks), dim3(256), 0, 0, tab, nlines, iters, sink);
            };
            for (int mode = 0; mode < 3; ++mode) {
                run(mode);
                CHECK(hipDeviceSynchronize());
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    CHECK(hipEventRecord(e0));
                    run(mode);
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    if (ms < best) best = ms;
                }
                const double lines_per_lane = mode == 2 ? 0.5 : 1.0;    // mode 2 reads half lines (64 B)
                const double bytes = (double)blocks * 256 * iters * 128.0 * lines_per_lane;
                printf("{\"table_mb\": %.0f, \"waves_per_cu\": %d, \"mode\": \"%s\", \"ms\": %.4f, \"TB_s\": %.2f}\n",
                       tb / 1048576.0, wpc, mode == 0 ? "per-lane 128B" : (mode == 1 ? "8 lanes/line 128B" : "per-lane 64B"),
                       best, bytes / (best * 1e-3) / 1e12);
            }
        }
    }
    return 0;
}
