// Microbenchmark: one dependent 128-B node fetch per lane per step (a BVH walk
// step), fetched (0) per lane -- eight dwordx4 loads, 64 distinct lines per wave
// instruction -- or (1) cooperatively: eight global_load_lds_dwordx4 in which the
// 8 lanes of each group load the 8 pieces of ONE lane's line (8 distinct lines
// per instruction) into a per-wave LDS image, then every lane reads its own line
// back (ds_read_b128).  VALU = dependent VALU ops per step (the step's compute).
//   hipcc --offload-arch=gfx950 -O3 -o ubench_coop ubench_coop.hip && ./ubench_coop
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ unsigned pick(unsigned h, unsigned n) { return (unsigned)(((unsigned long long)h * n) >> 32); }

template <int MODE, int VALU>
__global__ __launch_bounds__(256) void walk(const float4* __restrict__ tab, unsigned nlines, int steps, unsigned* sink) {
    __shared__ float4 img[4][64 * 8];                  // per wave: 64 lines x 8 pieces (8 KB)
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned line = pick(mix32(blockIdx.x * 256 + threadIdx.x), nlines);
    unsigned acc = 0;
    float x = 1.0f;
    for (int st = 0; st < steps; ++st) {
        float4 v[8];
        if (MODE == 0) {
            const float4* q = tab + (size_t)line * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = q[j];
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const unsigned owner_line = (unsigned)__shfl((int)line, (int)(8 * j + (lane >> 3)), 64);
                const float4* src = tab + (size_t)owner_line * 8 + (lane & 7);
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                                 reinterpret_cast<void*>(&img[wave][j * 64]), 16, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0x3f70);          // vmcnt(0) (gfx9 encoding: lgkm/exp untouched)
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = img[wave][lane * 8 + j];
        }
        unsigned h = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
            h ^= __float_as_uint(v[j].x) ^ __float_as_uint(v[j].y) ^ __float_as_uint(v[j].z) ^ __float_as_uint(v[j].w);
#pragma unroll
        for (int k = 0; k < VALU; ++k) x = x * 1.0001f + 0.5f;
        acc ^= h;
        line = pick(mix32(h ^ (unsigned)st ^ (threadIdx.x * 0x9e3779b1u) ^ (__float_as_uint(x) & 0u)), nlines);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc + (unsigned)x;
}

int main() {
    const size_t max_bytes = size_t(8) << 20;
    float4* tab;
    unsigned* sink;
    CHECK(hipMalloc(&tab, max_bytes));
    CHECK(hipMalloc(&sink, 64));
    {
        float4* h = (float4*)malloc(max_bytes);
        for (size_t i = 0; i < max_bytes / 16; ++i) h[i] = make_float4((float)(i * 7 % 1013), 1.0f, 2.0f, (float)(i % 17));
        CHECK(hipMemcpy(tab, h, max_bytes, hipMemcpyHostToDevice));
        free(h);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int steps = 256;
    for (size_t tb : {size_t(2) << 20, size_t(5) << 20}) {
        const unsigned nlines = (unsigned)(tb / 128);
        for (int wpc : {8, 12, 16, 20}) {
            const int blocks = cus * wpc / 4;
            for (int mode = 0; mode < 4; ++mode) {
                auto run = [&]() {
                    if (mode == 0) hipLaunchKernelGGL((walk<0, 0>), dim3(blocks), dim3(256), 0, 0, tab, nlines, steps, sink);
                    else if (mode == 1) hipLaunchKernelGGL((walk<1, 0>), dim3(blocks), dim3(256), 0, 0, tab, nlines, steps, sink);
                    else if (mode == 2) hipLaunchKernelGGL((walk<0, 100>), dim3(blocks), dim3(256), 0, 0, tab, nlines, steps, sink);
                    else hipLaunchKernelGGL((walk<1, 100>), dim3(blocks), dim3(256), 0, 0, tab, nlines, steps, sink);
                };
                run();
                CHECK(hipDeviceSynchronize());
                float best = 1e30f;
                for (int r = 0; r < 5; ++r) {
                    CHECK(hipEventRecord(e0));
                    run();
                    CHECK(hipEventRecord(e1));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    if (ms < best) best = ms;
                }
                const double bytes = (double)blocks * 256 * steps * 128.0;
                printf("{\"table_mb\": %.0f, \"waves_per_cu\": %d, \"mode\": \"%s\", \"valu\": %d, \"ms\": %.4f, \"TB_s\": %.2f, "
                       "\"ns_per_step\": %.1f}\n", tb / 1048576.0, wpc, (mode & 1) ? "coop-glds" : "per-lane",
                       mode >= 2 ? 100 : 0, best, bytes / (best * 1e-3) / 1e12, best * 1e6 / steps);
            }
        }
    }
    return 0;
}
