// Microbenchmark: dependent 64-B record chase over an L2-resident table
// (the memory pattern of one BVH walk step), to separate memory latency
// from instruction count.  Build: hipcc --offload-arch=gfx950 -O3 -o ubench_chase ubench_chase.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int VALU, int NLD>
__global__ __launch_bounds__(256) void chase(const float4* __restrict__ tab, int n, int steps, int* out) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    int i = (int)(((long long)tid * 7919) % n);
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
        const float4* q = tab + 4 * (size_t)i;
        const float4 a = q[0];
        const float4 b = NLD > 1 ? q[1] : a, c = NLD > 2 ? q[2] : a, d = NLD > 3 ? q[3] : a;
        float x = a.x + b.y + c.z + d.x;
#pragma unroll
        for (int k = 0; k < VALU; ++k) x = x * 1.0001f + 0.5f;   // dependent VALU chain
        acc += x;
        i = (__float_as_int(a.w) ^ (__float_as_int(x) & 0)) % n;   // next index from the record
    }
    if (acc == 12345.0f) out[0] = i;
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 25000;          // records (64 B each)
    const int steps = 200;
    std::vector<float> h(16 * (size_t)n);
    srand(1);
    for (int r = 0; r < n; ++r) {
        for (int k = 0; k < 16; ++k) h[16 * r + k] = 1.0f + (rand() % 100) * 0.01f;
        int nx = rand() % n;
        std::memcpy(&h[16 * r + 3], &nx, 4);
    }
    float4* d;
    int* out;
    CHECK(hipMalloc(&d, h.size() * 4));
    CHECK(hipMalloc(&out, 4));
    CHECK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int cus = 256;
    printf("{\"table_bytes\": %zu, \"steps\": %d}\n", h.size() * 4, steps);
    for (int wpc : {1, 4, 8, 16, 32}) {          // waves per CU
        for (int valu : {0, 1, 2, 4}) {   // 0: 4 loads, else valu = loads per step, no VALU chain
            const int blocks = cus * wpc / 4;               // 4 waves per 256-thread block
            auto run = [&]() {
                if (valu == 0) hipLaunchKernelGGL((chase<64, 4>), dim3(blocks), dim3(256), 0, 0, d, n, steps, out);
                else if (valu == 1) hipLaunchKernelGGL((chase<0, 1>), dim3(blocks), dim3(256), 0, 0, d, n, steps, out);
                else if (valu == 2) hipLaunchKernelGGL((chase<0, 2>), dim3(blocks), dim3(256), 0, 0, d, n, steps, out);
                else hipLaunchKernelGGL((chase<0, 4>), dim3(blocks), dim3(256), 0, 0, d, n, steps, out);
            };
            if (blocks < 1) continue;
            run();
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            for (int r = 0; r < 5; ++r) run();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ms /= 5;
            const double lane_steps = (double)blocks * 256 * steps;
            printf("{\"waves_per_cu\": %d, \"valu_chain\": %d, \"ms\": %.4f, \"ns_per_step_per_wave\": %.1f, "
                   "\"G_lane_steps_per_s\": %.2f}\n",
                   wpc, valu, ms, ms * 1e6 / steps, lane_steps / (ms * 1e-3) / 1e9);
        }
    }
    return 0;
}
