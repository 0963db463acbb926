// Microbenchmark: cost of a wave's 64-B record fetch (4 x dwordx4) as a
// function of how many DISTINCT records the 64 lanes touch (D = 1..64), from
// an L2-resident table, at 8 waves/CU.  Dependent chain per lane (each step's
// record gives the next index), so this is the traversal access pattern.
// Also: the same from an LDS-resident table (ds_read_b128).
// Build: hipcc --offload-arch=gfx950 -O3 -o ubench_div ubench_div.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// Lane group g = lane / (64 / D) follows its own chain; lanes of a group share addresses.
__global__ __launch_bounds__(256) void chase_g(const float4* __restrict__ tab, int n, int steps, int D, int* out) {
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int grp = lane / (64 / D);
    int i = (int)(((long long)(wave * 64 + grp) * 7919) % n);
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
        const float4* q = tab + 4 * (size_t)i;
        const float4 a = q[0], b = q[1], c = q[2], d = q[3];
        acc += a.x + b.y + c.z + d.x;
        i = __float_as_int(a.w) % n;
    }
    if (acc == 12345.0f) out[0] = i;
}

__global__ __launch_bounds__(256) void chase_lds(const float4* __restrict__ tab, int n, int steps, int D, int* out) {
    __shared__ float4 t[4 * 1024];     // 64 KiB: 1024 records
    for (int k = threadIdx.x; k < 4 * 1024; k += 256) t[k] = tab[k];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int grp = lane / (64 / D);
    int i = (int)(((long long)(wave * 64 + grp) * 7919) % 1024);
    float acc = 0.0f;
    for (int s = 0; s < steps; ++s) {
        const float4 a = t[4 * i], b = t[4 * i + 1], c = t[4 * i + 2], d = t[4 * i + 3];
        acc += a.x + b.y + c.z + d.x;
        i = (__float_as_int(a.w) % n) & 1023;
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
    const int cus = 256;
    printf("{\"table_bytes\": %zu, \"steps\": %d}\n", h.size() * 4, steps);
    for (int lds = 0; lds < 2; ++lds)
        for (int wpc : {1, 8}) {
            for (int D : {1, 2, 4, 8, 16, 32, 64}) {
                const int blocks = cus * wpc / 4;
                auto run = [&]() {
                    if (lds) hipLaunchKernelGGL(chase_lds, dim3(blocks), dim3(256), 0, 0, d, n, steps, D, out);
                    else hipLaunchKernelGGL(chase_g, dim3(blocks), dim3(256), 0, 0, d, n, steps, D, out);
                };
                run();
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(e0));
                for (int r = 0; r < 5; ++r) run();
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                ms /= 5;
                const double wave_steps = (double)blocks * 4 * steps;
                printf("{\"lds\": %d, \"waves_per_cu\": %d, \"distinct\": %d, \"ns_per_step\": %.1f, "
                       "\"cycles_per_wave_step_per_cu\": %.1f}\n",
                       lds, wpc, D, ms * 1e6 / steps, ms * 1e-3 * 2.4e9 / (wave_steps / cus));
            }
        }
    return 0;
}
