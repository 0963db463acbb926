// Microbenchmark: VALU issue throughput on one MI355X (gfx950) at full occupancy.
// Each lane runs N iterations of 16 independent ops (scalar fma, packed fma, cvt_f32_f16,
// v_max3, v_cndmask) over 8 waves per SIMD; reports device time and ops per SIMD per cycle
// (ops = wave64 instructions).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));
template <int K>
__global__ __launch_bounds__(256) void kbench(float* out, int iters, float a, float b) {
    float x[16];
    f2v y[8];
    for (int i = 0; i < 16; ++i) x[i] = threadIdx.x * 0.001f + i;
    for (int i = 0; i < 8; ++i) y[i] = f2v{x[2 * i], x[2 * i + 1]};
    unsigned u[16];
    for (int i = 0; i < 16; ++i) u[i] = threadIdx.x * 977u + i * 31u;
#pragma unroll 1
    for (int it = 0; it < iters; ++it) {
        if (K == 0) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaf(x[i], a, b);
        } else if (K == 1) {
            const f2v aa = {a, a}, bb = {b, b};
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = __builtin_elementwise_fma(y[i], aa, bb);
#pragma unroll
            for (int i = 0; i < 8; ++i) y[i] = __builtin_elementwise_fma(y[i], aa, bb);
        } else if (K == 2) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = x[i] + (float)__builtin_bit_cast(_Float16, (unsigned short)(u[i] + it));
        } else if (K == 3) {
#pragma unroll
            for (int i = 0; i < 16; ++i) x[i] = __builtin_fmaxf(__builtin_fmaxf(x[i], a), x[(i + 1) & 15]);
        } else if (K == 4) {
#pragma unroll
            for (int i = 0; i < 16; ++i) u[i] = (u[i] & 1u) ? u[i] * 3u : u[i] + 7u;
        }
    }
    float s = 0;
    for (int i = 0; i < 16; ++i) s += x[i] + (float)u[i];
    for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}
int main() {
    float* d;
    const int blocks = 256 * 8;    // 8 blocks of 256 per CU = 8 waves per SIMD
    hipMalloc(&d, blocks * 256 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;
    const char* names[] = {"v_fma_f32", "v_pk_fma_f32 (2 per 2 floats)", "cvt_f32_f16+add", "v_max3/max", "int select"};
    for (int k = 0; k < 5; ++k) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0, 0);
            if (k == 0) hipLaunchKernelGGL(kbench<0>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 0.5f);
            if (k == 1) hipLaunchKernelGGL(kbench<1>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 0.5f);
            if (k == 2) hipLaunchKernelGGL(kbench<2>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 0.5f);
            if (k == 3) hipLaunchKernelGGL(kbench<3>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 0.5f);
            if (k == 4) hipLaunchKernelGGL(kbench<4>, dim3(blocks), dim3(256), 0, 0, d, iters, 1.0001f, 0.5f);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // wave64 instructions per SIMD: (blocks*4 waves / 1024 SIMDs) * iters * 16 (k=1: 16 pk ops)
            const double insts = (double)blocks * 4 / 1024 * iters * 16;
            if (rep == 2) printf("%-32s %.3f ms  %.2f ns per wave-instruction per SIMD\n", names[k], ms, ms * 1e6 / insts);
        }
    }
    return 0;
}
