// Experiment (CLI start-up): the HIP runtime's start-up steps in a fresh process, ms on the steady
// clock from main.  tools/exp_hipinit.sh runs it under environment variants (device visibility,
// hardware queues), each several times.
//   hipcc -O2 tools/exp_hipinit.cpp -o tools/_ref_hipinit   (any arch: no kernels)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const double t0 = now_ms();
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    const double t1 = now_ms();
    (void)hipSetDevice(0);
    (void)hipFree(nullptr);
    const double t2 = now_ms();
    void* p = nullptr;
    (void)hipMalloc(&p, 1 << 20);
    (void)hipMemset(p, 0, 1 << 20);
    (void)hipDeviceSynchronize();
    const double t3 = now_ms();
    (void)hipFree(p);
    const char* rv = std::getenv("ROCR_VISIBLE_DEVICES");
    const char* hv = std::getenv("HIP_VISIBLE_DEVICES");
    std::printf("{\"devices\": %d, \"err\": %d, \"device_count_ms\": %.2f, \"context_ms\": %.2f, \"first_op_ms\": %.2f, "
                "\"ROCR_VISIBLE_DEVICES\": \"%s\", \"HIP_VISIBLE_DEVICES\": \"%s\"}\n",
                n, (int)e, t1 - t0, t2 - t1, t3 - t2, rv ? rv : "", hv ? hv : "");
    std::fflush(stdout);
    std::_Exit(0);
}
