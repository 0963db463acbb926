// Multi-GPU rendering inside the C-ABI (rt_set_devices, include/rt/rt.h).
//
// the reference parallelises one frame over host threads
// with row-interleaved pixel rows (raytracer.cpp:352-383); here a frame is
// split over the N GPUs of one node as round-robin row stripes (stripe s ->
// device s mod N, the reference's interleave at stripe granularity), every
// device renders its stripes into a contiguous HBM slab on its own HIP
// stream, ONE RCCL ncclGather (rccl.h:745) over xGMI brings the N slabs to
// device 0, where rt_unshuffle_stripes restores row order before the D2H copy.
// The scene is read-only and small, so every device holds a full replica
// (rt_internal_replicate).  No other data moves between devices.
//
// RCCL is opened with dlopen on first use: single-GPU users never map the
// (large) library, and a missing librccl fails group creation loudly.
#include <dlfcn.h>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "rt/rt.h"
#include "rt_internal.hpp"

namespace {

int fail(int code, const std::string& msg) { return rt_internal_set_error(code, msg.c_str()); }

#define HIP_OK(expr)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorName(e_)); \
    } while (0)

struct Rccl {
    void* handle = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGather) gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.handle = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (r.handle) break;
        }
        if (!r.handle) {
            r.error = std::string("cannot load librccl: ") + dlerror();
            return;
        }
        auto sym = [&](auto& fn, const char* name) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(r.handle, name));
            if (!fn && r.error.empty()) r.error = std::string("librccl lacks ") + name;
        };
        sym(r.comm_init_all, "ncclCommInitAll");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.gather, "ncclGather");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
    });
    return r;
}

int nccl_fail(const char* what, ncclResult_t e) {
    const Rccl& r = rccl();
    return fail(RT_ERR_HIP, std::string(what) + ": " + (r.error_string ? r.error_string(e) : "RCCL error"));
}

// Device buffer grown on demand (the device's stream must be idle when it grows).
int grow(uint8_t** p, size_t* cap, size_t bytes) {
    if (*cap >= bytes) return RT_OK;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_OK(hipMalloc(reinterpret_cast<void**>(p), bytes));
    *cap = bytes;
    return RT_OK;
}

}  // namespace

struct rt_group {
    int n = 0;
    std::vector<rt_scene*> rep;          // rep[0]: the primary scene (not owned); rep[d]: replica on device d
    std::vector<ncclComm_t> comms;       // one communicator over the n devices, rank d on device d
    std::vector<hipStream_t> streams;    // one render + gather stream per device
    std::vector<uint8_t*> slabs;         // device d: its stripes, slab_rows * W * 3
    std::vector<size_t> slab_cap;
    uint8_t* gathered = nullptr;         // device 0: n slabs
    size_t gathered_cap = 0;
    uint8_t* image = nullptr;            // device 0: the assembled frame
    size_t image_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;   // device 0: kernel time of a group frame
    int stripe_rows = 8;                 // RT_GROUP_STRIPE

    ~rt_group() {
        for (int d = 0; d < n; ++d) {
            (void)hipSetDevice(d);
            if (d < (int)streams.size() && streams[d]) (void)hipStreamSynchronize(streams[d]);
            if (d < (int)slabs.size()) (void)hipFree(slabs[d]);
            if (d < (int)comms.size() && comms[d] && rccl().comm_destroy) rccl().comm_destroy(comms[d]);
            if (d < (int)streams.size() && streams[d]) (void)hipStreamDestroy(streams[d]);
        }
        (void)hipSetDevice(0);
        (void)hipFree(gathered);
        (void)hipFree(image);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        for (int d = 1; d < (int)rep.size(); ++d) rt_scene_destroy(rep[d]);
        (void)hipSetDevice(0);
    }
};

int rt_internal_group_size(const rt_group* g) { return g ? g->n : 1; }

int rt_internal_group_create(rt_scene* primary, int n, rt_group** out) {
    *out = nullptr;
    const Rccl& r = rccl();
    if (!r.error.empty()) return fail(RT_ERR_NO_DEVICE, "multi-GPU group: " + r.error);
    rt_group* g = new rt_group();
    g->n = n;
    g->rep.assign(n, nullptr);
    g->rep[0] = primary;
    g->comms.assign(n, nullptr);
    g->streams.assign(n, nullptr);
    g->slabs.assign(n, nullptr);
    g->slab_cap.assign(n, 0);
    if (const char* e = std::getenv("RT_GROUP_STRIPE")) g->stripe_rows = std::max(1, std::atoi(e));
    auto bail = [&](int rc) {
        g->rep[0] = nullptr;             // the primary is the caller's
        delete g;
        return rc;
    };
    for (int d = 1; d < n; ++d) {
        const int rc = rt_internal_replicate(primary, d, &g->rep[d]);
        if (rc) return bail(rc);
    }
    for (int d = 0; d < n; ++d) {
        if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&g->streams[d], hipStreamNonBlocking) != hipSuccess)
            return bail(fail(RT_ERR_HIP, "multi-GPU group: stream creation failed on device " + std::to_string(d)));
    }
    (void)hipSetDevice(0);
    if (hipEventCreate(&g->ev0) != hipSuccess || hipEventCreate(&g->ev1) != hipSuccess)
        return bail(fail(RT_ERR_HIP, "multi-GPU group: event creation failed"));
    std::vector<int> devs(n);
    for (int d = 0; d < n; ++d) devs[d] = d;
    const ncclResult_t e = r.comm_init_all(g->comms.data(), n, devs.data());
    if (e != ncclSuccess) {
        g->comms.assign(n, nullptr);
        return bail(nccl_fail("ncclCommInitAll", e));
    }
    (void)hipSetDevice(0);
    *out = g;
    return RT_OK;
}

void rt_internal_group_destroy(rt_group* g) {
    if (!g) return;
    g->rep[0] = nullptr;
    delete g;
}

int rt_internal_group_set_max_depth(rt_group* g, int depth) {
    for (int d = 1; d < g->n; ++d) {
        const int rc = rt_scene_set_max_depth(g->rep[d], depth);
        if (rc) return rc;
    }
    return RT_OK;
}

int rt_internal_group_render(rt_group* g, const rt_camera* cam, int aa, uint8_t* out_rgb, rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    const int n = g->n, W = cam->image_width, H = cam->image_height, S = g->stripe_rows;
    const int rows = rt_slab_rows(H, S, n);
    const size_t slab_bytes = (size_t)rows * W * 3, frame_bytes = (size_t)W * H * 3;
    const int flags = stats ? RT_RENDER_COUNT : 0;
    // buffers (every stream idle between group frames: each call ends synchronised)
    for (int d = 0; d < n; ++d) {
        HIP_OK(hipSetDevice(d));
        int rc = grow(&g->slabs[d], &g->slab_cap[d], slab_bytes);
        if (rc) return rc;
        if (stats && (rc = rt_counters_reset(g->rep[d], g->streams[d]))) return rc;
    }
    HIP_OK(hipSetDevice(0));
    int rc = grow(&g->gathered, &g->gathered_cap, slab_bytes * n);
    if (!rc) rc = grow(&g->image, &g->image_cap, frame_bytes);
    if (rc) return rc;
    HIP_OK(hipEventRecord(g->ev0, g->streams[0]));
    // every device renders its stripes (rank d of n), each on its own stream
    for (int d = 0; d < n; ++d) {
        rc = rt_render_device(g->rep[d], cam, aa, S, d, n, g->slabs[d], g->streams[d], flags);
        if (rc) return rc;
    }
    // one gather of the uint8 slabs to device 0 over xGMI
    const Rccl& r = rccl();
    ncclResult_t e = r.group_start();
    for (int d = 0; d < n && e == ncclSuccess; ++d)
        e = r.gather(g->slabs[d], d == 0 ? g->gathered : nullptr, slab_bytes, ncclUint8, 0, g->comms[d], g->streams[d]);
    const ncclResult_t e2 = r.group_end();
    if (e != ncclSuccess) return nccl_fail("ncclGather", e);
    if (e2 != ncclSuccess) return nccl_fail("ncclGroupEnd", e2);
    // device 0: slabs -> row order, then to the caller's buffer
    HIP_OK(hipSetDevice(0));
    rc = rt_unshuffle_stripes(g->gathered, g->image, W, H, S, n, g->streams[0]);
    if (rc) return rc;
    HIP_OK(hipEventRecord(g->ev1, g->streams[0]));
    HIP_OK(hipMemcpyAsync(out_rgb, g->image, frame_bytes, hipMemcpyDeviceToHost, g->streams[0]));
    for (int d = 0; d < n; ++d) {
        HIP_OK(hipSetDevice(d));
        HIP_OK(hipStreamSynchronize(g->streams[d]));
    }
    HIP_OK(hipSetDevice(0));
    // walks cut off by their step bound on any device (rt_scene_check), then the counters
    rt_stats sum{};
    for (int d = 0; d < n; ++d) {
        if (stats) {
            rt_stats one{};
            if ((rc = rt_counters_read(g->rep[d], &one))) return rc;
            sum.primary_rays += one.primary_rays; sum.shadow_rays += one.shadow_rays;
            sum.reflection_rays += one.reflection_rays; sum.node_visits += one.node_visits;
            sum.tri_tests += one.tri_tests; sum.sphere_tests += one.sphere_tests;
            sum.shadow_rays_skipped += one.shadow_rays_skipped;
        } else if ((rc = rt_scene_check(g->rep[d]))) {
            return rc;
        }
    }
    HIP_OK(hipSetDevice(0));
    if (stats) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, g->ev0, g->ev1));
        *stats = sum;
        stats->kernel_ms = ms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}
