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
    bool virt = false;                   // RT_GROUP_VIRTUAL rehearsal: every rank on device 0, copies for the gather
    std::vector<rt_scene*> rep;          // rep[0]: the primary scene (not owned); rep[d]: replica of rank d
    std::vector<ncclComm_t> comms;       // one communicator over the n devices, rank d on device d
    std::vector<hipStream_t> streams;    // one render + gather stream per rank
    std::vector<hipEvent_t> joined;      // rank d's gather issued (device 0's stream waits on it)
    std::vector<uint8_t*> slabs;         // rank d: its stripes of every frame of a batch, frame-major
    std::vector<size_t> slab_cap;
    uint8_t* gathered = nullptr;         // device 0: [frame][rank] slabs
    size_t gathered_cap = 0;
    uint8_t* image = nullptr;            // device 0: the assembled frames
    size_t image_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;   // device 0: kernel time of a group call
    int stripe_rows = 4;                 // RT_GROUP_STRIPE (4: 5.5x at N = 8 in the rehearsal, 8: 5.0x)

    int dev(int d) const { return virt ? 0 : d; }

    ~rt_group() {
        for (int d = 0; d < n; ++d) {
            (void)hipSetDevice(dev(d));
            if (d < (int)streams.size() && streams[d]) (void)hipStreamSynchronize(streams[d]);
            if (d < (int)slabs.size()) (void)hipFree(slabs[d]);
            if (d < (int)comms.size() && comms[d] && rccl().comm_destroy) rccl().comm_destroy(comms[d]);
            if (d < (int)streams.size() && streams[d]) (void)hipStreamDestroy(streams[d]);
            if (d < (int)joined.size() && joined[d]) (void)hipEventDestroy(joined[d]);
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

bool rt_internal_group_virtual() {
    const char* e = std::getenv("RT_GROUP_VIRTUAL");
    return e && std::atoi(e) != 0;
}

int rt_internal_group_create(rt_scene* primary, int n, rt_group** out) {
    *out = nullptr;
    const bool virt = rt_internal_group_virtual();
    const Rccl& r = rccl();
    if (!virt && !r.error.empty()) return fail(RT_ERR_NO_DEVICE, "multi-GPU group: " + r.error);
    rt_group* g = new rt_group();
    g->n = n;
    g->virt = virt;
    g->rep.assign(n, nullptr);
    g->rep[0] = primary;
    g->comms.assign(n, nullptr);
    g->streams.assign(n, nullptr);
    g->joined.assign(n, nullptr);
    g->slabs.assign(n, nullptr);
    g->slab_cap.assign(n, 0);
    if (const char* e = std::getenv("RT_GROUP_STRIPE")) g->stripe_rows = std::max(1, std::atoi(e));
    auto bail = [&](int rc) {
        g->rep[0] = nullptr;             // the primary is the caller's
        delete g;
        return rc;
    };
    for (int d = 1; d < n; ++d) {
        const int rc = rt_internal_replicate(primary, g->dev(d), &g->rep[d]);
        if (rc) return bail(rc);
    }
    for (int d = 0; d < n; ++d) {
        if (hipSetDevice(g->dev(d)) != hipSuccess ||
            hipStreamCreateWithFlags(&g->streams[d], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&g->joined[d], hipEventDisableTiming) != hipSuccess)
            return bail(fail(RT_ERR_HIP, "multi-GPU group: stream creation failed for rank " + std::to_string(d)));
    }
    (void)hipSetDevice(0);
    if (hipEventCreate(&g->ev0) != hipSuccess || hipEventCreate(&g->ev1) != hipSuccess)
        return bail(fail(RT_ERR_HIP, "multi-GPU group: event creation failed"));
    if (!virt) {
        std::vector<int> devs(n);
        for (int d = 0; d < n; ++d) devs[d] = d;
        const ncclResult_t e = r.comm_init_all(g->comms.data(), n, devs.data());
        if (e != ncclSuccess) {
            g->comms.assign(n, nullptr);
            return bail(nccl_fail("ncclCommInitAll", e));
        }
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

// nf frames of one size on the group, in flight together: every rank renders its row stripes of all
// of them as one frame batch (rt_render_frames_device: one persistent grid walks the frames, so one
// frame's mirror-chain tail overlaps the others' bulk), ONE grouped RCCL call gathers every frame's
// slabs to device 0 (one ncclGather per frame inside ncclGroupStart/End), device 0 un-interleaves
// each frame and copies it to outs[f].  nf = 1 is rt_render's frame.
int rt_internal_group_render_frames(rt_group* g, const rt_camera* cams, int nf, int aa, uint8_t* const* outs,
                                    rt_stats* stats) {
    const auto t0 = std::chrono::steady_clock::now();
    const int n = g->n, W = cams[0].image_width, H = cams[0].image_height, S = g->stripe_rows;
    for (int f = 1; f < nf; ++f)
        if (cams[f].image_width != W || cams[f].image_height != H)
            return fail(RT_ERR_ARG, "internal: a group frame batch mixes image sizes");
    const int rows = rt_slab_rows(H, S, n);
    const size_t slab_bytes = (size_t)rows * W * 3, frame_bytes = (size_t)W * H * 3;
    const int flags = stats ? RT_RENDER_COUNT : 0;
    // buffers (every stream idle between group calls: each call ends synchronised)
    for (int d = 0; d < n; ++d) {
        HIP_OK(hipSetDevice(g->dev(d)));
        int rc = grow(&g->slabs[d], &g->slab_cap[d], slab_bytes * nf);
        if (rc) return rc;
        if (stats && (rc = rt_counters_reset(g->rep[d], g->streams[d]))) return rc;
    }
    HIP_OK(hipSetDevice(0));
    int rc = grow(&g->gathered, &g->gathered_cap, slab_bytes * n * nf);
    if (!rc) rc = grow(&g->image, &g->image_cap, frame_bytes * nf);
    if (rc) return rc;
    HIP_OK(hipEventRecord(g->ev0, g->streams[0]));
    // every rank renders its stripes of every frame (rank d of n), each on its own stream
    std::vector<void*> ptrs(nf);
    for (int d = 0; d < n; ++d) {
        for (int f = 0; f < nf; ++f) ptrs[f] = g->slabs[d] + f * slab_bytes;
        rc = nf == 1 ? rt_render_device(g->rep[d], cams, aa, S, d, n, ptrs[0], g->streams[d], flags)
                     : rt_render_frames_device(g->rep[d], cams, nf, aa, S, d, n, ptrs.data(), g->streams[d], flags);
        if (rc) return rc;
    }
    // the uint8 slabs of every frame to device 0 over xGMI: one grouped RCCL call
    if (g->virt) {               // rehearsal: the ranks share device 0, plain copies stand in for RCCL
        for (int d = 0; d < n; ++d)
            for (int f = 0; f < nf; ++f)
                HIP_OK(hipMemcpyAsync(g->gathered + ((size_t)f * n + d) * slab_bytes, g->slabs[d] + f * slab_bytes,
                                      slab_bytes, hipMemcpyDeviceToDevice, g->streams[d]));
    } else {
        const Rccl& r = rccl();
        ncclResult_t e = r.group_start();
        for (int f = 0; f < nf && e == ncclSuccess; ++f)
            for (int d = 0; d < n && e == ncclSuccess; ++d)
                e = r.gather(g->slabs[d] + f * slab_bytes, d == 0 ? g->gathered + (size_t)f * n * slab_bytes : nullptr,
                             slab_bytes, ncclUint8, 0, g->comms[d], g->streams[d]);
        const ncclResult_t e2 = r.group_end();
        if (e != ncclSuccess) return nccl_fail("ncclGather", e);
        if (e2 != ncclSuccess) return nccl_fail("ncclGroupEnd", e2);
    }
    for (int d = 1; d < n; ++d) {
        HIP_OK(hipSetDevice(g->dev(d)));
        HIP_OK(hipEventRecord(g->joined[d], g->streams[d]));
        HIP_OK(hipSetDevice(0));
        HIP_OK(hipStreamWaitEvent(g->streams[0], g->joined[d], 0));
    }
    // device 0: slabs -> row order, then to the caller's buffers
    HIP_OK(hipSetDevice(0));
    for (int f = 0; f < nf; ++f) {
        rc = rt_unshuffle_stripes(g->gathered + (size_t)f * n * slab_bytes, g->image + f * frame_bytes, W, H, S, n,
                                  g->streams[0]);
        if (rc) return rc;
    }
    HIP_OK(hipEventRecord(g->ev1, g->streams[0]));
    for (int f = 0; f < nf; ++f)
        HIP_OK(hipMemcpyAsync(outs[f], g->image + f * frame_bytes, frame_bytes, hipMemcpyDeviceToHost, g->streams[0]));
    for (int d = 0; d < n; ++d) {
        HIP_OK(hipSetDevice(g->dev(d)));
        HIP_OK(hipStreamSynchronize(g->streams[d]));
    }
    HIP_OK(hipSetDevice(0));
    // walks cut off by their step bound on any rank (rt_scene_check), then the counters
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

int rt_internal_group_render(rt_group* g, const rt_camera* cam, int aa, uint8_t* out_rgb, rt_stats* stats) {
    uint8_t* outs[1] = {out_rgb};
    return rt_internal_group_render_frames(g, cam, 1, aa, outs, stats);
}
