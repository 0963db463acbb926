// C-ABI implementation (include/rt/rt.h): scene lifetime, upload, render
// entry points, host utilities.  No exceptions cross the ABI.
#include "rt/rt.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <mutex>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "host_scene.hpp"
#include "render_kernels.hpp"
#include "pathchain.hpp"
#include "rt_internal.hpp"

// phase-B workgroups per CU x 4 in frame batches (a compile-time setting for same-box A/B builds)
#ifndef RT_GB_BATCH_Q4
#define RT_GB_BATCH_Q4 6
#endif

namespace {

thread_local std::string g_err;
std::atomic<int> g_devices{0};          // rt_set_devices: device group of scenes created afterwards (0: none)

// RT_DEBUG: diagnostics and measurement modes, one bit mask (read when used, so a caller may change it between
// scenes): 0x01 log the start-up phases (tools/exp_cli.py --phases), 0x02 log workspace growths, 0x04 log each
// frame batch's submission and GPU span (makes batched calls synchronous), 0x08 no device warm-up thread,
// 0x10 per-kernel times of chain launches (scenes created with it: rt_kernel_times), 0x20 production-fetch
// counting passes (scenes created with it count the bytes the timed walks fetch: bench.py roofline).
enum : int { kDbgLogInit = 1, kDbgLogAlloc = 2, kDbgLogSubmit = 4, kDbgNoWarmup = 8, kDbgKtime = 16, kDbgCountProd = 32 };
int debug_flags() {
    const char* e = std::getenv("RT_DEBUG");
    return e ? (int)std::strtol(e, nullptr, 0) : 0;
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(RT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorName(e_) + " (" + \
                                        hipGetErrorString(e_) + ")");                         \
    } while (0)

// theta = (float)(acos(c) * 180 / 3.1415); specular iff theta <= 90.01
// (raytracer.cpp:411-412).  Each step is monotone in c, so the predicate is
// exactly "c >= threshold" on [-1, 1] (NaN outside).  The threshold is found
// with glibc's correctly rounded acos, making the device test bit-exact with
// the reference without a device acos.
bool theta_ok(float c) {
    const float theta = (float)(std::acos((double)c) * 180 / 3.1415);
    return theta <= 90.01;
}

int32_t ordered(float f) {
    int32_t i;
    std::memcpy(&i, &f, 4);
    return i < 0 ? (int32_t)(0x80000000u - (uint32_t)i) : i;   // -0 and +0 -> 0
}

float from_ordered(int32_t o) {
    int32_t i = o < 0 ? (int32_t)(0x80000000u - (uint32_t)o) : o;
    float f;
    std::memcpy(&f, &i, 4);
    return f;
}

float cos_threshold() {
    int32_t lo = ordered(-1.0f), hi = ordered(1.0f);   // theta_ok(lo) false, theta_ok(hi) true
    while (hi - lo > 1) {
        const int32_t mid = lo + (hi - lo) / 2;
        if (theta_ok(from_ordered(mid))) hi = mid; else lo = mid;
    }
    return from_ordered(hi);
}

}  // namespace

int rt_internal_set_error(int code, const char* msg) { return fail(code, msg); }

struct rt_scene {
    rtx::HostScene host;
    rtx::FlatBVH bvh;
    int device = 0;
    bool host_only = false;
    int opt_flags = 0;                         // rt_options.flags at creation (replicas use the same)
    rt_group* group = nullptr;                 // multi-GPU (rt_set_devices): replicas + RCCL comm, rt_multi.cpp
    rtk::DevScene dev{};
    dl::Node* d_nodes = nullptr;
    dl::Prim* d_prims = nullptr;
    dl::TriShade* d_tri = nullptr;
    dl::Material* d_mats = nullptr;
    dl::Light* d_lights = nullptr;
    char* d_block = nullptr;                   // the flat arrays above and the two below (upload_flat)
    char* d_block2 = nullptr;                  // the wide trees and the occlusion pairs (upload_rest)
    unsigned long long* d_counters = nullptr;
    unsigned* d_err = nullptr;                 // device error word (DevScene.err)
    unsigned* h_err = nullptr;                 // pinned host copy of it (rt_render reads it with the frame)
    uint8_t* d_out = nullptr;
    size_t out_cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    dl::Pair* d_pairs = nullptr;
    dl::Pair* d_spairs = nullptr;
    dl::Wide* d_swnodes = nullptr;
    dl::Wide* d_wnodes = nullptr;
    dl::Vec4* d_lrec = nullptr;
    dl::LeafBig* d_leafbig = nullptr;
    int num_cus = 256;
    int chain_grid = 0, occl_grid = 0, mix_grid = 0;   // resident-sized persistent grids (lazily queried)
    // Scheduling constants (the measured defaults of DESIGN.md §7; the knobs that varied them were removed in
    // round 6 with the settings measured slower).  Task chunks: tasks c*ch .. c*ch+ch-1 go to workgroup c mod G
    // -- continuations in chunks of 128 in frame batches, one at a time in a lone frame (its clustered mirror
    // chains spread over every workgroup: a lone frame 1.36 -> 1.15 ms), shadow tasks in chunks of 256 in
    // frame batches and 128 in lone frames (0.8826 -> 0.8776 ms, profiles/r05_lone_knobs.txt).
    static constexpr int kKinline = 1;           // deepest level of phase A
    // samples per chain-path launch at most (bigger launches leave fewer tails per sample: C3 batches 4 M 0.72,
    // 8 M 0.66, 16 M 0.63, 32 M 0.59 ms/frame); the workspace budget usually binds first
    static constexpr size_t kChunkSamples = size_t(32) << 20;
    static constexpr int kContDen = 6;           // phase-B records for at least cap / 6 continuations (C3: ~9 %)
    int tune_orefill = 32;      // RT_OREFILL (tests: the leaf-queue walker's refill threshold)
    int tune_lq_wait = 32;      // RT_LQ_WAIT (tests: the leaf-queue flush threshold)
    long long tune_batch_samples = 1ll << 21;   // RT_BATCH_SAMPLES: a multi-frame call's batches hold at least ~this
                                                // many samples each (fewer batches than slots for small frames)
    int tune_slots = 3;         // RT_SLOTS: frame batches in flight together (workspace slots, <= kSlots;
                                // default GPU_MAX_HW_QUEUES - 1)
    int tune_bq_cap = 1 << 30;  // RT_BQ_CAP: phase-B shadow queue slots (tests force the k_occlude spill path)
    int tune_hot_units = 1;     // RT_HOT_UNITS: lone frames deal phase-A units heaviest-first by the previous frame's steps
    int tune_deep = 5;          // RT_DEEP: PcParams::deep_min (frame batches' deep-first deal; 0: off)
    int tune_mix = 5 | 1 << 8;  // RT_MIX: PcParams::mix_cls: lone frames deal the units of >= 64 steps (classes
                                // 0-4) in pairs with light ones, half of each wave's first lanes (C3 one frame
                                // 0.876 -> 0.837 ms; 16 of 64 lanes the same, 8 of 64 +-0; profiles/r06_mix_*.jsonl)
    int tune_compact = 3;       // RT_COMPACT: phase-A records without directions (16 B instead of 32): 1 frame batches,
                                // 2 every launch, 0 none, 3 (round 5) frame batches only where full records would leave
                                // fewer than 4 frames per launch (full_records_fit; C3 AA1 20-frame calls 0.4151 -> 0.4040
                                // ms/frame with full records, 96-frame calls -0.4 %; profiles/r05_ab_compact.txt)
    // RT_WS_BUDGET_MB: HBM for the scene on its device -- the uploaded scene, the host-output staging (its
    // live size, at least a 64 MB reserve), and the chain-path workspace arenas of all slots together, each
    // slot's arena (headroom included) within an even share of the rest.  A launch's arena is sized for the worst case (every
    // sample recording every level), so the budget bounds the samples per launch (and the frames per frame
    // batch).  A lone frame's arena follows the frame (chain_launch_units), not the share.
    size_t ws_budget = size_t(16) << 30;
    int tune_cont_cb = 0;       // RT_CONT_CB (tests): exactly this many (k_fallback finishes the rest)
    int tune_fbs_cap = 0;       // RT_FBS_CAP (tests): k_fallback shadow-queue slots (0: one per sample)
    size_t scene_bytes = 0;     // device bytes of the uploaded scene (trees, primitives, tables)
    bool ktime = false;         // RT_DEBUG 0x10: per-kernel times of chain launches (rt_kernel_times; syncs each launch)
    double kt_ms[rtc::kKKinds] = {};
    long long kt_launches = 0;
    rtc::KTimer kt;
    static constexpr size_t kStagingReserve = size_t(64) << 20;
    size_t slot_budget() const {
        // the scene, and the host-output staging (rt_render's frame, rt_render_cameras' frames) at its live
        // size or the reserve, whichever is larger; fit_arenas drops an arena a staging growth leaves over
        const size_t fixed = scene_bytes + std::max(kStagingReserve, out_cap + batch_out_cap);
        const size_t arenas = ws_budget > 2 * fixed ? ws_budget - fixed : ws_budget / 2;
        // (1 % of each share for the slot's side tables beside its arena: the deep-first deal's depth table,
        // 1 B per sample of a launch, and the lone frame's unit tables, 16 B per 256 samples -- an arena
        // holds well over 100 B per sample)
        return arenas / (size_t)std::max(1, std::min(tune_slots, kSlots)) / 101 * 100;
    }
    double xml_ms = 0, prep_ms = 0, upload_ms = 0;   // scene creation phases (rt_scene_bvh_info)
    bool warned_budget = false;    // one row unit alone exceeds the slot budget (chain_launch_units): told once
    std::string trace_file;     // RT_TRACE: dump per-sample wall-clock timings after each render (diagnostics)
    unsigned* d_trace = nullptr;
    size_t trace_cap = 0;
    // chain-path workspaces: one device arena per concurrent-frame slot (grown
    // on demand, carved per frame); slot 0 serves single renders, slots
    // [0, kSlots) the concurrent frames of rt_render_cameras*.
    static constexpr int kSlots = 6;
    // An arena may be used from any caller stream: `last` is recorded after each
    // use on `last_stream`, and a use from another stream first waits on it.
    struct Arena {
        char* p = nullptr;
        size_t bytes = 0;
        hipEvent_t last = nullptr;
        hipStream_t last_stream = nullptr;
        // lone frames' phase-A unit order (PcParams::ucost / uorder): ucost, uorder, ucol, ugrp, hist_units each
        unsigned* hist = nullptr;
        unsigned hist_units = 0;
        uint64_t hist_key = 0;               // the launch geometry uorder was ranked for (0: none yet)
        // frame batches' deep-first deal (PcParams::pdepth): the levels of the previous frame's chains per frame slot
        uint8_t* pdepth = nullptr;
        size_t pdepth_n = 0;
        uint64_t pdepth_key = 0;
    } arenas[kSlots];
    // continuation share of frame batches (phase B's record space, cb): each batched launch copies its
    // continuation count (k_pack_a's or k_mix's total) to pinned memory behind it; once that copy is done the share
    // is folded into cont_frac, which sizes the next launches' cb (and so their frames per launch)
    double cont_frac = 0;                      // 0: none seen yet (cap / kContDen)
    unsigned* h_cont = nullptr;                // pinned, per slot
    unsigned* d_cont_peak = nullptr;           // a frame of several chunks: its chunks' most continuations
    hipEvent_t cont_ev[kSlots] = {};
    size_t cont_cap[kSlots] = {};
    bool cont_pending[kSlots] = {};
    hipStream_t slot_stream[kSlots] = {};
    hipEvent_t slot_done[kSlots] = {};
    hipEvent_t fork_ev = nullptr;
    uint8_t* batch_out = nullptr;              // device frames of rt_render_cameras (host outputs)
    size_t batch_out_cap = 0;
    float* dbg_t = nullptr;                    // rt_primary_hits_production: the level-0 hit dump (PcParams::dbg_t)
    int* dbg_m = nullptr;

    ~rt_scene() {
        if (group) rt_internal_group_destroy(group);
        for (int i = 0; i < kSlots; ++i) {
            (void)hipFree(arenas[i].p);
            if (arenas[i].last) (void)hipEventDestroy(arenas[i].last);
            if (slot_stream[i]) (void)hipStreamDestroy(slot_stream[i]);
            if (slot_done[i]) (void)hipEventDestroy(slot_done[i]);
        }
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        for (int i = 0; i < rtc::KTimer::kMax; ++i) {
            if (kt.ev0[i]) (void)hipEventDestroy(kt.ev0[i]);
            if (kt.ev1[i]) (void)hipEventDestroy(kt.ev1[i]);
        }
        for (auto& a : arenas) (void)hipFree(a.hist);
        for (auto& a : arenas) (void)hipFree(a.pdepth);
        for (auto& e : cont_ev)
            if (e) (void)hipEventDestroy(e);
        if (h_cont) (void)hipHostFree(h_cont);
        (void)hipFree(d_cont_peak);
        (void)hipFree(batch_out);
        (void)hipFree(d_block);           // the scene arrays, counters and error word (upload_flat / _rest)
        (void)hipFree(d_block2);
        (void)hipFree(d_out); (void)hipFree(d_trace);
        if (h_err) (void)hipHostFree(h_err);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
    }
};

namespace {

int select_device(const rt_options* opts, int* dev) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
    if (opts && opts->device >= 0) {
        if (opts->device >= n) return fail(RT_ERR_ARG, "device ordinal out of range");
        HIP_TRY(hipSetDevice(opts->device));
    }
    HIP_TRY(hipGetDevice(dev));
    return RT_OK;
}

int upload_scene(rt_scene* s, const rt_options* opts);

// The process's first scene: HIP's runtime and device initialisation (~0.25 s on the GPU box: runtime,
// device context, the kernels' code objects) runs on a helper thread while this thread reads the XML
// and builds the trees on the host, and is joined before the upload (a drop-in caller's first frame no
// longer pays both in sequence).  RT_DEBUG 0x08 disables it (A/B).
std::mutex g_warm_mu;
std::future<void> g_warm, g_warm2;
bool g_warm_started = false;

// Only for an explicit device (opts->device >= 0) or a device group (whose primary is device 0): -1
// means the calling thread's current device, which a helper thread cannot know without initialising HIP
// on the caller's thread first (a one-process-per-GPU caller passing -1 got an extra context
// and code-object load on GPU 0 in every rank).
void start_device_warmup(const rt_options* opts) {
    if ((opts && (opts->flags & RT_OPT_HOST_ONLY)) || (debug_flags() & kDbgNoWarmup)) return;
    const int want = g_devices.load() >= 1 ? 0 : (opts ? opts->device : -1);
    if (want < 0) return;
    std::lock_guard<std::mutex> lk(g_warm_mu);
    if (g_warm_started) return;
    g_warm_started = true;
    g_warm = std::async(std::launch::async, [want] {
        // RT_DEBUG 0x01 (tools/exp_cli.py --phases): the warm-up's steps on the steady clock, ms
        const bool log = (debug_flags() & kDbgLogInit) != 0;
        auto now = [] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        const double t0 = log ? now() : 0.0;
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0 || want >= n) return;
        const double t1 = log ? now() : 0.0;
        (void)hipSetDevice(want);
        (void)hipFree(nullptr);
        const double t2 = log ? now() : 0.0;
        // what only the first render needs goes on a second thread, joined once the scene is uploaded
        // (join_device_warmup_full): the kernels' code objects, and a pageable read-back (a drop-in frame's
        // first copy back otherwise paid ~9 ms of staging set-up, tools/exp_cli.py --phases)
        g_warm2 = std::async(std::launch::async, [want, log, now] {
            (void)hipSetDevice(want);
            int a = 0, b = 0, c = 0;
            (void)rtc::chain_occupancy(&a, &b, &c);
            const double t3 = log ? now() : 0.0;
            const size_t wb = 1u << 20;
            void* d = nullptr;
            std::vector<unsigned char> h(wb);
            if (hipMalloc(&d, wb) == hipSuccess) {
                (void)hipMemset(d, 0, wb);
                (void)hipMemcpy(h.data(), d, wb, hipMemcpyDeviceToHost);
                (void)hipFree(d);
            }
            if (log) std::fprintf(stderr, "{\"rt_init2\": {\"code_objects\": %.3f, \"readback\": %.3f}}\n", t3, now());
        });
        // the scene upload's needs: the process's first allocation, copy and fill (~20 ms on the box)
        void* d = nullptr;
        unsigned char h[256] = {};
        if (hipMalloc(&d, 4096) == hipSuccess) {
            (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
            (void)hipMemset(d, 0, 4096);
            (void)hipStreamSynchronize(nullptr);
            (void)hipFree(d);
        }
        if (log)
            std::fprintf(stderr, "{\"rt_init\": {\"start\": %.3f, \"device_count\": %.3f, \"context\": %.3f, \"first_op\": %.3f}}\n",
                         t0, t1, t2, now());
    });
}

void join_device_warmup() {
    std::lock_guard<std::mutex> lk(g_warm_mu);
    if (g_warm.valid()) g_warm.get();
}
void join_device_warmup_full() {
    join_device_warmup();
    std::lock_guard<std::mutex> lk(g_warm_mu);
    if (g_warm2.valid()) g_warm2.get();
}

double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int upload_flat(rt_scene* s);
int upload_rest(rt_scene* s, const rt_options* opts);

int finish_scene(rt_scene* s, const rt_options* opts) {
    auto t = std::chrono::steady_clock::now();
    rtx::prepare_triangles(s->host);
    s->prep_ms = ms_since(t);
    s->host_only = opts && (opts->flags & RT_OPT_HOST_ONLY);
    s->opt_flags = opts ? opts->flags : 0;
    const int ndev = g_devices.load();
    rt_options o = opts ? *opts : rt_options{0, 0, 0};
    if (ndev >= 1) o.device = 0;          // device group: the primary on device 0, replicas on 1..n-1
    // the arrays final after the flatten go to the device while the wide trees are still being built
    // (their own thread, which also joins the HIP warm-up): an explicit device only, since -1 means the
    // calling thread's current device
    std::future<int> early;
    bool started = false;
    std::function<void()> on_flat = [&] {
        started = true;
        early = std::async(std::launch::async, [s, o]() -> int {
            join_device_warmup();
            const int rc = select_device(&o, &s->device);
            return rc ? rc : upload_flat(s);
        });
    };
    std::string err = rtx::build_bvh(s->host, s->bvh, opts ? opts->build_threads : 0,
                                     !s->host_only && o.device >= 0 ? &on_flat : nullptr);
    t = std::chrono::steady_clock::now();
    int rc = early.valid() ? early.get() : RT_OK;
    if (!err.empty()) return fail(RT_ERR_LIMIT, err);
    if (s->host_only || rc) return rc;
    if (!started) {
        join_device_warmup();
        if ((rc = select_device(&o, &s->device)) || (rc = upload_flat(s))) return rc;
    } else {
        HIP_TRY(hipSetDevice(s->device));    // (the early upload set it on its own thread)
    }
    rc = upload_rest(s, &o);
    join_device_warmup_full();
    if (!rc && ndev >= 1) rc = rt_internal_group_create(s, ndev, &s->group);
    s->upload_ms = ms_since(t);              // (the part after the build: the early upload overlaps it)
    return rc;
}

// Device copies of scene arrays in one fresh allocation: 256-B aligned parts, each at least one element,
// then `zero` bytes zeroed; returns the zeroed region's offset in *zero_at.
struct UpPart { void** dst; const void* src; size_t bytes, min; };
template <class T, class V>
UpPart up_part(T** dst, const V& v) {
    return UpPart{reinterpret_cast<void**>(dst), v.data(), v.size() * sizeof(v[0]), sizeof(v[0])};
}
int upload_parts(char** block, const UpPart* parts, int n, size_t zero, size_t* zero_at, size_t* bytes) {
    auto up = [](size_t b) { return (b + 255) & ~size_t(255); };
    size_t off = 0;
    *bytes = 0;
    for (int i = 0; i < n; ++i) {
        off += up(std::max(parts[i].bytes, parts[i].min));
        *bytes += parts[i].bytes;
    }
    if (zero_at) *zero_at = off;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(block), std::max<size_t>(off + zero, 1)));
    off = 0;
    for (int i = 0; i < n; ++i) {
        *parts[i].dst = *block + off;
        if (parts[i].bytes) HIP_TRY(hipMemcpy(*parts[i].dst, parts[i].src, parts[i].bytes, hipMemcpyHostToDevice));
        off += up(std::max(parts[i].bytes, parts[i].min));
    }
    if (zero) HIP_TRY(hipMemset(*block + off, 0, zero));
    return RT_OK;
}

// Device copies of a built scene (s->host, s->bvh) on opts->device, plus the
// per-scene tuning knobs.
int upload_scene(rt_scene* s, const rt_options* opts) {
    int rc = select_device(opts, &s->device);
    if (!rc) rc = upload_flat(s);
    return rc ? rc : upload_rest(s, opts);
}

// The arrays final once the flatten is done (the reference tree, its prims, pairs and leaf records, the
// shading tables), the counters and the error word; on the current device.
int upload_flat(rt_scene* s) {
    std::vector<dl::Material> mats(s->host.materials.size());
    for (size_t i = 0; i < mats.size(); ++i) {
        const rtx::MaterialRec& m = s->host.materials[i];
        const rtx::V3& ia = s->host.ambient;
        dl::Material& o = mats[i];
        o.kax = m.ambient.x * ia.x; o.kay = m.ambient.y * ia.y; o.kaz = m.ambient.z * ia.z;  // :394
        o.phong = m.phong;
        o.kdx = m.diffuse.x; o.kdy = m.diffuse.y; o.kdz = m.diffuse.z; o.is_mirror = m.is_mirror ? 1 : 0;
        o.ksx = m.specular.x; o.ksy = m.specular.y; o.ksz = m.specular.z; o.pad0 = 0;
        o.kmx = m.mirror.x; o.kmy = m.mirror.y; o.kmz = m.mirror.z; o.pad1 = 0;
    }
    std::vector<dl::Light> lights(s->host.lights.size());
    for (size_t i = 0; i < lights.size(); ++i) {
        const rtx::LightRec& l = s->host.lights[i];
        lights[i] = dl::Light{l.position.x, l.position.y, l.position.z, 0, l.intensity.x, l.intensity.y,
                              l.intensity.z, 0};
    }
    const UpPart parts[] = {up_part(&s->d_nodes, s->bvh.nodes), up_part(&s->d_prims, s->bvh.prims),
                            up_part(&s->d_tri, s->bvh.tri_shade), up_part(&s->d_mats, mats),
                            up_part(&s->d_lights, lights), up_part(&s->d_pairs, s->bvh.pairs),
                            up_part(&s->d_leafbig, s->bvh.leaf_big), up_part(&s->d_lrec, s->bvh.lrec)};
    const size_t cbytes = (rtc::kCounters * sizeof(unsigned long long) + 255) & ~size_t(255);
    size_t zat = 0, bytes = 0;
    if (const int rc = upload_parts(&s->d_block, parts, 8, cbytes + 256, &zat, &bytes)) return rc;
    s->d_counters = reinterpret_cast<unsigned long long*>(s->d_block + zat);
    s->d_err = reinterpret_cast<unsigned*>(s->d_block + zat + cbytes);
    s->scene_bytes = bytes;
    return RT_OK;
}

// The wide trees and the occlusion tree's pairs (the build's last results), events, grids and knobs.
int upload_rest(rt_scene* s, const rt_options* opts) {
    {
        const UpPart parts[] = {up_part(&s->d_spairs, s->bvh.spairs), up_part(&s->d_swnodes, s->bvh.swnodes),
                                up_part(&s->d_wnodes, s->bvh.wnodes)};
        size_t bytes = 0;
        if (const int rc = upload_parts(&s->d_block2, parts, 3, 0, nullptr, &bytes)) return rc;
        s->scene_bytes += bytes;
    }
    HIP_TRY(hipEventCreate(&s->ev0));
    HIP_TRY(hipEventCreate(&s->ev1));

    {
        int cus = 0;
        HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device));
        s->num_cus = std::max(1, cus);
    }
    if (const char* e = std::getenv("RT_OREFILL")) s->tune_orefill = std::max(0, std::min(63, std::atoi(e)));
    if (const char* e = std::getenv("RT_LQ_WAIT")) s->tune_lq_wait = std::max(1, std::min(64, std::atoi(e)));
    if (const char* e = std::getenv("RT_BATCH_SAMPLES")) s->tune_batch_samples = std::max(1ll, std::atoll(e));
    // frame batches in flight: one HIP stream each beside the caller's; HIP multiplexes streams beyond
    // GPU_MAX_HW_QUEUES hardware queues (4 by default) onto the same queues, which serialises them
    // (C3: 4 slots on 4 queues 0.60 ms/frame, on 8 queues 0.51)
    {
        const char* q = std::getenv("GPU_MAX_HW_QUEUES");
        const int hwq = q ? std::atoi(q) : 4;
        s->tune_slots = std::max(1, std::min(rt_scene::kSlots, (hwq > 0 ? hwq : 4) - 1));
    }
    if (const char* e = std::getenv("RT_SLOTS")) s->tune_slots = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("RT_BQ_CAP")) s->tune_bq_cap = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("RT_COMPACT")) s->tune_compact = std::max(0, std::min(3, std::atoi(e)));
    if (const char* e = std::getenv("RT_HOT_UNITS")) s->tune_hot_units = std::atoi(e) != 0;
    if (const char* e = std::getenv("RT_MIX")) s->tune_mix = std::atoi(e);
    if (const char* e = std::getenv("RT_DEEP")) s->tune_deep = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("RT_TRACE")) s->trace_file = e;
    const int dbg = debug_flags();
    s->ktime = (dbg & kDbgKtime) != 0;
    if (const char* e = std::getenv("RT_CONT_CB")) s->tune_cont_cb = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("RT_FBS_CAP")) s->tune_fbs_cap = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("RT_WS_BUDGET_MB"))
        s->ws_budget = std::max<size_t>(64, std::strtoull(e, nullptr, 10)) << 20;

    rtk::DevScene& d = s->dev;
    d.nodes = s->d_nodes; d.prims = s->d_prims; d.tri_shade = s->d_tri; d.mats = s->d_mats; d.lights = s->d_lights;
    d.nnodes = (int)s->bvh.nodes.size();
    d.nlights = (int)s->host.lights.size();
    d.nmats = (int)s->host.materials.size();
    d.max_depth = s->host.max_depth;
    d.stack_entries = std::max(2, s->bvh.max_stack);
    d.eps = s->host.eps;
    d.bgx = (float)s->host.bg[0]; d.bgy = (float)s->host.bg[1]; d.bgz = (float)s->host.bg[2];
    d.cos_thr = cos_threshold();
    d.pairs = s->d_pairs;
    d.leaf_big = s->d_leafbig;
    for (int i = 0; i < 3; ++i) {
        d.root_lo[i] = s->bvh.root_lo[i];
        d.root_hi[i] = s->bvh.root_hi[i];
    }
    d.root_info = s->bvh.root_info;
    d.spairs = s->d_spairs;
    for (int i = 0; i < 3; ++i) {
        d.sroot_lo[i] = s->bvh.sroot_lo[i];
        d.sroot_hi[i] = s->bvh.sroot_hi[i];
    }
    d.sroot_info = s->bvh.sroot_info;
    d.swnodes = s->d_swnodes;
    d.lrec = reinterpret_cast<const float4*>(s->d_lrec);
    d.swroot = s->bvh.swroot;
    // occlusion tree for NaN-free shadow rays: 2 = 4-wide quantized form, 1 = binary, 0 = off (RT_STREE)
    d.use_stree = !s->bvh.swnodes.empty() ? 2 : (s->bvh.spairs.empty() ? 0 : 1);
    // closest-hit walks of NaN-free rays: the reference tree's wide form, reference order (tests, RT_WIDE_WALK=0:
    // the binary forms of both trees, every walk in k_fallback)
    d.wnodes = s->d_wnodes;
    d.wroot = s->bvh.wroot;
    d.use_wide = !s->bvh.nodes.empty() && !s->bvh.lrec.empty() &&
                 (!s->bvh.wnodes.empty() || (s->bvh.root_info < 0 && s->bvh.root_lrec >= 0));
    if (const char* e = std::getenv("RT_WIDE_WALK"); e && std::atoi(e) == 0) {
        d.use_wide = 0;
        d.use_stree = s->bvh.spairs.empty() ? 0 : 1;
    }
    d.err = s->d_err;
    {   // walk_runaway: 64 x (every node of the largest tree + leaves); RT_WALK_CAP overrides (tests)
        const long long nodes = (long long)s->bvh.pairs.size() + s->bvh.leaves + 64;   // the largest tree
        d.walk_cap = (int)std::min<long long>(INT32_MAX / 2, 64 * nodes);
        if (const char* e = std::getenv("RT_WALK_CAP")) d.walk_cap = std::max(1, std::atoi(e));
    }
    // spin_over: 2^24 iterations of a wait that sees no progress (with s_sleep ~0.5 s, far beyond the
    // longest legitimate wait: one walk of at most nodes + leaves steps); RT_SPIN_CAP overrides (tests)
    d.spin_cap = 1 << 24;
    if (const char* e = std::getenv("RT_SPIN_CAP")) d.spin_cap = std::max(0, std::atoi(e));   // 0: every wait gives up
    d.leaf_wait = 24;   // measured: 0 1.20, 8 1.19, 16-32 1.166, 48 1.22, 64 1.46 ms (C3; round 6 at HEAD: 0 / 16 +4 / +3 %)
    d.leaf_wait_any = d.leaf_wait;
    // shadow rays of lights behind the surface add +-0 when kd is finite (pathchain.hip light_needed)
    d.cull_shadows = 1;
    for (const auto& m : s->host.materials)
        if (!std::isfinite(m.diffuse.x) || !std::isfinite(m.diffuse.y) || !std::isfinite(m.diffuse.z)) d.cull_shadows = 0;
    if (const char* e = std::getenv("RT_CULL")) d.cull_shadows = d.cull_shadows && std::atoi(e) != 0;
    if (const char* e = std::getenv("RT_FORCE_FALLBACK")) d.force_fb = std::atoi(e);
    // measurement (RT_DEBUG 0x20): counting passes walk the production trees and count fetched bytes (bench.py)
    d.count_prod = (dbg & kDbgCountProd) ? 1 : 0;
    return RT_OK;
}

// EyeRayGenerator::init (raytracer.cpp:292-314) for the internal resolution.
rtk::Eye make_eye(const rt_camera& c, int nx, int ny) {
    using rtx::V3;
    const V3 e{c.position.x, c.position.y, c.position.z};
    const V3 w{-c.gaze.x, -c.gaze.y, -c.gaze.z};
    const float dist = c.near_distance;
    const float l = c.near_plane[0], r = c.near_plane[1], b = c.near_plane[2], t = c.near_plane[3];
    const V3 v{c.up.x, c.up.y, c.up.z};
    const V3 u{v.y * w.z - v.z * w.y, v.z * w.x - v.x * w.z, v.x * w.y - v.y * w.x};   // v x w
    const V3 mw{-w.x, -w.y, -w.z};
    const V3 m{e.x + mw.x * dist, e.y + mw.y * dist, e.z + mw.z * dist};
    const V3 q1{m.x + u.x * l, m.y + u.y * l, m.z + u.z * l};
    const V3 q{q1.x + v.x * t, q1.y + v.y * t, q1.z + v.z * t};
    rtk::Eye g;
    g.qx = q.x; g.qy = q.y; g.qz = q.z;
    g.ux = u.x; g.uy = u.y; g.uz = u.z;
    g.vx = v.x; g.vy = v.y; g.vz = v.z;
    g.ex = e.x; g.ey = e.y; g.ez = e.z;
    g.su = (r - l) / (float)nx;
    g.sv = (t - b) / (float)ny;
    return g;
}

int check_camera(const rt_camera* cam, int aa) {
    if (!cam) return fail(RT_ERR_ARG, "camera is NULL");
    if (aa < 1 || aa > 64) return fail(RT_ERR_ARG, "aa_factor must be in [1, 64]");
    if (cam->image_width < 1 || cam->image_height < 1) return fail(RT_ERR_ARG, "empty image");
    const long long iw = (long long)cam->image_width * aa, ih = (long long)cam->image_height * aa;
    if (iw > (1 << 24) || ih > (1 << 24)) return fail(RT_ERR_ARG, "internal resolution too large");
    return RT_OK;
}


// RT_TRACE diagnostics: a device buffer of n u32 and, after the frame, a raw
// dump {magic, path, a, b, n, payload...} (see tools/trace_report.py).
unsigned* trace_buffer(rt_scene* s, size_t n) {
    if (s->trace_file.empty()) return nullptr;
    if (!rtc::kTraceBuild) {
        std::fprintf(stderr, "librt_hip: RT_TRACE needs a build with RT_TRACE_BUILD=1 (make EXTRA=-DRT_TRACE_BUILD=1)\n");
        s->trace_file.clear();
        return nullptr;
    }
    if (s->trace_cap < n) {
        (void)hipFree(s->d_trace);
        s->d_trace = nullptr;
        s->trace_cap = 0;
        if (hipMalloc(reinterpret_cast<void**>(&s->d_trace), n * sizeof(unsigned)) != hipSuccess) return nullptr;
        s->trace_cap = n;
    }
    (void)hipMemset(s->d_trace, 0, n * sizeof(unsigned));
    return s->d_trace;
}

void trace_dump(rt_scene* s, hipStream_t st, unsigned path, unsigned a, unsigned b, size_t n) {
    if (s->trace_file.empty() || !s->d_trace) return;
    std::vector<unsigned> h(n);
    if (hipStreamSynchronize(st) != hipSuccess ||
        hipMemcpy(h.data(), s->d_trace, n * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess)
        return;
    if (FILE* f = std::fopen(s->trace_file.c_str(), "wb")) {
        const unsigned hdr[5] = {0x52545452u, path, a, b, (unsigned)n};
        std::fwrite(hdr, sizeof(unsigned), 5, f);
        std::fwrite(h.data(), sizeof(unsigned), n, f);
        std::fclose(f);
    }
}

// Chain path: chunks of whole 8*aa-row groups, workspace sized for the worst
// case (every sample recording every level) so no queue can overflow; the
// arenas of all slots together stay within the scene's workspace budget
// (rt_scene::ws_budget, RT_WS_BUDGET_MB).

// Bump layout of the chain-path workspace (one device arena, grown on demand).
struct ArenaLayout {
    size_t off = 0;
    template <typename T>
    size_t take(size_t n) {                   // returns the byte offset of n T's, 256-B aligned
        const size_t o = off;
        off += (std::max<size_t>(n, 1) * sizeof(T) + 255) & ~size_t(255);
        return o;
    }
};

// Sizes of one chain-path launch of `units` row units (phase split, queue capacities, grids).
struct ChainPlan {
    size_t cap = 0;                 // samples of the launch
    int G = 1, gb = 0, levels_a = 1, kinline = 0;
    bool phase_b = false, split_occ = false;
    bool rlists = false;   // a whole lone frame in one launch: phase A's lists read in their regions (no k_pack_a)
    unsigned dyn_units = 0, scapA = 0, ccapA = 0, scapB = 0;
    int la = 1, tchunk = 1;         // levels stored per sample; phase-B continuation chunk
    size_t cb = 0;                  // continuations with phase-B records
    // arena offsets
    size_t dbase = 0;               // records below it without directions (pathchain.hpp)
    int clevels = 0;
    size_t o_rec = 0, o_recd = 0, o_pinfo = 0, o_occ = 0, o_sqA = 0, o_scntA = 0, o_sflatA = 0, o_cq = 0, o_ccnt = 0,
           o_cflat = 0, o_ccntd = 0, o_sqB = 0, o_scntB = 0, o_sflatB = 0, o_totals = 0, o_cid = 0, o_tail = 0,
           o_fbc = 0, o_fbs = 0, bytes = 0;
};

// Geometry of one chain-path launch series (a frame, or a frame batch stacked as one slab).
struct ChainGeom {
    int levels, nl, wi, tiles_x, li, unit, nframes;
    size_t unit_samples, units_total;
};
ChainGeom chain_geom(const rt_scene* s, const rtk::FrameParams& f) {
    ChainGeom g;
    g.levels = std::max(s->dev.max_depth, 0) + 1;
    g.nl = std::max(s->dev.nlights, 1);
    g.wi = f.width * f.aa;
    g.tiles_x = (g.wi + 7) / 8;
    g.li = f.slab_rows * f.aa;
    g.unit = 8 * f.aa;
    g.unit_samples = (size_t)g.tiles_x * f.aa * 64;
    g.units_total = (size_t)(g.li + g.unit - 1) / g.unit;
    g.nframes = std::max(1, f.nframes);
    return g;
}

// The kernels' grids from their occupancy (once per scene).
int ensure_chain_grids(rt_scene* s) {
    if (s->chain_grid != 0) return RT_OK;
    int cb = 0, mb = 0, ob = 0;
    HIP_TRY(rtc::chain_occupancy(&cb, &mb, &ob));
    s->chain_grid = std::min(rtc::kMaxChainGrid, std::max(1, cb) * s->num_cus);
    s->mix_grid = std::max(1, mb) * s->num_cus;
    s->occl_grid = std::max(1, ob) * s->num_cus;
    return RT_OK;
}

// Every size of a launch of `nunits` row units, and its arena layout: worst-case queue sizing (every
// sample recording every level), so no queue can overflow.  (ensure_chain_grids first.)
ChainPlan chain_plan(const rt_scene* s, const ChainGeom& g, size_t nunits, bool count, size_t cb_want = 0,
                     int cmp_mode = -1, bool use_share = true);

// RT_COMPACT=3 (the default): frame batches keep full 32-B phase-A records where a 4-frame launch of this
// frame size fits the slot's workspace share with them (C3 AA1: faster, §7 round 5), and compact 16-B ones
// where it does not (C3 AA2: 1.83 -> 1.53 ms/frame with compact records: more frames per launch).  Decided
// with the default phase-B record space (not the measured continuation share, which moves as read-backs
// arrive): one frame geometry always gets the same record size, so a timed call never switches it and
// reallocates a workspace.
bool full_records_fit(const rt_scene* s, const ChainGeom& g) {
    ChainGeom g4 = g;
    g4.nframes = 4;
    const size_t per_frame = (g.units_total + (size_t)g.nframes - 1) / (size_t)g.nframes;
    return chain_plan(s, g4, 4 * per_frame, false, 0, 0, false).bytes <= s->slot_budget();
}

ChainPlan chain_plan(const rt_scene* s, const ChainGeom& g, size_t nunits, bool count, size_t cb_want, int cmp_mode,
                     bool use_share) {
    const int levels = g.levels, nl = g.nl;
    const int max_grid = s->chain_grid;
    ChainPlan P;
    P.cap = nunits * g.unit_samples;
    const size_t cap = P.cap;
    P.G = std::max(1, std::min(max_grid, (int)((std::min<size_t>(cap, INT32_MAX) + 255) / 256)));
    // phase split: A walks levels [0, kinline], B the rest (k_mix chain role, gb workgroups)
    P.kinline = rt_scene::kKinline;
    P.phase_b = P.kinline < s->dev.max_depth;
    // phase-B workgroups: a lone frame's deep chains are its critical path (1.875 per CU best since
    // round 3: C3 one frame, 61-frame medians, 1.5625 0.946-0.948, 1.72 0.940, 1.875 0.925-0.935,
    // 2.03 0.956 ms);
    // in frame batches other frames hide them and the shadow role wants the CUs (C3: 0.5 per CU
    // 0.550 ms/frame, 0.75 0.552, 1 0.554, 1.25 0.557, 1.5625 0.568)
    // frame batches: A's shadow rays in their own 5-wave k_occlude launch (split_occ) and (round 3) 1 phase-B
    // workgroup per CU (6 slots in flight: 0.504-0.512 -> 0.495 ms/frame; 0.5 per CU 0.500, 2 0.4995)
    P.split_occ = g.nframes > 1;
    // a whole lone frame in one launch reads phase A's lists where k_chain left them (no packing kernel between
    // its phases: C3 -10 us); the chunks of a larger frame keep k_pack_a (C5: region lists +2.5-4 % per frame,
    // profiles/r06_nopack_ab.jsonl)
    P.rlists = g.nframes <= 1 && nunits >= g.units_total;
    // (round 5, the driver's 20-frame call on 5 slots: 1.5 per CU 0.4175 against 1 per CU 0.4282 ms/frame, three
    // interleaved same-box rounds, 96-frame calls +-0; profiles/r05_ab_gb.txt)
    const int gb_default = g.nframes > 1 ? RT_GB_BATCH_Q4 * s->num_cus / 4 : 30 * s->num_cus / 16;
    P.gb = P.phase_b ? std::max(1, std::min(s->mix_grid - 1, gb_default)) : 0;
    P.levels_a = std::min(P.kinline, std::max(s->dev.max_depth, 0)) + 1;
    // dynamic phase-A units: a workgroup may take up to twice its static share (at most
    // rtc::kDynUnits), and its queues are sized for that
    const unsigned share = rtc::chain_block_units((int)std::min<size_t>(cap, INT32_MAX), P.G);
    P.dyn_units = share <= (unsigned)rtc::kDynUnits ? std::min(2u * share, (unsigned)rtc::kDynUnits) : 0u;
    const unsigned units_a = P.dyn_units ? P.dyn_units : share;
    P.scapA = units_a * 256u * (unsigned)(P.levels_a * nl);
    P.ccapA = units_a * 256u;
    // records: levels [0, la) for every sample; deeper ones (phase B) for the first cb continuations
    // (the rest finish in k_fallback; counting passes keep every one: cb = cap)
    P.la = !P.phase_b ? levels : P.levels_a;
    // (at least cap / kContDen, more once frame batches report a larger continuation share: that share + 10 %)
    const size_t cb_guess = std::max(cap / (size_t)rt_scene::kContDen,
                                     use_share ? (size_t)((double)cap * std::min(1.0, s->cont_frac * 1.1 + 0.005)) : 0);
    P.cb = P.la >= levels ? 0 : (count ? cap : std::min(cap, std::max(cb_guess, std::min<size_t>(cap, 65536))));
    if (cb_want > 0 && !count && P.la < levels) P.cb = std::min(cap, std::max(P.cb, cb_want));
    if (s->tune_cont_cb > 0 && !count && P.la < levels) P.cb = std::min(cap, (size_t)s->tune_cont_cb);
    P.tchunk = g.nframes > 1 ? 128 : 1;
    {   // a phase-B workgroup's continuations: at most ceil(chunks / gb) chunks of tchunk (chunk_count)
        const size_t ch = (size_t)P.tchunk, nch = (P.cb + ch - 1) / ch;
        const size_t per_wg = P.gb > 0 ? (nch + P.gb - 1) / P.gb * ch : 0;
        P.scapB = P.phase_b ? (unsigned)(per_wg * (size_t)(levels - P.la) * nl) : 0u;
    }
    const size_t nrec = cap * P.la + P.cb * (levels - P.la);
    ArenaLayout L;
    // phase A's records without their directions where k_finish can rebuild them (pathchain.hpp dbase)
    // (RT_COMPACT=1 frame batches, 2 everywhere, 0 nowhere, 3 frame batches whose 4-frame launches would not fit
    // with full records (full_records_fit): the rebuilt directions cost k_finish more than the saved bytes gain
    // k_chain and k_occlude, unless the bytes buy frames per launch)
    const bool cmp = cmp_mode >= 0 ? cmp_mode != 0
                                   : s->tune_compact == 2 || (s->tune_compact == 1 && g.nframes > 1) ||
                                         (s->tune_compact == 3 && g.nframes > 1 && !full_records_fit(s, g));
    P.clevels = cmp ? std::min(P.la, rtc::kCompactLevels) : 0;
    P.dbase = cap * (size_t)P.clevels;
    P.o_rec = L.take<float4>(nrec);
    P.o_recd = L.take<float4>(nrec - P.dbase);
    P.o_pinfo = L.take<int>(cap);
    P.o_occ = L.take<uint8_t>(nrec * nl + 8);   // + 8: k_finish reads aligned dwords
    P.o_cid = L.take<unsigned>(cap);
    P.o_tail = L.take<float4>(cap);
    P.o_fbc = L.take<unsigned>(cap);
    P.o_fbs = L.take<unsigned>(cap);
    {
        P.o_sqA = L.take<unsigned>((size_t)P.G * P.scapA); P.o_scntA = L.take<unsigned>(P.G);
        if (!P.split_occ && !P.rlists) P.o_sflatA = L.take<unsigned>(cap * P.levels_a * nl);   // packed (k_pack_a)
        P.o_cq = L.take<unsigned>((size_t)P.G * P.ccapA); P.o_ccnt = L.take<unsigned>(P.G);
        if (P.split_occ) P.o_ccntd = L.take<unsigned>(P.G);   // deep-first continuations (PcParams::ccntd)
        P.o_cflat = L.take<unsigned>(cap);   // packed continuations (k_pack_a; a lone frame's k_mix / k_fallback)
        P.o_sqB = L.take<unsigned>((size_t)P.gb * P.scapB); P.o_scntB = L.take<unsigned>(P.gb + 1);
        P.o_sflatB = L.take<unsigned>(P.cb * (levels - P.la) * nl);
    }
    P.o_totals = L.take<unsigned>(rtc::kTotalsWords);
    P.bytes = L.off;
    return P;
}

// Row units of one launch: as many as the chunk target (kChunkSamples), the u32 task ids and the
// slot's share of the workspace budget (RT_WS_BUDGET_MB over the slots) allow -- the largest count
// whose chain_plan arena fits the budget (at least one unit, whatever its size).
size_t chain_launch_units(rt_scene* s, const ChainGeom& g, bool count, size_t* cb_out = nullptr) {
    const size_t id_limit = (size_t)(INT32_MAX - 1) / ((size_t)g.levels * g.nl);   // u32 task owner ids (pathchain.hpp)
    size_t units = std::min(g.units_total, std::max<size_t>(1, std::min(rt_scene::kChunkSamples, id_limit) / g.unit_samples));
    const size_t budget = s->slot_budget();
    if (chain_plan(s, g, units, count).bytes > budget) {
        size_t lo = 1, hi = units;                 // largest units in [1, units] whose arena fits the budget
        while (lo < hi) {
            const size_t mid = lo + (hi - lo + 1) / 2;
            if (chain_plan(s, g, mid, count).bytes <= budget) lo = mid; else hi = mid - 1;
        }
        units = lo;
        if (units == 1 && chain_plan(s, g, 1, count).bytes > budget && !s->warned_budget) {
            s->warned_budget = true;
            std::fprintf(stderr, "librt_hip: one row unit (%zu samples) needs a %.1f MB workspace, over the slot's "
                                 "%.1f MB share of RT_WS_BUDGET_MB; allocating it anyway\n",
                         g.unit_samples, chain_plan(s, g, 1, count).bytes / 1e6, budget / 1e6);
        }
    }
    if (cb_out) {
        // phase-B record space: cap/6 continuations by default (C3 continues ~9 % of its samples); the
        // rest of the slot's budget then raises it, up to every sample, so a mirror-heavy frame
        // (marbles: 60 % continue) keeps its deep chains in phase B instead of k_fallback's serial
        // whole-path walks.  Bytes grow linearly with cb.
        const ChainPlan P = chain_plan(s, g, units, count);
        *cb_out = P.cb;
        if (!count && P.la < g.levels && P.cb < P.cap && P.bytes < budget) {
            const ChainPlan F = chain_plan(s, g, units, count, P.cap);
            if (F.bytes <= budget) {
                *cb_out = P.cap;
            } else {
                const double per = (double)(F.bytes - P.bytes) / (double)(F.cb - P.cb);
                const size_t extra = (size_t)((double)(budget - P.bytes) / per * 0.98);
                *cb_out = std::min(P.cap, P.cb + extra);
                while (*cb_out > P.cb && chain_plan(s, g, units, count, *cb_out).bytes > budget)
                    *cb_out = P.cb + (*cb_out - P.cb) / 2;
            }
        }
    }
    return units;
}

// Fold the continuation-share read-backs that are done (wait: wait for them) into s->cont_frac: the
// largest recent share, decaying.
void poll_cont(rt_scene* s, bool wait) {
    for (int k = 0; k < rt_scene::kSlots; ++k) {
        if (!s->cont_pending[k]) continue;
        if (wait) (void)hipEventSynchronize(s->cont_ev[k]);
        if (hipEventQuery(s->cont_ev[k]) != hipSuccess) continue;
        s->cont_pending[k] = false;
        const double f = s->cont_cap[k] ? (double)s->h_cont[k] / (double)s->cont_cap[k] : 0.0;
        s->cont_frac = std::max(f, s->cont_frac * 0.75);
    }
}

// A launch's continuation count (k_pack_a's or k_mix's total, or a frame's chunk peak) copied to pinned memory behind
// it on `st`; poll_cont folds it into the scene's continuation share once the copy is done.
int read_back_cont(rt_scene* s, hipStream_t st, int slot, const unsigned* src, size_t cap) {
    if (!s->h_cont) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->h_cont), rt_scene::kSlots * sizeof(unsigned)));
    if (!s->cont_ev[slot]) HIP_TRY(hipEventCreateWithFlags(&s->cont_ev[slot], hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(&s->h_cont[slot], src, sizeof(unsigned), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipEventRecord(s->cont_ev[slot], st));
    s->cont_cap[slot] = cap;
    s->cont_pending[slot] = true;
    return RT_OK;
}

int render_chain(rt_scene* s, const rtk::Eye& eye, const rtk::FrameParams& f, bool count, hipStream_t st,
                 int slot = 0) {
    rt_scene::Arena& arena = s->arenas[slot];
    const ChainGeom g = chain_geom(s, f);
    const int levels = g.levels, nl = g.nl, wi = g.wi, tiles_x = g.tiles_x, li = g.li, unit = g.unit;
    if (const int rc = ensure_chain_grids(s)) return rc;
    const int max_grid = s->chain_grid;
    auto grid_for = [&](int n0) { return std::max(1, std::min(max_grid, (n0 + 255) / 256)); };
    size_t cb = 0;
    // read-backs of earlier frames' chunks (C5-sized lone frames); never for a frame batch: its frame count
    // was fitted to one launch with the share its caller (render_cameras) polled, and a larger share
    // here would split the batch into chunks forked over every slot, from inside one slot's stream
    if (f.chunk_k == 1 && f.nframes <= 1) poll_cont(s, false);
    const size_t units = chain_launch_units(s, g, count, &cb);
    const ChainPlan P = chain_plan(s, g, units, count, cb);
    const int chunk_rows = (int)units * unit;
    const size_t cap = P.cap;
    if (cap * levels * nl >= (size_t)INT32_MAX) return fail(RT_ERR_LIMIT, "frame chunk too large for the chain path");
    // A frame of several chunks (C5: 17 of 32 M samples): chunks on the workspace slots' streams
    // (chunk j on slot j mod K), so one chunk's tail overlaps the next chunks' bulk.  Chunks write
    // disjoint output rows.
    const int nchunks = (li + chunk_rows - 1) / chunk_rows;
    const int K = std::min({nchunks, s->tune_slots, rt_scene::kSlots});
    // a frame of several chunks reports its chunks' largest continuation share (the record space must
    // hold the mirror-heavy chunks', not the last chunk's): k_mix's / k_pack_a's atomicMax into one word, cleared
    // here, on the caller's stream before the chunks fork
    const bool peak = nchunks > 1 && !count && P.phase_b && s->tune_cont_cb == 0;
    if (peak && f.chunk_k == 1) {
        if (!s->d_cont_peak) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s->d_cont_peak), sizeof(unsigned)));
        HIP_TRY(hipMemsetAsync(s->d_cont_peak, 0, sizeof(unsigned), st));
    }
    if (f.chunk_k == 1 && K > 1 && !s->trace_file.size()) {
        if (!s->fork_ev) HIP_TRY(hipEventCreateWithFlags(&s->fork_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->fork_ev, st));
        for (int j = 0; j < K; ++j) {
            if (!s->slot_stream[j]) HIP_TRY(hipStreamCreateWithFlags(&s->slot_stream[j], hipStreamNonBlocking));
            if (!s->slot_done[j]) HIP_TRY(hipEventCreateWithFlags(&s->slot_done[j], hipEventDisableTiming));
            HIP_TRY(hipStreamWaitEvent(s->slot_stream[j], s->fork_ev, 0));
            rtk::FrameParams g = f;
            g.chunk_k = K;
            g.chunk_j = j;
            const int rc = render_chain(s, eye, g, count, s->slot_stream[j], j);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(s->slot_done[j], s->slot_stream[j]));
            HIP_TRY(hipStreamWaitEvent(st, s->slot_done[j], 0));
        }
        // the frame's chunk peak, once every slot's chunks have folded theirs in (a read-back per
        // sub-call could miss other slots' pending atomicMax)
        if (peak) return read_back_cont(s, st, slot, s->d_cont_peak, cap);
        return RT_OK;
    }
    // order this use after the arena's previous one (possibly on another stream)
    if (arena.last && arena.last_stream != st) HIP_TRY(hipStreamWaitEvent(st, arena.last, 0));
    if (arena.bytes < P.bytes) {
        const bool log_alloc = (debug_flags() & kDbgLogAlloc) != 0;   // diagnostics: a growth inside a timed
        const auto ta = std::chrono::steady_clock::now();                // region serialises it
        if (log_alloc)
            std::fprintf(stderr, "librt_hip: slot %d workspace %.1f -> %.1f MB (frames %d, cb %zu of %zu)\n", slot,
                         arena.bytes / 1e6, P.bytes / 1e6, g.nframes, P.cb, P.cap);
        if (arena.p) HIP_TRY(hipStreamSynchronize(st));   // the previous frames on it may still use it
        (void)hipFree(arena.p);
        arena.p = nullptr;
        arena.bytes = 0;
        // (+1/16, within the slot's share of the budget: a slightly larger plan later -- the measured record
        // space moving -- fits without another synchronising reallocation; ADVICE r4: the headroom is part
        // of the budget, not on top of it)
        const size_t want = std::min(P.bytes + P.bytes / 16, std::max(P.bytes, s->slot_budget()));
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&arena.p), want));
        arena.bytes = want;
        if (log_alloc) std::fprintf(stderr, "librt_hip: slot %d workspace growth took %.2f ms\n", slot, ms_since(ta));
    }
    auto at = [&](size_t o) { return static_cast<void*>(arena.p + o); };
    rtc::PcParams p{};
    p.width = f.width; p.height = f.height; p.aa = f.aa; p.stripe_rows = f.stripe_rows;
    p.rank = f.rank; p.nranks = f.nranks; p.slab_rows = f.slab_rows;
    p.wi = wi; p.tiles_x = tiles_x; p.cap = (int)cap; p.levels = levels; p.nlights = s->dev.nlights;
    p.rec = static_cast<float4*>(at(P.o_rec));
    p.recd = static_cast<float4*>(at(P.o_recd));
    p.dbase = (unsigned)P.dbase;
    p.clevels = P.clevels;
    p.pinfo = static_cast<int*>(at(P.o_pinfo));
    p.occ = static_cast<uint8_t*>(at(P.o_occ));
    p.sqA = static_cast<unsigned*>(at(P.o_sqA)); p.scapA = P.scapA;
    p.scntA = static_cast<unsigned*>(at(P.o_scntA));
    p.sflatA = !P.split_occ && !P.rlists ? static_cast<unsigned*>(at(P.o_sflatA)) : nullptr;
    p.rlists = P.rlists ? 1 : 0;
    p.cq = static_cast<unsigned*>(at(P.o_cq)); p.ccapA = P.ccapA;
    p.ccnt = static_cast<unsigned*>(at(P.o_ccnt));
    p.cflat = static_cast<unsigned*>(at(P.o_cflat));
    p.sqB = static_cast<unsigned*>(at(P.o_sqB)); p.scapB = P.scapB;
    p.scntB = static_cast<unsigned*>(at(P.o_scntB)); p.sflatB = static_cast<unsigned*>(at(P.o_sflatB));
    p.totals = static_cast<unsigned*>(at(P.o_totals));
    p.la = P.la;
    p.cb = (unsigned)P.cb;
    p.cid = static_cast<unsigned*>(at(P.o_cid));
    p.tail = static_cast<float4*>(at(P.o_tail));
    p.fbc = static_cast<unsigned*>(at(P.o_fbc));
    p.fbc_cap = (unsigned)cap;
    p.fbs = static_cast<unsigned*>(at(P.o_fbs));
    p.fbs_cap = s->tune_fbs_cap > 0 ? (unsigned)std::min<size_t>(cap, s->tune_fbs_cap) : (unsigned)cap;
    // k_fallback: one workgroup per CU (it is empty or nearly so); a scene without the wide trees (their
    // build or containment check failed, or RT_WIDE_WALK=0 / RT_STREE<2) defers every walk to it, so it
    // then fills the GPU (those scenes would otherwise render in num_cus workgroups)
    p.fb_grid = (s->dev.use_wide && s->dev.use_stree == 2 && !s->dev.force_fb) ? s->num_cus : 4 * s->num_cus;
    p.kinline = P.phase_b ? P.kinline : 1 << 30;
    p.gb = P.gb;
    p.ogrid = P.phase_b ? std::max(1, s->mix_grid - P.gb) : s->mix_grid;
    p.occ_grid = s->occl_grid;
    p.fin_grid = 8 * s->num_cus;        // k_finish: at most 8 workgroups per CU (dispatch-bound at a lane per pixel)
    p.split_occ = P.split_occ ? 1 : 0;
    // A's shadow tasks walked where k_chain left them, region by region, by k_occlude in frame batches (a
    // lone frame's k_mix shadow role deals them in chunks of the region-order list instead, region_prefix:
    // region by region, their uneven sizes cost k_mix +60 us); B's LDS-queue overflow region by region in a
    // lone frame.  The region-by-region walks are the leaf-queue walker's (RT_LEAF_QUEUE builds).
    p.occ_inplace = RT_LEAF_QUEUE && !count && P.split_occ ? 1 : 0;
    p.occ_inplace_b = RT_LEAF_QUEUE && !P.split_occ && !count ? 1 : 0;
    p.cont_peak = peak ? s->d_cont_peak : nullptr;
    p.dbg_t = count ? nullptr : s->dbg_t;
    p.dbg_m = count ? nullptr : s->dbg_m;
    // wave service policy (pathchain.hpp PcParams; round 6 re-sweep at HEAD, every other setting +-0.5 % or slower:
    // profiles/r06_lone_knob_resweep.jsonl): phase A refills a wave once all its lanes are idle and services it once
    // all are done; phase B refills once <= 32 lanes walk and services once all 64 are done, at top priority
    p.refill = 0;
    p.service = 64;
    p.bservice = 64;
    p.btail = 64;
    p.bq_cap = std::min(s->tune_bq_cap, rtc::kMaxBq);
    p.orefill = s->tune_orefill;
    p.brefill = 32;
    p.bprio = 1;
    // continuations dealt one at a time round-robin for a lone frame (its deep chains spread over
    // the phase-B workgroups: 1.12 -> 1.10 ms; 2: 1.11-1.14, 4: 1.12-1.13), in chunks of 128 in batches
    p.tchunk = P.tchunk;
    p.ochunk = P.split_occ ? 256 : 128;
    p.lq_wait = s->tune_lq_wait;
    p.dyn_units = (int)P.dyn_units;
    p.ublk_h = -1;                      // phase-A units in column blocks a frame high and 8 units (2,048 px) wide
    p.ublk_w = 8;
    p.out = f.out; p.counters = f.counters;
    p.out_k = f.out_k; p.out_j = f.out_j;
    p.nframes = std::max(1, f.nframes);
    p.frame_rows = p.nframes > 1 ? f.frame_rows : f.slab_rows;
    if (p.nframes > rtc::kMaxFrames || (p.nframes > 1 && (!f.eyes || !f.outs || f.out_k != 1 ||
                                                          f.frame_rows * p.nframes != f.slab_rows)))
        return fail(RT_ERR_LIMIT, "internal: bad frame batch");
    for (int i = 0; i < rtc::kMaxFrames; ++i) {
        p.eyes[i] = i < p.nframes && p.nframes > 1 ? f.eyes[i] : eye;
        p.fouts[i] = i < p.nframes && p.nframes > 1 ? f.outs[i] : f.out;
    }
    p.trace_blocks = std::max(s->mix_grid, s->occl_grid);
    const size_t trace_n = 2 * (cap + (size_t)p.trace_blocks) + 4 * cap;
    p.trace = trace_buffer(s, trace_n);
    // lone frames in one launch (a drop-in caller's repeated frames): phase-A units heaviest-first by the
    // previous frame of the same geometry (PcParams::uorder), and this frame's costs ranked for the next
    const bool hot = s->tune_hot_units && !count && p.nframes == 1 && P.dyn_units > 0 &&
                     units == g.units_total;
    // frame batches' deep-first deal (PcParams::pdepth): one launch of whole frames; the depths of the slot's
    // previous launch of the same geometry (frame size and frames per launch) per sample slot (zero, all
    // shallow, else)
    p.pdepth = nullptr;
    p.ccntd = nullptr;
    p.deep_min = 0;
    if (s->tune_deep > 0 && !count && P.split_occ && P.phase_b && !P.rlists && units == g.units_total) {
        const size_t fs = cap;
        uint64_t key = 1469598103934665603ull;
        for (long long v : {(long long)p.width, (long long)p.height, (long long)p.aa, (long long)p.stripe_rows,
                            (long long)p.rank, (long long)p.nranks, (long long)p.frame_rows, (long long)p.nframes,
                            (long long)p.n0, (long long)fs})
            key = (key ^ (uint64_t)v) * 1099511628211ull;
        if (arena.pdepth_n < fs) {
            if (arena.pdepth) HIP_TRY(hipStreamSynchronize(st));   // earlier launches may still use it
            (void)hipFree(arena.pdepth);
            arena.pdepth = nullptr;
            arena.pdepth_n = 0;
            HIP_TRY(hipMalloc(reinterpret_cast<void**>(&arena.pdepth), fs));
            arena.pdepth_n = fs;
            arena.pdepth_key = 0;
        }
        if (arena.pdepth_key != key) {
            HIP_TRY(hipMemsetAsync(arena.pdepth, 0, fs, st));
            arena.pdepth_key = key;
        }
        p.pdepth = arena.pdepth;
        p.ccntd = static_cast<unsigned*>(at(P.o_ccntd));
        p.deep_min = s->tune_deep;
    }
    p.urank = p.uorder_on = 0;
    p.ugrp = nullptr;
    p.mix_cls = 0;
    for (int r0 = f.chunk_j * chunk_rows; r0 < li; r0 += f.chunk_k * chunk_rows) {
        p.chunk_row0 = r0;
        p.chunk_rows = std::min(chunk_rows, li - r0);
        p.n0 = tiles_x * ((p.chunk_rows + 7) / 8) * 64;
        p.grid = grid_for(p.n0);
        if (hot) {
            const unsigned nu = (unsigned)((p.n0 + 255) / 256);
            if (arena.hist_units != nu) {
                if (arena.hist) HIP_TRY(hipStreamSynchronize(st));   // earlier frames may still use it
                (void)hipFree(arena.hist);
                arena.hist = nullptr;
                arena.hist_units = 0;
                arena.hist_key = 0;
                HIP_TRY(hipMalloc(reinterpret_cast<void**>(&arena.hist), 4 * (size_t)nu * sizeof(unsigned)));
                HIP_TRY(hipMemsetAsync(arena.hist, 0, 2 * (size_t)nu * sizeof(unsigned), st));
                arena.hist_units = nu;
            }
            uint64_t key = 1469598103934665603ull;   // the geometry the order is valid for
            for (long long v : {(long long)p.width, (long long)p.height, (long long)p.aa, (long long)p.stripe_rows,
                                (long long)p.rank, (long long)p.nranks, (long long)p.slab_rows, (long long)p.n0,
                                (long long)p.tiles_x, (long long)p.ublk_h, (long long)p.ublk_w})
                key = (key ^ (uint64_t)v) * 1099511628211ull;
            p.ucost = arena.hist;
            p.uorder = arena.hist + nu;
            p.ucol = arena.hist + 2 * (size_t)nu;
            p.ugrp = arena.hist + 3 * (size_t)nu;
            p.mix_cls = s->tune_mix;
            if (arena.hist_key != key) {           // this geometry's column order (unit_col), once
                std::vector<unsigned> col(nu);
                for (unsigned u = 0; u < nu; ++u) col[u] = rtc::unit_col(p.tiles_x, p.ublk_h, p.ublk_w, p.nframes, u, nu);
                HIP_TRY(hipMemcpyAsync(arena.hist + 2 * (size_t)nu, col.data(), nu * sizeof(unsigned),
                                       hipMemcpyHostToDevice, st));
                HIP_TRY(hipStreamSynchronize(st));   // (the pageable source goes out of scope)
            }
            p.urank = 1;
            p.uorder_on = arena.hist_key == key ? 1 : 0;   // ranked by the previous frame of this geometry
            arena.hist_key = key;                          // (its k_mix ran before this k_chain: stream order)
        }
        if (p.grid > P.G) return fail(RT_ERR_LIMIT, "internal: chain grid exceeds the workspace");
        if (s->ktime) {
            // diagnostics: each kernel's own start / stop timestamps (KTimer), then the launch's per-kernel split
            // (synchronous)
            for (int i = 0; i < rtc::KTimer::kMax; ++i) {
                if (!s->kt.ev0[i]) HIP_TRY(hipEventCreate(&s->kt.ev0[i]));
                if (!s->kt.ev1[i]) HIP_TRY(hipEventCreate(&s->kt.ev1[i]));
            }
            s->kt.n = 0;
            HIP_TRY(rtc::launch_chain_chunk(s->dev, eye, p, count, st, &s->kt));
            HIP_TRY(hipStreamSynchronize(st));
            for (int i = 0; i < s->kt.n; ++i) {
                float ms = 0;
                HIP_TRY(hipEventElapsedTime(&ms, s->kt.ev0[i], s->kt.ev1[i]));
                s->kt_ms[s->kt.kind[i]] += ms;
            }
            s->kt_launches++;
        } else {
            HIP_TRY(rtc::launch_chain_chunk(s->dev, eye, p, count, st));
        }
    }
    // the share, read back later (a chunk of a forked frame: the parent call reads the frame's peak)
    if (!count && P.phase_b && (p.nframes > 1 || chunk_rows < li) && s->tune_cont_cb == 0 && f.chunk_k == 1) {
        const int rc = read_back_cont(s, st, slot, p.cont_peak ? p.cont_peak : p.totals + 1, cap);
        if (rc) return rc;
    }
    if (p.trace) trace_dump(s, st, 0, (unsigned)cap, (unsigned)p.trace_blocks, trace_n);   // last chunk only
    if (!arena.last) HIP_TRY(hipEventCreateWithFlags(&arena.last, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(arena.last, st));
    arena.last_stream = st;
    return RT_OK;
}

// The device error word after the device is idle: RT_ERR_LIMIT (and the word
// cleared) when a walk was cut off by walk_runaway (bit 0) or a wait loop by
// spin_over (bit 1) since the last check.
int device_error(unsigned e) {
    if (e & 2u)
        return fail(RT_ERR_LIMIT, "a wait on other lanes or waves exceeded its bound (spin_cap) and was cut off; "
                                  "the frame is invalid");
    return fail(RT_ERR_LIMIT, "a BVH walk exceeded its step bound (walk_cap) and was cut off; the frame is invalid");
}

int check_device_error(rt_scene* s) {
    unsigned e = 0;
    HIP_TRY(hipMemcpy(&e, s->d_err, sizeof(e), hipMemcpyDeviceToHost));
    if (e == 0) return RT_OK;
    HIP_TRY(hipMemset(s->d_err, 0, sizeof(unsigned)));
    return device_error(e);
}

// After a host-output staging buffer grew (slot_budget takes it off the budget): free the arenas now over
// their slot's share (the device is idle: the growth synchronised); each is re-made within it at its next use.
void fit_arenas(rt_scene* s) {
    const size_t share = s->slot_budget();
    for (auto& a : s->arenas)
        if (a.bytes > share) {
            (void)hipFree(a.p);
            a.p = nullptr;
            a.bytes = 0;
        }
}

}  // namespace

extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_device_count(int* count) {
    if (!count) return fail(RT_ERR_ARG, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = e == hipSuccess ? n : 0;
    return RT_OK;
}

int rt_scene_create(const rt_scene_desc* desc, const rt_options* opts, rt_scene** out) {
    if (!desc || !out) return fail(RT_ERR_ARG, "desc/out is NULL");
    *out = nullptr;
    rt_scene* s = new (std::nothrow) rt_scene();
    if (!s) return fail(RT_ERR_ARG, "out of host memory");
    start_device_warmup(opts);
    rtx::HostScene& h = s->host;
    for (int i = 0; i < 3; ++i) h.bg[i] = desc->background_color[i];
    h.eps = desc->shadow_ray_epsilon;
    h.max_depth = desc->max_recursion_depth;
    h.ambient = rtx::V3{desc->ambient_light.x, desc->ambient_light.y, desc->ambient_light.z};
    auto v3 = [](const rt_vec3f& v) { return rtx::V3{v.x, v.y, v.z}; };
    for (int i = 0; i < desc->num_lights; ++i)
        h.lights.push_back(rtx::LightRec{v3(desc->lights[i].position), v3(desc->lights[i].intensity)});
    for (int i = 0; i < desc->num_materials; ++i) {
        const rt_material& m = desc->materials[i];
        h.materials.push_back(rtx::MaterialRec{m.is_mirror, v3(m.ambient), v3(m.diffuse), v3(m.specular),
                                               v3(m.mirror), m.phong_exponent});
    }
    for (int i = 0; i < desc->num_vertices; ++i) h.verts.push_back(v3(desc->vertices[i]));
    const int nv = desc->num_vertices, nm = desc->num_materials;
    for (int i = 0; i < desc->num_triangles; ++i) {
        const rt_triangle& t = desc->triangles[i];
        if (t.v0_id < 1 || t.v1_id < 1 || t.v2_id < 1 || t.v0_id > nv || t.v1_id > nv || t.v2_id > nv ||
            t.material_id < 1 || t.material_id > nm) {
            delete s;
            return fail(RT_ERR_ARG, "triangle " + std::to_string(i) + " references a missing vertex or material");
        }
        h.tris.push_back(rtx::TriRec{t.material_id, t.v0_id, t.v1_id, t.v2_id, {0, 0, 0}, {0, 0, 0}});
    }
    for (int i = 0; i < desc->num_spheres; ++i) {
        const rt_sphere& sp = desc->spheres[i];
        if (sp.center_vertex_id < 1 || sp.center_vertex_id > nv || sp.material_id < 1 || sp.material_id > nm) {
            delete s;
            return fail(RT_ERR_ARG, "sphere " + std::to_string(i) + " references a missing vertex or material");
        }
        h.spheres.push_back(rtx::SphereRec{sp.material_id, sp.center_vertex_id, sp.radius});
    }
    int rc = finish_scene(s, opts);
    if (rc) { delete s; return rc; }
    *out = s;
    return RT_OK;
}

int rt_scene_load_xml(const char* path, const rt_options* opts, rt_scene** out) {
    if (!path || !out) return fail(RT_ERR_ARG, "path/out is NULL");
    *out = nullptr;
    rt_scene* s = new (std::nothrow) rt_scene();
    if (!s) return fail(RT_ERR_ARG, "out of host memory");
    start_device_warmup(opts);
    const auto t = std::chrono::steady_clock::now();
    std::string err = rtx::load_xml(path, s->host, opts ? opts->build_threads : 0);
    s->xml_ms = ms_since(t);
    if (!err.empty()) {
        delete s;
        return fail(err.find("cannot be loaded") != std::string::npos ? RT_ERR_IO : RT_ERR_PARSE, err);
    }
    int rc = finish_scene(s, opts);
    if (rc) { delete s; return rc; }
    *out = s;
    return RT_OK;
}

void rt_scene_destroy(rt_scene* scene) {
    if (!scene) return;
    if (!scene->host_only) (void)hipSetDevice(scene->device);
    delete scene;
}

int rt_scene_num_cameras(const rt_scene* s) { return s ? (int)s->host.cameras.size() : 0; }

int rt_scene_get_camera(const rt_scene* s, int index, rt_camera* cam, char* name, int name_len) {
    if (!s || !cam) return fail(RT_ERR_ARG, "scene/cam is NULL");
    if (index < 0 || index >= (int)s->host.cameras.size()) return fail(RT_ERR_ARG, "camera index out of range");
    const rtx::CameraRec& c = s->host.cameras[index];
    cam->position = rt_vec3f{c.position.x, c.position.y, c.position.z};
    cam->gaze = rt_vec3f{c.gaze.x, c.gaze.y, c.gaze.z};
    cam->up = rt_vec3f{c.up.x, c.up.y, c.up.z};
    for (int i = 0; i < 4; ++i) cam->near_plane[i] = c.near_plane[i];
    cam->near_distance = c.near_distance;
    cam->image_width = c.width;
    cam->image_height = c.height;
    if (name && name_len > 0) std::snprintf(name, name_len, "%s", c.name.c_str());
    return RT_OK;
}

int rt_scene_bvh_info(const rt_scene* s, rt_bvh_info* info) {
    if (!s || !info) return fail(RT_ERR_ARG, "scene/info is NULL");
    info->nodes = (int)s->bvh.nodes.size();
    info->leaves = s->bvh.leaves;
    info->max_leaf_prims = s->bvh.max_leaf;
    info->max_depth = s->bvh.max_depth;
    info->max_stack = s->bvh.max_stack;
    info->triangles = (int)s->host.tris.size();
    info->spheres = (int)s->host.spheres.size();
    info->build_ms = s->bvh.build_ms;
    info->ref_ms = s->bvh.ref_ms;
    info->wide_ms = s->bvh.stree_ms;
    info->xml_ms = s->xml_ms;
    info->prep_ms = s->prep_ms;
    info->flat_ms = s->bvh.flat_ms;
    info->refwide_ms = s->bvh.refwide_ms;
    info->stree_ms = s->bvh.stree_ms;
    info->upload_ms = s->upload_ms;
    info->build_threads = s->bvh.threads;
    info->wide_nodes = (int)(s->bvh.swnodes.size() + s->bvh.wnodes.size());
    uint64_t h = 1469598103934665603ull;           // FNV-1a over the 4-wide tree's bytes
    auto mix = [&h](const void* p, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(p);
        for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
    };
    mix(s->bvh.swnodes.data(), s->bvh.swnodes.size() * sizeof(dl::Wide));
    mix(s->bvh.wnodes.data(), s->bvh.wnodes.size() * sizeof(dl::Wide));
    mix(s->bvh.lrec.data(), s->bvh.lrec.size() * sizeof(dl::Vec4));
    mix(&s->bvh.swroot, sizeof(s->bvh.swroot));
    mix(&s->bvh.wroot, sizeof(s->bvh.wroot));
    info->wide_hash = h;
    info->ref_wide_bytes = s->bvh.wnodes.size() * sizeof(dl::Wide);
    info->occ_wide_bytes = s->bvh.swnodes.size() * sizeof(dl::Wide);
    info->leaf_record_bytes = s->bvh.lrec.size() * sizeof(dl::Vec4);
    info->tri_shade_bytes = s->bvh.tri_shade.size() * sizeof(dl::TriShade);
    return RT_OK;
}

int rt_scene_set_max_depth(rt_scene* s, int d) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    if (d < -1 || d > 64) return fail(RT_ERR_ARG, "max_recursion_depth out of range [-1, 64]");
    s->host.max_depth = d;
    s->dev.max_depth = d;
    if (s->group) return rt_internal_group_set_max_depth(s->group, d);
    return RT_OK;
}

int rt_scene_export_nodes(const rt_scene* s, void* out, int capacity) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    const int n = (int)s->bvh.nodes.size();
    if (out && capacity > 0) std::memcpy(out, s->bvh.nodes.data(), (size_t)std::min(n, capacity) * sizeof(dl::Node));
    return n;
}

int rt_scene_memory(const rt_scene* s, uint64_t* scene_bytes, uint64_t* workspace_bytes) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    size_t ws = s->out_cap + s->batch_out_cap + s->trace_cap * sizeof(unsigned);
    for (const auto& a : s->arenas) ws += a.bytes + a.pdepth_n + 4 * (size_t)a.hist_units * sizeof(unsigned);
    if (scene_bytes) *scene_bytes = s->host_only ? 0 : s->scene_bytes;
    if (workspace_bytes) *workspace_bytes = ws;
    return RT_OK;
}

int rt_slab_rows(int height, int stripe_rows, int nranks) {
    if (height < 1 || stripe_rows < 1 || nranks < 1) return 0;
    const int stripes = (height + stripe_rows - 1) / stripe_rows;
    return ((stripes + nranks - 1) / nranks) * stripe_rows;
}

}  // extern "C"

namespace {
constexpr long long kMergeFrameSamples = 1 << 19;   // render_cameras: frames below this are merged into larger batches

// One frame (rank `rank`'s stripes) on `stream`, chain-path workspace `slot`.  (Splitting a frame into
// concurrent interleaved sub-frames measured slower, +8 % / +18 % for 2 / 3, and was removed in round 6.)
int render_frame(rt_scene* s, const rt_camera* cam, int aa, int stripe_rows, int rank, int nranks, void* out_dev,
                 hipStream_t stream, int flags, int slot) {
    if (!s || !out_dev) return fail(RT_ERR_ARG, "scene/out is NULL");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    int rc = check_camera(cam, aa);
    if (rc) return rc;
    if (stripe_rows < 1 || nranks < 1 || rank < 0 || rank >= nranks) return fail(RT_ERR_ARG, "bad stripe/rank");
    HIP_TRY(hipSetDevice(s->device));
    const rtk::Eye eye = make_eye(*cam, cam->image_width * aa, cam->image_height * aa);
    rtk::FrameParams p;
    p.width = cam->image_width;
    p.height = cam->image_height;
    p.aa = aa;
    p.stripe_rows = stripe_rows;
    p.rank = rank;
    p.nranks = nranks;
    p.slab_rows = rt_slab_rows(cam->image_height, stripe_rows, nranks);
    p.out = static_cast<uint8_t*>(out_dev);
    p.counters = s->d_counters;
    const bool count = (flags & RT_RENDER_COUNT) != 0;
    return render_chain(s, eye, p, count, stream, slot);
}
}  // namespace

extern "C" {


int rt_render_device(rt_scene* s, const rt_camera* cam, int aa, int stripe_rows, int rank, int nranks,
                     void* out_dev, void* stream, int flags) {
    return render_frame(s, cam, aa, stripe_rows, rank, nranks, out_dev, static_cast<hipStream_t>(stream), flags, 0);
}

// raytracer.cpp:505-519 (one render per camera), batched: the cameras' frames
// run concurrently, frame i on slot i mod kSlots (its own stream and
// workspace), forked from and joined back into `stream`.  Each frame's tail
// (its few long mirror chains) overlaps the other frames' bulk.  The chain
// path runs the slots concurrently; the other paths render one after another.
// Frame batch: n frames of one size (rank `rank`'s stripes of each) as ONE
// chain-path launch sequence.  The frames' samples form one virtual slab of
// n * slab_rows rows (pathchain.hpp PcParams.nframes): one persistent grid
// walks them all, so one frame's slow mirror-chain tail runs beside the other
// frames' bulk instead of after it.
int render_batch(rt_scene* s, const rt_camera* cams, int n, int aa, int stripe_rows, int rank, int nranks,
                 void* const* outs_dev, hipStream_t stream, int flags, int slot) {
    if (n == 1)
        return render_frame(s, cams, aa, stripe_rows, rank, nranks, outs_dev[0], stream, flags, slot);
    if (n > rtc::kMaxFrames) return fail(RT_ERR_LIMIT, "internal: frame batch too large");
    if (stripe_rows < 1 || nranks < 1 || rank < 0 || rank >= nranks) return fail(RT_ERR_ARG, "bad stripe/rank");
    HIP_TRY(hipSetDevice(s->device));
    rtk::Eye eyes[rtc::kMaxFrames];
    for (int i = 0; i < n; ++i) eyes[i] = make_eye(cams[i], cams[i].image_width * aa, cams[i].image_height * aa);
    rtk::FrameParams p;
    p.width = cams[0].image_width;
    p.height = cams[0].image_height;
    p.aa = aa;
    p.stripe_rows = stripe_rows;
    p.rank = rank;
    p.nranks = nranks;
    p.frame_rows = rt_slab_rows(p.height, stripe_rows, nranks);
    p.nframes = n;
    p.slab_rows = p.frame_rows * n;
    p.eyes = eyes;
    p.outs = reinterpret_cast<uint8_t* const*>(outs_dev);
    p.out = static_cast<uint8_t*>(outs_dev[0]);
    p.counters = s->d_counters;
    return render_chain(s, eyes[0], p, (flags & RT_RENDER_COUNT) != 0, stream, slot);
}

// stripe_rows <= 0: whole frames (each camera's own height); otherwise every
// frame is this rank's row stripes (rt_render_frames_device).  may_wait: a synchronous entry point
// (rt_render_cameras), which may wait on the host for a scene's first batch (below).
int render_cameras(rt_scene* s, const rt_camera* cams, int n, int aa, void* const* outs_dev, hipStream_t stream,
                   int flags, int stripe_rows = 0, int rank = 0, int nranks = 1, bool may_wait = false,
                   int batch_max = 0, int slot0 = 0) {
    auto rows_of = [&](int i) { return stripe_rows > 0 ? stripe_rows : cams[i].image_height; };
    if (n > 1) {
        // consecutive same-size frames, up to kMaxFrames and one chain chunk of samples per batch
        const int nslot = std::max(1, std::min(s->tune_slots, rt_scene::kSlots));
        // (batch_max, slot0: the rest of a call after its first batch, on the next slots -- batches of the
        // same size as the calls that follow, on every slot, so no workspace grows inside those)
        const int bmax = std::min(rtc::kMaxFrames, batch_max > 0 ? batch_max : rtc::kMaxFrames);
        std::vector<int> starts;
        HIP_TRY(hipSetDevice(s->device));
        if (const int rc = ensure_chain_grids(s)) return rc;
        // every slot's stream and event up front: created inside a later call (its first use) it stalled
        // that call (mirror_spheres batches 0.10 -> 0.25 ms/frame when a scene's first call left slot 0's
        // stream unused)
        for (int k = 0; k < nslot; ++k) {
            if (!s->slot_stream[k]) HIP_TRY(hipStreamCreateWithFlags(&s->slot_stream[k], hipStreamNonBlocking));
            if (!s->slot_done[k]) HIP_TRY(hipEventCreateWithFlags(&s->slot_done[k], hipEventDisableTiming));
        }
        poll_cont(s, false);
        // runs of consecutive same-size frames; a run of L frames goes out as batches of min(m, ceil(L / nslot))
        // frames, m the most frames one launch's plan fits in the slot's workspace share: a 20-frame call on 6
        // slots runs 4,4,4,4,4 on 5.  (Round 5's balanced deal, 4,4,3,3,3,3 with every slot busy, measured
        // slower -- the sixth concurrent batch's first kernel starts ~0.65 ms after the others whatever the
        // hardware-queue count -- and was removed in round 6.)
        for (int i = 0; i < n;) {
            const auto& c = cams[i];
            // a batch of k frames: one launch (render_chain's own plan fits the slot's workspace share)
            auto fits = [&](int k) {
                rtk::FrameParams f;
                f.width = c.image_width;
                f.aa = aa;
                f.slab_rows = rt_slab_rows(c.image_height, rows_of(i), nranks) * k;
                f.nframes = k;
                const ChainGeom g = chain_geom(s, f);
                return chain_launch_units(s, g, (flags & RT_RENDER_COUNT) != 0) >= g.units_total;
            };
            int L = 1;
            while (i + L < n && cams[i + L].image_width == c.image_width && cams[i + L].image_height == c.image_height)
                ++L;
            int m = 1;
            while (m < std::min(bmax, L) && fits(m + 1)) ++m;
            // as many batches as slots, but, for small frames (< kMergeFrameSamples each, such as a rank's 1/8 share
            // of a C3 frame), at least ~batch_samples samples each: 20 such frames go out in 3 batches of 7 rather
            // than 5 of 4 -- each batch ends with its own phase-B tail, which few samples do not hide (the one-GPU
            // rehearsal of 8 ranks: 0.105 -> 0.094 ms per frame, profiles/r05_shard20.txt).  Frames of
            // kMergeFrameSamples or more are never merged beyond that: round 5's rule, applied to every frame size,
            // put a 2-frame marbles call in one batch, 1.27 -> 1.68 ms per frame (the round-6 call-size sweep,
            // profiles/r06_sweep_callsize_*.jsonl)
            const double frame_samples = (double)rt_slab_rows(c.image_height, rows_of(i), nranks) * c.image_width * aa * aa;
            const double need = frame_samples < (double)kMergeFrameSamples ? (double)s->tune_batch_samples : 1.0;
            const int nbat = std::max(1, std::min(nslot, (int)std::ceil((double)L * frame_samples / need)));
            const int ch = std::min(m, (L + nbat - 1) / nbat);
            for (int b = 0; b < L; b += ch) starts.push_back(i + b);
            i += L;
        }
        starts.push_back(n);
        const int nb = (int)starts.size() - 1;
        if (nb == 1) return render_batch(s, cams, n, aa, rows_of(0), rank, nranks, outs_dev, stream, flags, 0);
        if (may_wait && s->cont_frac == 0 && !(flags & RT_RENDER_COUNT) && s->tune_cont_cb == 0 &&
            s->dev.max_depth > rt_scene::kKinline) {
            // the scene's continuation share is not known yet: one batch first, waited for, so the rest
            // are sized by it (once per scene; a mirror-heavy scene otherwise sends most of its deep
            // chains to k_fallback until the first read-backs arrive).  Synchronous callers only (ADVICE
            // r4): the asynchronous entries never block the caller's stream; their first call runs with
            // the default record space and the later calls are sized by the read-backs that are done.
            const int rc = render_batch(s, cams, starts[1], aa, rows_of(0), rank, nranks, outs_dev, stream, flags, 0);
            if (rc) return rc;
            poll_cont(s, true);
            s->cont_frac = std::max(s->cont_frac, 1e-9);
            return render_cameras(s, cams + starts[1], n - starts[1], aa, outs_dev + starts[1], stream, flags,
                                  stripe_rows, rank, nranks, may_wait, starts[2] - starts[1], 1);
        }
        if (!s->fork_ev) HIP_TRY(hipEventCreateWithFlags(&s->fork_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(s->fork_ev, stream));
        const int used = std::min(nb, nslot);
        for (int j = 0; j < used; ++j) {
            const int k = (j + slot0) % nslot;
            if (!s->slot_stream[k]) HIP_TRY(hipStreamCreateWithFlags(&s->slot_stream[k], hipStreamNonBlocking));
            if (!s->slot_done[k]) HIP_TRY(hipEventCreateWithFlags(&s->slot_done[k], hipEventDisableTiming));
            HIP_TRY(hipStreamWaitEvent(s->slot_stream[k], s->fork_ev, 0));
        }
        // RT_DEBUG 0x04 (diagnostics): per batch, the host's submission time and (HIP events on the slot
        // streams, waited for at the end of the call: this makes the call synchronous) its GPU start and end
        const bool log_submit = (debug_flags() & kDbgLogSubmit) != 0;
        auto now_us = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
        const double ts0 = log_submit ? now_us() : 0.0;
        std::vector<hipEvent_t> bev;
        std::vector<double> host_us;
        for (int b = 0; b < nb; ++b) {
            const int k = (b + slot0) % nslot, i = starts[b];
            const double tb = log_submit ? now_us() : 0.0;
            if (log_submit) {
                bev.resize(bev.size() + 2);
                HIP_TRY(hipEventCreate(&bev[bev.size() - 2]));
                HIP_TRY(hipEventCreate(&bev[bev.size() - 1]));
                HIP_TRY(hipEventRecord(bev[bev.size() - 2], s->slot_stream[k]));
            }
            const int rc = render_batch(s, cams + i, starts[b + 1] - i, aa, rows_of(i), rank, nranks, outs_dev + i,
                                        s->slot_stream[k], flags, k);
            if (rc) return rc;
            if (log_submit) {
                HIP_TRY(hipEventRecord(bev.back(), s->slot_stream[k]));
                host_us.push_back(tb - ts0);
                host_us.push_back(now_us() - tb);
            }
        }
        if (log_submit) {
            for (auto e : bev) HIP_TRY(hipEventSynchronize(e));
            for (int b = 0; b < nb; ++b) {
                float g0 = 0, g1 = 0;
                HIP_TRY(hipEventElapsedTime(&g0, bev[0], bev[2 * b]));
                HIP_TRY(hipEventElapsedTime(&g1, bev[0], bev[2 * b + 1]));
                std::fprintf(stderr, "{\"submit\": {\"batch\": %d, \"frames\": %d, \"slot\": %d, \"host_start_us\": %.1f, "
                             "\"host_us\": %.1f, \"gpu_start_ms\": %.4f, \"gpu_end_ms\": %.4f}}\n",
                             b, starts[b + 1] - starts[b], (b + slot0) % nslot, host_us[2 * b], host_us[2 * b + 1], g0, g1);
            }
            for (auto e : bev) (void)hipEventDestroy(e);
        }
        for (int j = 0; j < used; ++j) {
            const int k = (j + slot0) % nslot;
            HIP_TRY(hipEventRecord(s->slot_done[k], s->slot_stream[k]));
            HIP_TRY(hipStreamWaitEvent(stream, s->slot_done[k], 0));
        }
        return RT_OK;
    }
    return render_frame(s, &cams[0], aa, rows_of(0), rank, nranks, outs_dev[0], stream, flags, 0);
}

int rt_render_cameras_device(rt_scene* s, const rt_camera* cams, int n, int aa, void* const* outs_dev, void* stream,
                             int flags) {
    if (!s || !cams || !outs_dev || n < 1) return fail(RT_ERR_ARG, "scene/cameras/outputs is NULL or n < 1");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    for (int i = 0; i < n; ++i) {
        const int rc = check_camera(&cams[i], aa);
        if (rc) return rc;
        if (!outs_dev[i]) return fail(RT_ERR_ARG, "output buffer is NULL");
    }
    HIP_TRY(hipSetDevice(s->device));
    return render_cameras(s, cams, n, aa, outs_dev, static_cast<hipStream_t>(stream), flags);
}

int rt_render_frames_device(rt_scene* s, const rt_camera* cams, int n, int aa, int stripe_rows, int rank,
                            int nranks, void* const* outs_dev, void* stream, int flags) {
    if (!s || !cams || !outs_dev || n < 1) return fail(RT_ERR_ARG, "scene/cameras/outputs is NULL or n < 1");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    if (stripe_rows < 1 || nranks < 1 || rank < 0 || rank >= nranks) return fail(RT_ERR_ARG, "bad stripe/rank");
    for (int i = 0; i < n; ++i) {
        const int rc = check_camera(&cams[i], aa);
        if (rc) return rc;
        if (!outs_dev[i]) return fail(RT_ERR_ARG, "output buffer is NULL");
    }
    HIP_TRY(hipSetDevice(s->device));
    return render_cameras(s, cams, n, aa, outs_dev, static_cast<hipStream_t>(stream), flags, stripe_rows, rank,
                          nranks);
}

int rt_render_cameras(rt_scene* s, const rt_camera* cams, int n, int aa, uint8_t* const* outs, rt_stats* stats) {
    if (!s || !cams || !outs || n < 1) return fail(RT_ERR_ARG, "scene/cameras/outputs is NULL or n < 1");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    for (int i = 0; i < n; ++i) {
        const int rc = check_camera(&cams[i], aa);
        if (rc) return rc;
        if (!outs[i]) return fail(RT_ERR_ARG, "output buffer is NULL");
    }
    const auto t0 = std::chrono::steady_clock::now();
    if (s->group) {
        // device group: runs of consecutive same-size cameras as frame batches (every device renders its
        // stripes of all of them in flight together, one grouped gather per run)
        // (RT_GROUP_BATCH: at most this many frames per grouped gather; 1 = one gather per frame, the
        // path without several gathers per communicator in one RCCL group)
        int batch = rtc::kMaxFrames;
        if (const char* e = std::getenv("RT_GROUP_BATCH")) batch = std::max(1, std::min(rtc::kMaxFrames, std::atoi(e)));
        rt_stats sum{}, one{};
        for (int i = 0; i < n;) {
            int j = i + 1;
            while (j < n && j - i < batch && cams[j].image_width == cams[i].image_width &&
                   cams[j].image_height == cams[i].image_height)
                ++j;
            const int rc = rt_internal_group_render_frames(s->group, cams + i, j - i, aa, outs + i,
                                                           stats ? &one : nullptr);
            if (rc) return rc;
            sum.primary_rays += one.primary_rays; sum.shadow_rays += one.shadow_rays;
            sum.reflection_rays += one.reflection_rays; sum.node_visits += one.node_visits;
            sum.tri_tests += one.tri_tests; sum.sphere_tests += one.sphere_tests; sum.kernel_ms += one.kernel_ms;
            sum.shadow_rays_skipped += one.shadow_rays_skipped;
            i = j;
        }
        if (stats) {
            *stats = sum;
            stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        }
        return RT_OK;
    }
    HIP_TRY(hipSetDevice(s->device));
    // one device frame per camera (one arena, grown on demand): every frame is
    // launched before any copy, so the frames run concurrently
    std::vector<size_t> off(n + 1, 0);
    for (int i = 0; i < n; ++i) off[i + 1] = off[i] + (((size_t)cams[i].image_width * cams[i].image_height * 3 + 255) & ~size_t(255));
    if (off[n] > s->batch_out_cap) {
        HIP_TRY(hipDeviceSynchronize());
        (void)hipFree(s->batch_out);
        s->batch_out = nullptr;
        s->batch_out_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s->batch_out), off[n]));
        s->batch_out_cap = off[n];
        fit_arenas(s);
    }
    std::vector<void*> dev(n);
    for (int i = 0; i < n; ++i) dev[i] = s->batch_out + off[i];
    const bool count = stats != nullptr;
    if (count) HIP_TRY(hipMemset(s->d_counters, 0, rtc::kCounters * sizeof(unsigned long long)));
    const bool log = (debug_flags() & kDbgLogInit) != 0;   // diagnostics (tools/exp_cli.py --phases)
    const double t_out = log ? ms_since(t0) : 0.0;
    int rc = render_cameras(s, cams, n, aa, dev.data(), nullptr, count ? RT_RENDER_COUNT : 0, 0, 0, 1, true);
    const double t_sub = log ? ms_since(t0) : 0.0;
    double t_gpu = 0.0;
    if (rc == RT_OK) {
        HIP_TRY(hipDeviceSynchronize());
        if (log) t_gpu = ms_since(t0);
        for (int i = 0; i < n; ++i)
            HIP_TRY(hipMemcpy(outs[i], dev[i], (size_t)cams[i].image_width * cams[i].image_height * 3,
                              hipMemcpyDeviceToHost));
    }
    HIP_TRY(hipDeviceSynchronize());
    if (log)
        std::fprintf(stderr, "{\"rt_render_cameras\": {\"outputs_ms\": %.3f, \"submitted_ms\": %.3f, \"gpu_done_ms\": %.3f, "
                     "\"copied_ms\": %.3f}}\n", t_out, t_sub, t_gpu, ms_since(t0));
    if (rc) return rc;
    if ((rc = check_device_error(s))) return rc;
    if (stats) {
        rc = rt_counters_read(s, stats);
        if (rc) return rc;
        stats->kernel_ms = 0;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

int rt_walk_timing(rt_scene* s, const float* rays, int n, int lanes, int reps, int mode, unsigned long long* out) {
    if (!s || !rays || !out || n < 1 || lanes < 1 || lanes > 64 || reps < 1) return fail(RT_ERR_ARG, "bad walk-timing arguments");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    HIP_TRY(hipSetDevice(s->device));
    float* dr = nullptr;
    unsigned long long* dout = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dr), (size_t)n * 6 * sizeof(float)));
    if (hipMalloc(reinterpret_cast<void**>(&dout), (size_t)n * 4 * sizeof(unsigned long long)) != hipSuccess) {
        (void)hipFree(dr);
        return fail(RT_ERR_HIP, "hipMalloc failed");
    }
    hipError_t e = hipMemcpy(dr, rays, (size_t)n * 6 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtc::launch_walk_timing(s->dev, dr, n, lanes, reps, mode, dout, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, dout, (size_t)n * 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(dr);
    (void)hipFree(dout);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("walk timing: ") + hipGetErrorName(e));
    return RT_OK;
}

int rt_phong_pow(const float* base, const float* exponent, float* out, int n) {
    if (!base || !exponent || !out || n < 0) return fail(RT_ERR_ARG, "bad phong_pow arguments");
    if (n == 0) return RT_OK;
    float* d = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * 3 * sizeof(float)));
    hipError_t e = hipMemcpy(d, base, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + n, exponent, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtc::launch_phong_pow(d, d + n, d + 2 * (size_t)n, n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 2 * (size_t)n, (size_t)n * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("phong_pow: ") + hipGetErrorName(e));
    return RT_OK;
}

int rt_cramer_div(const float* den, const float* num, float* out, int n) {
    if (!den || !num || !out || n < 0) return fail(RT_ERR_ARG, "bad cramer_div arguments");
    if (n == 0) return RT_OK;
    float* d = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * 7 * sizeof(float)));
    hipError_t e = hipMemcpy(d, den, (size_t)n * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d + n, num, (size_t)n * 3 * sizeof(float), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtc::launch_cramer_div(d, d + n, d + 4 * (size_t)n, n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, d + 4 * (size_t)n, (size_t)n * 3 * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("cramer_div: ") + hipGetErrorName(e));
    return RT_OK;
}

int rt_udiv(const uint32_t* v, int nv, const uint32_t* d, int nd, uint32_t* q) {
    if (!v || !d || !q || nv < 0 || nd < 0) return fail(RT_ERR_ARG, "bad udiv arguments");
    for (int j = 0; j < nd; ++j)
        if (d[j] == 0) return fail(RT_ERR_ARG, "udiv: divisor 0");
    if (nv == 0 || nd == 0) return RT_OK;
    unsigned* b = nullptr;
    const size_t nq = (size_t)nv * nd;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&b), ((size_t)nv + nd + nq) * sizeof(unsigned)));
    hipError_t e = hipMemcpy(b, v, (size_t)nv * sizeof(unsigned), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(b + nv, d, (size_t)nd * sizeof(unsigned), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = rtc::launch_udiv(b, nv, b + nv, nd, b + nv + nd, nullptr);
    if (e == hipSuccess) e = hipMemcpy(q, b + nv + nd, nq * sizeof(unsigned), hipMemcpyDeviceToHost);
    (void)hipFree(b);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("udiv: ") + hipGetErrorName(e));
    return RT_OK;
}

int rt_unshuffle_stripes(const void* slabs, void* image, int width, int height, int stripe_rows, int nranks,
                         void* stream) {
    if (!slabs || !image || width < 1 || height < 1 || stripe_rows < 1 || nranks < 1)
        return fail(RT_ERR_ARG, "bad unshuffle arguments");
    HIP_TRY(rtk::launch_unshuffle(static_cast<const uint8_t*>(slabs), static_cast<uint8_t*>(image), width, height,
                                  stripe_rows, nranks, rt_slab_rows(height, stripe_rows, nranks),
                                  static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_counters_reset(rt_scene* s, void* stream) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipMemsetAsync(s->d_counters, 0, rtc::kCounters * sizeof(unsigned long long), static_cast<hipStream_t>(stream)));
    return RT_OK;
}

int rt_kernel_times(rt_scene* s, double* ms, int n, int reset) {
    if (!s || !ms || n < 1) return fail(RT_ERR_ARG, "scene/ms is NULL or n < 1");
    for (int i = 0; i < n; ++i) ms[i] = i < rtc::kKKinds ? s->kt_ms[i] : 0.0;
    const int launches = (int)std::min<long long>(INT32_MAX, s->kt_launches);
    if (reset) {
        for (double& v : s->kt_ms) v = 0;
        s->kt_launches = 0;
    }
    return s->ktime ? launches : fail(RT_ERR_ARG, "kernel timing is off (create the scene with RT_KTIME=1)");
}

int rt_counters_read_raw(rt_scene* s, uint64_t* out, int n) {
    if (!s || !out || n < 1) return fail(RT_ERR_ARG, "scene/out is NULL or n < 1");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long c[rtc::kCounters];
    HIP_TRY(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int i = 0; i < n; ++i) out[i] = i < rtc::kCounters ? c[i] : 0;
    return std::min(n, (int)rtc::kCounters);
}

int rt_counters_read(rt_scene* s, rt_stats* st) {
    if (!s || !st) return fail(RT_ERR_ARG, "scene/stats is NULL");
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    unsigned long long c[8];
    HIP_TRY(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    st->primary_rays = c[0]; st->shadow_rays = c[1]; st->reflection_rays = c[2];
    st->node_visits = c[3]; st->tri_tests = c[4]; st->sphere_tests = c[5]; st->shadow_rays_skipped = c[6];
    return check_device_error(s);
}

int rt_set_devices(int n) {
    if (n < 0) return fail(RT_ERR_ARG, "device count must be >= 0");
    if (n >= 1) {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(RT_ERR_NO_DEVICE, "no HIP device visible");
        if (n > count && !(rt_internal_group_virtual() && n <= 16))
            return fail(RT_ERR_ARG, "rt_set_devices(" + std::to_string(n) + "): only " + std::to_string(count) +
                                        " devices visible");
    }
    g_devices.store(n);
    return RT_OK;
}

int rt_scene_num_devices(const rt_scene* s) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    if (s->host_only) return 0;
    return s->group ? rt_internal_group_size(s->group) : 1;
}

int rt_scene_check(rt_scene* s) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    if (s->host_only) return RT_OK;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(hipDeviceSynchronize());
    return check_device_error(s);
}

int rt_render(rt_scene* s, const rt_camera* cam, int aa, uint8_t* out_rgb, rt_stats* stats) {
    if (!s || !out_rgb) return fail(RT_ERR_ARG, "scene/out is NULL");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    int rc = check_camera(cam, aa);
    if (rc) return rc;
    if (s->group) return rt_internal_group_render(s->group, cam, aa, out_rgb, stats);
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipSetDevice(s->device));
    const size_t bytes = (size_t)cam->image_width * cam->image_height * 3;
    if (bytes > s->out_cap) {
        (void)hipFree(s->d_out);
        s->d_out = nullptr;
        s->out_cap = 0;
        HIP_TRY(hipMalloc(reinterpret_cast<void**>(&s->d_out), bytes));
        s->out_cap = bytes;
        HIP_TRY(hipDeviceSynchronize());
        fit_arenas(s);
    }
    const bool count = stats != nullptr;
    if (count) HIP_TRY(hipMemset(s->d_counters, 0, rtc::kCounters * sizeof(unsigned long long)));
    HIP_TRY(hipEventRecord(s->ev0, nullptr));
    rc = rt_render_device(s, cam, aa, cam->image_height, 0, 1, s->d_out, nullptr, count ? RT_RENDER_COUNT : 0);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(s->ev1, nullptr));
    // the error word travels with the frame (one synchronisation instead of two)
    if (!s->h_err) HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->h_err), sizeof(unsigned)));
    HIP_TRY(hipMemcpyAsync(s->h_err, s->d_err, sizeof(unsigned), hipMemcpyDeviceToHost, nullptr));
    HIP_TRY(hipMemcpy(out_rgb, s->d_out, bytes, hipMemcpyDeviceToHost));
    HIP_TRY(hipEventSynchronize(s->ev1));
    if (const unsigned e = *s->h_err) {
        *s->h_err = 0;
        HIP_TRY(hipMemset(s->d_err, 0, sizeof(unsigned)));
        return device_error(e);
    }
    if (stats) {
        rc = rt_counters_read(s, stats);
        if (rc) return rc;
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        stats->kernel_ms = ms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return RT_OK;
}

int rt_primary_hits(rt_scene* s, const rt_camera* cam, int aa, float* t_out, int32_t* m_out) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    int rc = check_camera(cam, aa);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(s->device));
    const int W = cam->image_width * aa, H = cam->image_height * aa;
    const size_t n = (size_t)W * H;
    float* dt = nullptr;
    int* dm = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dt), n * 4));
    if (hipMalloc(reinterpret_cast<void**>(&dm), n * 4) != hipSuccess) {
        (void)hipFree(dt);
        return fail(RT_ERR_HIP, "hipMalloc failed");
    }
    const rtk::Eye eye = make_eye(*cam, W, H);
    hipError_t e = rtk::launch_primary_hits(s->dev, eye, W, H, dt, dm, nullptr);
    if (e == hipSuccess && t_out) e = hipMemcpy(t_out, dt, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && m_out) e = hipMemcpy(m_out, dm, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    (void)hipFree(dt);
    (void)hipFree(dm);
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("primary hits: ") + hipGetErrorName(e));
    return RT_OK;
}

int rt_primary_hits_production(rt_scene* s, const rt_camera* cam, int aa, float* t_out, int32_t* m_out) {
    if (!s) return fail(RT_ERR_ARG, "scene is NULL");
    if (s->host_only) return fail(RT_ERR_NO_DEVICE, "scene was created with RT_OPT_HOST_ONLY");
    int rc = check_camera(cam, aa);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(s->device));
    const int W = cam->image_width * aa, H = cam->image_height * aa;
    const size_t n = (size_t)W * H, out_bytes = (size_t)cam->image_width * cam->image_height * 3;
    char* d = nullptr;             // t, material, then the frame itself
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), 8 * n + out_bytes));
    float* dt = reinterpret_cast<float*>(d);
    int* dm = reinterpret_cast<int*>(d + 4 * n);
    // unset entries read back as NaN / -1: a sample the production kernels never recorded shows up
    hipError_t e = hipMemset(d, 0xff, 8 * n);
    if (e == hipSuccess) {
        s->dbg_t = dt;
        s->dbg_m = dm;
        // the production kernels of one whole frame on this device (rt_render_device's launch sequence; no
        // sub-frame split, whose virtual ranks would index their own slabs)
        rc = render_frame(s, cam, aa, cam->image_height, 0, 1, d + 8 * n, nullptr, 0, 0);
        s->dbg_t = nullptr;
        s->dbg_m = nullptr;
        e = hipDeviceSynchronize();
    }
    if (!rc && e == hipSuccess && t_out) e = hipMemcpy(t_out, dt, n * 4, hipMemcpyDeviceToHost);
    if (!rc && e == hipSuccess && m_out) e = hipMemcpy(m_out, dm, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (rc) return rc;
    if (e != hipSuccess) return fail(RT_ERR_HIP, std::string("primary hits (production): ") + hipGetErrorName(e));
    return check_device_error(s);
}

int rt_downsample_host(const uint8_t* in, int width, int height, int factor, uint8_t* out) {
    // ImageProcessor::downSample (raytracer.cpp:459-484); width/height are the
    // INPUT (internal) dims, output is (width/factor) x (height/factor).
    if (!in || !out || factor < 1 || width < factor || height < factor) return fail(RT_ERR_ARG, "bad downsample args");
    const int nw = width / factor, nh = height / factor, ff = factor * factor;
    for (int i = 0; i < nh; ++i)
        for (int j = 0; j < nw; ++j) {
            int sum[3] = {0, 0, 0};
            for (int k = 0; k < factor; ++k)
                for (int l = 0; l < factor; ++l) {
                    const uint8_t* px = in + ((size_t)(i * factor + k) * width + j * factor + l) * 3;
                    sum[0] += px[0]; sum[1] += px[1]; sum[2] += px[2];
                }
            uint8_t* o = out + ((size_t)i * nw + j) * 3;
            o[0] = (uint8_t)(sum[0] / ff); o[1] = (uint8_t)(sum[1] / ff); o[2] = (uint8_t)(sum[2] / ff);
        }
    return RT_OK;
}

}  // extern "C"

int rt_internal_replicate(const rt_scene* src, int device, rt_scene** out) {
    *out = nullptr;
    rt_scene* s = new (std::nothrow) rt_scene();
    if (!s) return fail(RT_ERR_ARG, "out of host memory");
    s->host = src->host;
    s->bvh = src->bvh;
    s->opt_flags = src->opt_flags;
    const rt_options o{device, src->opt_flags, 0};
    const int rc = upload_scene(s, &o);
    if (rc) {
        delete s;
        return rc;
    }
    s->dev.max_depth = src->dev.max_depth;
    *out = s;
    return RT_OK;
}
