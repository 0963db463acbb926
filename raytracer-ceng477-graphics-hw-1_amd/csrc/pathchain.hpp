// "Chain" renderer (default path): per-pixel closest-hit chains in one
// kernel, shadow rays and shading deferred to the two kernels after it.
//
// Why: the frame time of this workload is set by its slowest pixels, not by
// throughput (a single 1x1 crop of the C3 frame's heaviest pixel takes ~1/3 of
// the whole frame).  A pixel's mirror chain is inherently serial (each bounce
// needs the previous hit), but its shadow rays are not: the reflection ray
// does not depend on occlusion.  So
//   k_chain    one lane per sample: eye ray -> closest hit -> record the hit
//              -> append one shadow ray per light to a queue -> reflect ->
//              closest hit ... (no shading, no shadow traversal on the chain)
//   k_occlude  any-hit over the shadow queue, fully parallel
//   k_finish   per output pixel: per sample, shade every recorded level with
//              the occlusion bytes and fold deepest-first
//              c_k = clamp(L_k + c_{k+1} (x) km_k) (raytracer.cpp:385-452),
//              toPixel, SSAA integer box filter
// The critical path becomes one closest-hit chain plus one shadow ray.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "render_kernels.hpp"

namespace rtc {

constexpr int kMaxChainGrid = 1280;   // k_chain workgroups (= task-queue regions; 5 per CU on 256 CUs): the
                                      // consumers' LDS region prefix (pathchain.hip g_pref) holds this many
constexpr int kMaxFrames = 32;        // frames of one batched launch (PcParams kernarg: 64 B each) (rt_render_frames_device)
#ifndef RT_BQ
#define RT_BQ 1536
#endif
constexpr int kMaxBq = RT_BQ;   // phase-B workgroup shadow queue (LDS slots, pathchain.hip)
// Diagnostics build (RT_TRACE_BUILD=1, tools/trace_report.py): the chain kernels record wall-clock
// timings per sample, continuation and shadow workgroup into PcParams::trace (env RT_TRACE names the
// dump).  Off in the product build: its counters cost the walk kernels registers.
#ifndef RT_TRACE_BUILD
#define RT_TRACE_BUILD 0
#endif
constexpr bool kTraceBuild = RT_TRACE_BUILD != 0;
// Shadow walks with the wave leaf queue (pathchain.hip occlude_queue_body), the only walker that reads
// task regions in place (PcParams::occ_inplace / occ_inplace_b): the host enables those only when it is
// built.
#ifndef RT_LEAF_QUEUE
#define RT_LEAF_QUEUE 1
#endif

enum PathKind : int {
    kEndBg = 0,     // deepest ray missed at depth 0: background
    kEndZero = 1,   // deepest ray missed at depth > 0, or beyond MaxRecursionDepth: black
    kEndLast = 2,   // last recorded hit is not a mirror: its own clamp(L)
    kEndTail = 3,   // levels >= nlev were finished by k_fallback: their folded colour is tail[path]
};
// k_fallback chain entries: the record id whose reflected ray was deferred, or kFbEye | sample for a
// deferred eye ray
constexpr unsigned kFbEye = 0x80000000u;
// occlusion byte of a deferred shadow task whose fallback-queue slot overflowed (k_fallback scans for it)
constexpr uint8_t kOccDeferred = 2;
// pinfo bit of a path continued in phase B (set by phase A's hand-off, kept by phase B's end)
constexpr int kPathCont = 1 << 16;

// Device counter block (u64 slots, RT_RENDER_COUNT launches).  0-6 are rt_stats' (primary, shadow,
// reflection, node visits, triangle tests, sphere tests, skipped shadow rays); the per-role slots
// split the walks by the kernel role that runs them in the timed path, so a production-fetch
// counting pass (RT_COUNT_PROD: "node visits" = fetched bytes) gives each kernel its own bytes.
constexpr int kCounters = 32;
enum CounterSlot : int {
    kCntAWalkBytes = 8,   // phase A closest-hit walks (k_chain)
    kCntAWalks,           //   walks started in phase A (primary + level-1 reflections)
    kCntAHits,            //   their hits (records written)
    kCntBWalkBytes,       // phase B closest-hit walks (k_mix chain role)
    kCntBWalks,
    kCntBHits,
    kCntConts,            // continuations handed from A to B
    kCntASBytes,          // A's shadow rays (k_mix shadow role for one frame; k_occlude in frame batches)
    kCntASRays,
    kCntBQBytes,          // B's shadow rays walked from the workgroup LDS queue (k_mix chain role)
    kCntBQRays,
    kCntBOBytes,          // B's shadow rays that overflowed to k_occlude
    kCntBORays,
    // every launch (timed or counting), added by k_fallback: what the timed walks left to it
    kCntFbLaunches = 24,  // chain launches
    kCntFbConts,          //   continuations handed from A to B (all of them)
    kCntFbContOvf,        //   of those, beyond the phase-B record space (cb): walked whole by k_fallback
    kCntFbChains,         //   closest-hit rays deferred (not in range of the wide trees' slab test)
    kCntFbShadows,        //   shadow rays deferred
    kCntFbOvfScans,       //   launches whose fallback shadow queue overflowed (occlusion bytes scanned)
    kCntCompactLaunches,  // chain launches with compact (16-B) phase-A records (PcParams::clevels > 0)
};

// Phase-A levels whose records may leave out the direction (PcParams::dbase): k_finish rebuilds them
// forward from the eye ray, one reflection per level.
#ifndef RT_COMPACT_LEVELS
#define RT_COMPACT_LEVELS 2
#endif
constexpr int kCompactLevels = RT_COMPACT_LEVELS;
// Phase-A unit u's column-order unit (pathchain.hip unit_order): the 256-sample units of a launch dealt
// in blocks ublk_w units wide and ublk_h rows high (-1: a frame high), so the units in flight cover a
// column of the image; identity when ublk_h == 0 or the units do not tile the rows.  Host and device
// (the host makes lone frames' column-order table, PcParams::ucol).
__host__ __device__ inline unsigned unit_col(int tiles_x, int ublk_h, int ublk_w, int nframes, unsigned u,
                                             unsigned units) {
    const unsigned upr = (unsigned)tiles_x / 4u;
    if (ublk_h == 0 || (tiles_x & 3) || units % upr) return u;
    const unsigned rows = units / upr, bw = (unsigned)ublk_w;
    const unsigned bh = ublk_h > 0 ? (unsigned)ublk_h : (rows % (unsigned)nframes ? rows : rows / (unsigned)nframes);
    const unsigned r0 = u / (bh * upr) * bh, h = bh < rows - r0 ? bh : rows - r0;
    const unsigned i = u - r0 * upr;            // index within the super-row (h rows x upr units)
    const unsigned c0 = i / (h * bw) * bw, w = bw < upr - c0 ? bw : upr - c0;
    const unsigned l = i - c0 * h;
    return (r0 + l / w) * upr + c0 + l % w;
}

// PcParams::totals words: task counts (0-2), the phase-A unit counter (3), k_fallback's chain /
// shadow counts and shadow-queue overflow (4-6), the rest spare.
constexpr int kTotalsWords = 12;

// Unit cost classes (PcParams::ucost): the most phase-A walk steps a sample of the unit took.
// Classes 0..5: at least kHotSteps[c] steps; class kUnitClasses - 1: the rest (and units no sample of which
// reached kHotSteps[5], which k_chain does not mark).
constexpr int kUnitClasses = 7;
#ifndef RT_HOT_MIN
#define RT_HOT_MIN 32     // (48 with the mixed deal: one frame +0.6 %, profiles/r06_mix_ab.jsonl)
#endif
constexpr unsigned kHotSteps[kUnitClasses - 1] = {224, 160, 128, 96, 64, RT_HOT_MIN};

struct PcParams {
    int width, height, aa, stripe_rows, rank, nranks, slab_rows;
    int wi, tiles_x, chunk_row0, chunk_rows, n0;
    int cap;          // path slots per chunk (>= n0)
    int levels;       // max_depth + 1 (>= 1)
    int nlights;
    // Hit records (pathchain.hip rec_write), by record id (rec_id): levels [0, la) of every sample
    // at k * cap + sample (phase A), deeper levels only for the first cb continuations, at
    // la * cap + (k - la) * cb + c for continuation c (phase B); occlusion bytes by record id * nl.
    // rec[id] = {hit point, surface code} for every record; recd[id - dbase] = {ray direction,
    // material} only for ids >= dbase (the chain path: dbase = la * cap, phase A's records rebuild
    // their directions from the eye ray; the fused path: dbase = 0).
    float4* rec;
    float4* recd;
    unsigned dbase;   // clevels * cap: records below it have no direction word
    int clevels;      // min(la, kCompactLevels) levels of every sample without direction words (0: none)
    int* pinfo;       // [cap]: nlev | kind << 8 | kPathCont
    uint8_t* occ;
    int la;           // levels stored for every sample (phase A's; all levels on the fused path)
    unsigned cb;      // continuations with records (the rest finish in k_fallback)
    unsigned* cid;    // [cap]: continuation index of a continued sample (k_pack_a; a lone frame's k_mix at its grab)
    float4* tail;     // [cap]: folded colour of the levels k_fallback finished (kEndTail)
    // k_fallback's work: rays the timed walks do not take (NaN-free and in range for the wide trees'
    // fused slab test, wide_walk_ok) and continuations beyond cb.  fbc: chain entries (kFbEye | sample
    // or the record id whose reflection was deferred), totals[4] of them; fbs: shadow task owner ids,
    // totals[5] of them, overflow flagged in totals[6] (the task's occlusion byte then kOccDeferred)
    unsigned* fbc;
    unsigned fbc_cap;
    unsigned* fbs;
    unsigned fbs_cap;
    int fb_grid;      // k_fallback workgroups
    // phase A (k_chain: levels [0, kinline]) and phase B (k_mix chain role: deeper levels).
    // Task queues hold u32 owner ids in per-workgroup regions with their counts.  Phase A's are packed by
    // k_pack_a (continuations: cflat; a lone frame's chunks' shadow tasks: sflatA), walked region by region
    // (frame batches' shadow tasks), or read as one list in region order (a whole lone frame, PcParams::rlists,
    // pathchain.hip region_prefix); phase B's overflow is packed by k_pack_b in frame batches.
    unsigned* sqA;    // shadow tasks of A: [grid][scapA], owner = (level*cap + sample)*nl + light
    unsigned scapA;
    unsigned* scntA;  // [grid]
    unsigned* sflatA; // the chunks of a lone frame: A's shadow tasks packed in region order (k_pack_a), totals[0]
    unsigned* cq;     // continuations of A: [grid][ccapA], owner = level*cap + sample of the last record
    unsigned ccapA;
    unsigned* ccnt;   // [grid]
    unsigned* cflat;  // continuations packed in region order (k_pack_a; a lone frame's k_mix / k_fallback at their
                      // grab), totals[1] of them
    unsigned* sqB;    // shadow tasks of B: [gb][scapB]
    unsigned scapB;
    unsigned* scntB;  // [gb]
    unsigned* sflatB; // B's shadow tasks packed (k_pack_b), totals[2] of them
    unsigned* totals; // [kTotalsWords]: task counts (0: A's packed shadow tasks; 1: A's continuations, k_pack_a /
                      // k_mix; 2: B's packed overflow), the phase-A unit counter, k_fallback chains / shadows /
                      // overflow
    int kinline;      // deepest level phase A walks (>= max_depth: no phase B)
    int gb;           // k_mix workgroups in the chain role (the other p.ogrid ones occlude A's tasks)
    int tchunk;       // continuation tasks (phase B) are dealt to workgroups in chunks of this many
    int ochunk;       // ... and shadow tasks (k_mix occlusion role, k_occlude) in chunks of this many
    int lq_wait;      // leaf-queue walks: test the queued records once this many lanes wait on them (RT_LQ_WAIT)
    int grid;         // k_chain persistent grid (= number of shadow-queue regions)
    int ogrid;        // k_occlude persistent grid
    int split_occ;    // 1: A's shadow tasks in their own k_occlude launch (occ_grid workgroups), not in k_mix
    int occ_grid;     // resident k_occlude workgroups
    // Lone frames' phase-A units, the previous frame's heaviest first (rt_api.cpp render_chain,
    // hot_units): k_chain records per unit the most walk steps a sample of it took (ucost: samples of at
    // least kHotSteps[5] only, atomicMax), k_mix's last shadow-role workgroup ranks the units into uorder by
    // that cost's class (kHotSteps, heaviest first; each class in the column order) and clears ucost; the
    // next frame of the same geometry deals its units in that order (uorder_on).  Where the work goes,
    // never what it computes.
    unsigned* ucost;
    unsigned* uorder;
    const unsigned* ucol;   // [units]: unit_col of 0, 1, ... (rank_units reads it instead of dividing)
    int urank, uorder_on;
    int occ_inplace_b;  // 1 (lone-frame production launches): k_occlude walks B's LDS-queue overflow in its
                        // phase-B regions (no k_pack_b)
    int occ_inplace;  // 1 (split_occ production launches): k_occlude walks A's shadow tasks in their phase-A
                      // regions (workgroup w: regions w, w + G, ...); k_pack_a packs only the continuations
    int fin_grid;     // k_finish workgroups at most (0: a lane per output pixel), a grid-stride loop beyond
    int fin_cont;     // k_finish: the continued paths' pixels first (chain path: the continuation list, kPathCont)
    int refill;       // a wave refills once <= refill of its lanes are still walking
    int orefill;      // the same for the shadow (any-hit) walks
    int brefill;      // the same for phase-B chains
    int bprio;        // 1: phase-B chain waves run at the highest issue priority
    int service;      // ... or once >= service of its lanes finished a walk (epilogue, next bounce)
    int bservice;     // the same for phase-B chains
    int btail;        // phase-B chains once no continuation is left to take: service at this many done lanes
    int bq_cap;       // phase-B workgroup shadow queue slots in use (<= kBq; 0: every task to k_occlude)
    int dyn_units;    // > 0: phase-A waves take 256-sample units from a launch-wide counter (totals[3]),
                      // at most this many per workgroup; 0: static per-workgroup interleave
    int ublk_h, ublk_w; // dynamic units taken in column blocks of ublk_h tile rows (< 0: a frame; 0: off)
                        // x ublk_w units (unit_order)
    uint8_t* out;
    // Frame batch: the slab's rows are nframes frames of frame_rows rows each (slab_rows = nframes *
    // frame_rows); frame f's samples use eyes[f] and its pixels go to fouts[f] (nframes > 1 only).
    int nframes, frame_rows;
    rtk::Eye eyes[kMaxFrames];
    uint8_t* fouts[kMaxFrames];
    int out_k, out_j;   // sub-frame j of k interleaved sub-frames (out_row); 1, 0 for a whole frame
    unsigned long long* counters;
    unsigned* trace;  // diagnostics (RT_TRACE): [cap][2] sample {grab, chain end}, then [trace_blocks][2]
                      // k_occlude workgroup {start, end}, then [cap][4] phase-B continuation {grab, end,
                      // last level, walk steps}; wall clock; or null
    int trace_blocks;
    // (new fields at the end: kernel arguments are loaded in runs of neighbours, so a field inserted
    // among the walk kernels' ones changed their SGPR spills 28 -> 67)
    unsigned* cont_peak;  // frames of several chunks: the most continuations of one chunk (k_mix / k_pack_a, atomicMax)
    // Diagnostics (rt_primary_hits_production): each sample's level-0 closest hit as the TIMED walk found it
    // -- tSmall (-1 on a miss) and material id (0 on a miss) at internal pixel row * wi + col -- written by
    // k_chain<false, true> (the production kernel with these two stores added) and, for an eye ray the
    // timed walks defer, by k_fallback.  Null in every other launch.
    float* dbg_t;
    int* dbg_m;
    // Lone frames' mixed deal (rank_units, unit_order): the units of the mix_cls heaviest cost classes ("hot")
    // are dealt first, each in a group with G - 1 of the lightest units, the group's 64-sample wave chunks
    // holding 64 / G samples (whole 8-pixel rows) of the hot unit and the rest of the light ones, so that no
    // wave starts with more than 64 / G heavy walks.  ugrp[g * G + 0] = group g's hot unit, [g * G + 1 + j] its
    // light ones; uorder holds kUidMix codes for the groups' virtual units.  mix_cls: bits 0-7 the classes
    // (0: off), bits 8-9 log2 G (0: from the hot-unit count and the grid, at most 8 hot rows per wave).
    unsigned* ugrp;
    int mix_cls;
    int rlists;       // 1: a whole lone frame -- k_mix reads phase A's lists in their regions (pathchain.hip
                      // region_prefix) and stores cflat / cid itself; 0: k_pack_a packs them (cflat, and sflatA
                      // where A's shadow tasks are not walked in place)
    // Frame batches' deep-first deal: pdepth[sample slot] = the levels its chain reached in the slot's previous
    // launch of this geometry (k_mix, at the chain's end); k_chain queues a continuation whose pdepth >= deep_min
    // at its region's end (ccntd counts them) and k_pack_a packs those first, so k_mix starts the deep chains first.
    // Null: off.  Where work runs, never what it computes.
    uint8_t* pdepth;
    unsigned* ccntd;
    int deep_min;
};

// Worst-case task-queue slots per workgroup: every sample of the workgroup
// recording `levels` levels, one task per light.
unsigned chain_block_scap(int n0, int grid, int levels, int nlights);
// A workgroup's static share of 256-sample units (k_chain with PcParams::dyn_units = 0).
unsigned chain_block_units(int n0, int grid);
// Dynamic phase-A units: most units one k_chain workgroup may take (its LDS unit table).
constexpr int kDynUnits = 128;

// Resident workgroups per CU of the (non-counting) k_chain / k_mix / k_occlude:
// the persistent grids are sized so every workgroup starts at t = 0 (a late-
// starting workgroup that owns slow pixels would stretch the frame).
hipError_t chain_occupancy(int* chain_blocks_per_cu, int* mix_blocks_per_cu, int* occlude_blocks_per_cu);

// Diagnostics: phong_pow on the device (rt_phong_pow).
hipError_t launch_phong_pow(const float* base, const float* expo, float* out, int n, hipStream_t st);
// Diagnostics: the triangle test's Cramer quotients on the device (rt_cramer_div).
hipError_t launch_cramer_div(const float* den, const float* num, float* out, int n, hipStream_t st);
// Diagnostics: the leaf-queue walker's uniform-divisor division on the device (rt_udiv).
hipError_t launch_udiv(const unsigned* v, int nv, const unsigned* d, int nd, unsigned* q, hipStream_t st);
// Diagnostics: dependent-step latency of single closest-hit walks (rt_walk_timing).
hipError_t launch_walk_timing(const rtk::DevScene& s, const float* rays, int n, int lanes, int reps, int mode,
                              unsigned long long* out, hipStream_t st);

// Diagnostics (RT_KTIME=1 scenes, rt_kernel_times): each kernel of a chain launch is launched with
// hipExtLaunchKernel's start / stop events, which take the dispatch's own begin and end timestamps
// (what rocprofv3 --kernel-trace reports), so the host can split the launch's time per kernel without
// markers between the kernels (round 5's inter-kernel events read 23 % above rocprof's kernel sums).
enum KernelKind : int { kKChain = 0, kKPackA, kKMix, kKOccA, kKPackB, kKOccB, kKFinish, kKFallback, kKKinds };
struct KTimer {
    static constexpr int kMax = 16;
    hipEvent_t ev0[kMax] = {}, ev1[kMax] = {};
    int kind[kMax] = {};
    int n = 0;
    // the next kernel's start / stop events (both null once full or not created)
    void take(int k, hipEvent_t* a, hipEvent_t* b) {
        if (n < kMax && ev0[n] && ev1[n]) {
            kind[n] = k;
            *a = ev0[n];
            *b = ev1[n++];
        }
    }
};

hipError_t launch_chain_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, bool count,
                              hipStream_t stream, KTimer* kt = nullptr);

}  // namespace rtc
