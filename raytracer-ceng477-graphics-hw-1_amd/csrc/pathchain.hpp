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
//   k_compose  per output pixel: per sample, shade every recorded level with
//              the occlusion bytes and fold deepest-first
//              c_k = clamp(L_k + c_{k+1} (x) km_k) (raytracer.cpp:385-452),
//              toPixel, SSAA integer box filter
// The critical path becomes one closest-hit chain plus one shadow ray.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "render_kernels.hpp"

namespace rtc {

enum PathKind : int {
    kEndBg = 0,     // deepest ray missed at depth 0: background
    kEndZero = 1,   // deepest ray missed at depth > 0, or beyond MaxRecursionDepth: black
    kEndLast = 2,   // last recorded hit is not a mirror: its own clamp(L)
};

struct PcParams {
    int width, height, aa, stripe_rows, rank, nranks, slab_rows;
    int wi, tiles_x, chunk_row0, chunk_rows, n0;
    int cap;          // path slots per chunk (>= n0)
    int levels;       // max_depth + 1 (>= 1)
    int nlights;
    float4* rec;      // [levels][cap][3]: {hitp.xyz, mat}, {n.xyz, t}, {d.xyz, 0}
    int* pinfo;       // [cap]: nlev | kind << 8
    float4* sray;     // [scap][2]: {p.xyz, owner}, {ldir.xyz, dist}; owner = (level*cap+path)*nl + l
    uint8_t* occ;     // [levels][cap][nl]
    unsigned* scount; // shadow rays appended
    unsigned scap;    // shadow queue capacity
    uint8_t* out;
    unsigned long long* counters;
};

hipError_t launch_chain_chunk(const rtk::DevScene& s, const rtk::Eye& e, const PcParams& p, int grid_blocks,
                              bool count, hipStream_t stream);

}  // namespace rtc
