// Wavefront (queue-per-bounce) renderer: the hot path split into small
// kernels per recursion level so each traversal kernel carries only its own
// state (low VGPR count -> high occupancy) and works on a compacted queue of
// live rays (SIMD lanes stay busy as paths terminate).
//
//   per chunk of level-0 samples (8x8-pixel tiles, one tile per wave):
//     for level k = 0..max_depth:
//       k_trace   closest-hit of queue k (level 0: eye rays generated in place),
//                 writes the hit record and appends one shadow ray per light
//       k_shadow  any-hit of the shadow queue -> occlusion bytes
//       k_shade   Blinn-Phong with the occlusion bytes; mirror hits append
//                 their reflection ray to queue k+1 and link it as child
//     k_fold     levels max_depth-1..1, deepest first: c = clamp(L + c_child*km)
//     k_resolve  level-0 fold + toPixel + SSAA integer box filter -> u8 slab
//
// The fold reproduces the reference's recursive evaluation order exactly
// (raytracer.cpp:436-451): each level's value is formed only after its child's.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "render_kernels.hpp"

namespace rtw {

struct WfParams {
    // frame -> slab mapping (same as rtk::FrameParams)
    int width, height, aa, stripe_rows, rank, nranks, slab_rows;
    int wi;           // internal width (width * aa)
    int tiles_x;      // ceil(wi / 8)
    int chunk_row0;   // first slab-local internal row of this chunk (multiple of 8*aa)
    int chunk_rows;   // slab-local internal rows in this chunk
    int n0;           // level-0 sample slots: tiles_x * ceil(chunk_rows/8) * 64
    int cap;          // per-level entry capacity (>= n0)
    int nlights;
    // workspace
    float4* q[2];      // ray queues (2 x float4 per ray: {o, 0}, {d, 0}); q[k&1] is level k's input
    float4* hit;       // 2 x float4 per entry: {p.xyz, mat}, {n.xyz, t}; mat = 0 -> no hit / invalid
    float4* sray;      // 2 x float4 per shadow ray: {p.xyz, owner*nl+l}, {ldir.xyz, dist}
    uint8_t* occ;      // [cap * nlights] shadow result per (entry, light)
    float4* R;         // [levels][cap] {L or c .xyz, mat}; mat = 0 -> value is final
    int* child;        // [levels][cap] reflection child slot at level+1, -1 none, -2 beyond max depth
    unsigned* qcount;  // [levels + 1] entries per level (level 0 unused)
    unsigned* scount;  // [levels] shadow rays per level
    uint8_t* out;      // slab (slab_rows * width * 3)
    unsigned long long* counters;
};

hipError_t launch_frame_chunk(const rtk::DevScene& s, const rtk::Eye& e, const WfParams& p, int grid_blocks,
                              bool count, hipStream_t stream);

}  // namespace rtw
