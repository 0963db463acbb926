// Kernel-launch interface between the C-ABI layer (rt_api.cpp) and the HIP
// kernels (pathchain.hip, render_kernels.hip).  Plain structs passed by value as kernel args.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "device_layout.hpp"

namespace rtk {

struct DevScene {
    const dl::Node* nodes;
    const dl::Prim* prims;
    const dl::TriShade* tri_shade;
    const dl::Material* mats;
    const dl::Light* lights;
    int nnodes;
    int nlights;
    int nmats;
    int max_depth;        // MaxRecursionDepth
    int stack_entries;    // LDS traversal-stack entries per thread
    float eps;            // ShadowRayEpsilon
    float bgx, bgy, bgz;  // BackgroundColor as float (raytracer.cpp:446-447)
    float cos_thr;        // smallest float c with (float)(acos(c)*180/3.1415) <= 90.01
    // child-pair layout of the same BVH (traverse2.hpp)
    const dl::Pair* pairs;
    const dl::LeafBig* leaf_big;
    float root_lo[3], root_hi[3];
    int root_info;
    // occlusion tree (host_scene.cpp build_shadow_tree): same leaves, SAH hierarchy above them
    const dl::Pair* spairs;
    float sroot_lo[3], sroot_hi[3];
    int sroot_info;
    int use_stree;        // NaN-free shadow rays walk: 0 the BVH, 1 the binary occlusion tree, 2 its wide form
    int count_prod;       // counting passes walk the production trees and count fetched BYTES in the node
                          // counter (bench.py roofline; RT_COUNT_PROD at scene creation)
    const dl::Wide* swnodes;  // the occlusion tree in wide form (any hit)
    const float4* lrec;   // leaf records (dl::LeafHead + prims), indexed in 16-B units
    int swroot;
    const dl::Wide* wnodes;  // the reference tree in wide form (closest hit, reference order)
    int wroot;
    int use_wide;         // NaN-free closest-hit rays walk wnodes (traverse2.hpp wide_closest_step)
    int leaf_wait_any;    // the same for any-hit walks (RT_LEAF_WAIT_ANY)
    unsigned* err;        // device error word (bit 0: a walk exceeded walk_cap; bit 1: a wait loop exceeded
                          // spin_cap), read by the host after renders
    int walk_cap;         // always-on bound on one walk's step calls (traverse2.hpp walk_runaway)
    int spin_cap;         // always-on bound on the iterations of a loop that waits on other lanes or waves
                          // without progress (pathchain.hip spin_over; RT_SPIN_CAP overrides)
    int leaf_wait;        // 4-wide walks: a lane at a leaf record waits while fewer than leaf_wait/64 of the
                          // wave's walking lanes are at one (0: never waits; RT_LEAF_WAIT)
    int cull_shadows;     // chain path: shadow rays that cannot change the pixel are not traced
                          // (pathchain.hip light_needed; every material's kd finite; RT_CULL=0 disables)
    int force_fb;         // tests (RT_FORCE_FALLBACK): the timed chain kernels defer every closest-hit (bit 0),
                          // any-hit (bit 1) and/or reflected closest-hit (bit 2) ray to k_fallback

    // Sphere prims carry ~sphere_index in p0.w (negative), triangles their id.
    __device__ __forceinline__ bool prim_is_sphere(int, const float4 p0) const {
        return __float_as_int(p0.w) < 0;
    }
};

// EyeRayGenerator state (raytracer.cpp:287-288), computed on host in fp32.
struct Eye {
    float qx, qy, qz, ux, uy, uz, vx, vy, vz, ex, ey, ez;
    float su, sv;   // suMultiplier, svMultiplier for the INTERNAL resolution
};

struct FrameParams {
    int width, height;    // OUTPUT image
    int aa;               // SSAA factor F (internal = F*W x F*H)
    int stripe_rows;      // output rows per stripe
    int rank, nranks;     // stripe round-robin
    int slab_rows;        // rows in this rank's slab
    uint8_t* out;         // slab_rows * width * 3
    int out_k = 1, out_j = 0;   // chain path: sub-frame j of out_k interleaved sub-frames (pathchain.hip out_row)
    int chunk_k = 1, chunk_j = 0;   // chain path: this call renders sample chunks j, j+k, ... of the frame
    unsigned long long* counters;  // 6 x u64 (RT_RENDER_COUNT)
    // chain path, frame batches (rt_render_frames_device): slab_rows = nframes * frame_rows virtual
    // rows, frame f's rows rendered with eyes[f] into outs[f] (host arrays of nframes entries)
    int nframes = 1, frame_rows = 0;
    const Eye* eyes = nullptr;
    uint8_t* const* outs = nullptr;
};

hipError_t launch_primary_hits(const DevScene& s, const Eye& e, int W, int H, float* t, int* m, hipStream_t stream);
hipError_t launch_unshuffle(const uint8_t* slabs, uint8_t* img, int width, int height, int stripe_rows, int nranks,
                            int slab_rows, hipStream_t stream);

}  // namespace rtk
