// Wave-level helpers (wave64) and the slab-sample -> eye-ray mapping shared by
// the multi-kernel render paths.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "traverse.hpp"

namespace rtd {

// Wave-aggregated append: one atomic per wave; lanes with `pred` get
// consecutive groups of `mult` slots.  Every active lane must reach it.
__device__ __forceinline__ unsigned wave_append(unsigned* counter, bool pred, unsigned mult) {
    const unsigned long long m = __ballot(pred);
    if (m == 0) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((unsigned long long)m) - 1;
    unsigned base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(m) * mult);
    base = __shfl(base, leader, 64);
    return base + (unsigned)__popcll(m & ((1ull << lane) - 1ull)) * mult;
}

template <typename T>
__device__ __forceinline__ T wave_sum64(T v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Sum over the wave, one atomic by lane 0.  Must be reached by all 64 lanes.
__device__ __forceinline__ void wave_add_counter(unsigned long long* c, unsigned long long v) {
    v = wave_sum64(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(c, v);
}

// Frame batches: virtual slab row lr -> frame index, *lr -> that frame's slab row.
template <class P>
__device__ __forceinline__ int batch_frame(const P& p, int* lr) {
    if (p.nframes <= 1) return 0;
    const int f = *lr / p.frame_rows;
    *lr -= f * p.frame_rows;
    return f;
}

// Slab-local sample slot -> eye ray.  Slots are ordered by 8x8 internal-pixel
// tiles (one tile per wave) for ray coherence; slab rows map to global rows
// through the stripe round-robin.  P needs: wi tiles_x chunk_row0 chunk_rows
// aa slab_rows stripe_rows nranks rank height nframes frame_rows eyes, with
// eyes[0] the camera of a lone frame too (read per lane from the kernel
// arguments: a kernel that also kept a separate Eye argument live held its
// 13 words in scalar registers, which the walk loops then spilled).
template <class P>
__device__ __forceinline__ bool slab_sample_ray(const P& p, unsigned s, Ray* r) {
    const unsigned tile = s >> 6, lane = s & 63;
    const int tx = (int)(tile % (unsigned)p.tiles_x), ty = (int)(tile / (unsigned)p.tiles_x);
    const int ix = tx * 8 + (int)(lane & 7);
    const int iyc = ty * 8 + (int)(lane >> 3);
    if (ix >= p.wi || iyc >= p.chunk_rows) return false;
    const int iy = p.chunk_row0 + iyc;
    int lr = iy / p.aa;
    const int sub = iy - lr * p.aa;
    if (lr >= p.slab_rows) return false;
    const int f = batch_frame(p, &lr);
    const int stripe = lr / p.stripe_rows;
    const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows);
    if (g >= p.height) return false;
    *r = eye_ray(p.eyes[f], g * p.aa + sub, ix);
    return true;
}

// The internal pixel (frame row, column) whose eye ray slab_sample_ray gives slot s (diagnostics).
template <class P>
__device__ __forceinline__ bool slab_sample_pixel(const P& p, unsigned s, int* row, int* col) {
    const unsigned tile = s >> 6, lane = s & 63;
    const int tx = (int)(tile % (unsigned)p.tiles_x), ty = (int)(tile / (unsigned)p.tiles_x);
    const int ix = tx * 8 + (int)(lane & 7);
    const int iyc = ty * 8 + (int)(lane >> 3);
    if (ix >= p.wi || iyc >= p.chunk_rows) return false;
    const int iy = p.chunk_row0 + iyc;
    int lr = iy / p.aa;
    const int sub = iy - lr * p.aa;
    if (lr >= p.slab_rows) return false;
    batch_frame(p, &lr);
    const int stripe = lr / p.stripe_rows;
    const int g = (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows);
    if (g >= p.height) return false;
    *row = g * p.aa + sub;
    *col = ix;
    return true;
}

// Does slot s of the chunk hold a sample of this rank's slab (slab_sample_ray's checks)?
template <class P>
__device__ __forceinline__ bool slab_slot_valid(const P& p, unsigned s) {
    const unsigned tile = s >> 6, lane = s & 63;
    const int tx = (int)(tile % (unsigned)p.tiles_x), ty = (int)(tile / (unsigned)p.tiles_x);
    const int ix = tx * 8 + (int)(lane & 7);
    const int iyc = ty * 8 + (int)(lane >> 3);
    if (ix >= p.wi || iyc >= p.chunk_rows) return false;
    int lr = (p.chunk_row0 + iyc) / p.aa;
    if (lr >= p.slab_rows) return false;
    batch_frame(p, &lr);
    const int stripe = lr / p.stripe_rows;
    return (stripe * p.nranks + p.rank) * p.stripe_rows + (lr - stripe * p.stripe_rows) < p.height;
}

// Inverse of the tile ordering: chunk-relative internal pixel -> slot.
__device__ __forceinline__ unsigned slab_slot(int tiles_x, int ix, int iyc) {
    return ((unsigned)((iyc >> 3) * tiles_x + (ix >> 3)) << 6) | (unsigned)((iyc & 7) * 8 + (ix & 7));
}

}  // namespace rtd
