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
    const unsigned f = (unsigned)*lr / (unsigned)p.frame_rows;
    *lr -= (int)(f * (unsigned)p.frame_rows);
    return (int)f;
}

// Slab-local sample slot -> (frame, internal row, column) of its eye ray.  Slots are ordered by 8x8
// internal-pixel tiles (one tile per wave) for ray coherence; slab rows map to global rows through the
// stripe round-robin.  Every quantity is non-negative, so the divisions by the launch's (wave-uniform)
// sizes are unsigned: no sign set-up per divisor, which the walk kernels otherwise kept in SGPRs across
// their loops (and spilled).  P needs: wi tiles_x chunk_row0 chunk_rows aa slab_rows stripe_rows nranks
// rank height nframes frame_rows.
template <class P>
__device__ __forceinline__ bool slab_sample_pos(const P& p, unsigned s, int* frame, int* row, int* col) {
    const unsigned tile = s >> 6, lane = s & 63;
    const unsigned ty = tile / (unsigned)p.tiles_x, tx = tile - ty * (unsigned)p.tiles_x;
    const unsigned ix = tx * 8u + (lane & 7u);
    const unsigned iyc = ty * 8u + (lane >> 3);
    if (ix >= (unsigned)p.wi || iyc >= (unsigned)p.chunk_rows) return false;
    const unsigned iy = (unsigned)p.chunk_row0 + iyc;
    const unsigned lr0 = iy / (unsigned)p.aa;
    const unsigned sub = iy - lr0 * (unsigned)p.aa;
    if (lr0 >= (unsigned)p.slab_rows) return false;
    int lri = (int)lr0;
    *frame = batch_frame(p, &lri);
    const unsigned lr = (unsigned)lri;
    const unsigned stripe = lr / (unsigned)p.stripe_rows;
    const unsigned g = (stripe * (unsigned)p.nranks + (unsigned)p.rank) * (unsigned)p.stripe_rows +
                       (lr - stripe * (unsigned)p.stripe_rows);
    if (g >= (unsigned)p.height) return false;
    *row = (int)(g * (unsigned)p.aa + sub);
    *col = (int)ix;
    return true;
}

// Slab-local sample slot -> eye ray (eyes[0] is the camera of a lone frame too; read per lane from the
// kernel arguments: a kernel that also kept a separate Eye argument live held its 13 words in scalar
// registers, which the walk loops then spilled).
template <class P>
__device__ __forceinline__ bool slab_sample_ray(const P& p, unsigned s, Ray* r) {
    int f, row, col;
    if (!slab_sample_pos(p, s, &f, &row, &col)) return false;
    *r = eye_ray(p.eyes[f], row, col);
    return true;
}

// The internal pixel (frame row, column) whose eye ray slab_sample_ray gives slot s (diagnostics).
template <class P>
__device__ __forceinline__ bool slab_sample_pixel(const P& p, unsigned s, int* row, int* col) {
    int f;
    return slab_sample_pos(p, s, &f, row, col);
}

// Does slot s of the chunk hold a sample of this rank's slab (slab_sample_ray's checks)?
template <class P>
__device__ __forceinline__ bool slab_slot_valid(const P& p, unsigned s) {
    int f, row, col;
    return slab_sample_pos(p, s, &f, &row, &col);
}

// Inverse of the tile ordering: chunk-relative internal pixel -> slot.
__device__ __forceinline__ unsigned slab_slot(int tiles_x, int ix, int iyc) {
    return ((unsigned)((iyc >> 3) * tiles_x + (ix >> 3)) << 6) | (unsigned)((iyc & 7) * 8 + (ix & 7));
}

}  // namespace rtd
