// Device (HBM) layout of a scene — shared by host flattener and HIP kernels.
//
//   Node  32 B  (one 32-B sector, two dwordx4 loads)   — 50 079 nodes for horse_and_mug = 1.6 MB
//     interior: {bmin.xyz, right child index} {bmax.xyz, axis}
//     leaf:     {bmin.xyz, first prim}        {bmax.xyz, LEAF | nsph<<20 | ntri}
//     left child of node i is i+1 (pre-order, bvh.h:81-105)
//   Prim  48 B  leaf-contiguous primitive copies (bvh.h:43-44 leaves own copies),
//               triangles first then spheres, in the reference's leaf order
//     triangle: {a.xyz, tri id} {a-b .xyz, 0} {a-c .xyz, 0}
//               (a-b, a-c are exactly the float differences Cramer's rule
//                forms at raytracer.cpp:135-160, so precomputing them is exact)
//     sphere:   {c.xyz, sphere id} {r, r*r, 0, 0} {0, 0, 0, material id}
//   TriShade 16 B per triangle id: {normal.xyz, material id}  (winner only)
//   Material 64 B: {ka*Ia .xyz, phong} {kd.xyz, is_mirror} {ks.xyz, 0} {km.xyz, 0}
//   Light    32 B: {pos.xyz, 0} {intensity.xyz, 0}
#pragma once
#include <cstdint>

namespace dl {

constexpr int32_t kLeafBit = (int32_t)0x80000000u;
constexpr int kNtriBits = 20;
constexpr int32_t kNtriMask = (1 << kNtriBits) - 1;
constexpr int kMaxLeafSpheres = (1 << 11) - 1;
constexpr int kMaxStack = 64;   // traversal stack entries (BVH depth cap 19 -> <= 20 used; wide walks: host-checked)

struct alignas(16) Node {
    float minx, miny, minz; int32_t a;
    float maxx, maxy, maxz; int32_t b;
};

struct alignas(16) Prim {
    float p0x, p0y, p0z; int32_t id;
    float p1x, p1y, p1z; float p1w;
    float p2x, p2y, p2z; int32_t p2w;
};

struct alignas(16) TriShade { float nx, ny, nz; int32_t material; };

struct alignas(16) Material {
    float kax, kay, kaz, phong;     // ambient reflectance * ambient light (raytracer.cpp:394)
    float kdx, kdy, kdz; int32_t is_mirror;
    float ksx, ksy, ksz, pad0;
    float kmx, kmy, kmz, pad1;
};

struct alignas(16) Light {
    float px, py, pz, pad0;
    float ix, iy, iz, pad1;
};

// Child-pair layout ("children in parent", 64 B = one load per expansion):
// pair p holds the boxes of BOTH children of interior node N plus N's split
// axis, so expanding N tests both child boxes from one 64-B record and a
// miss never costs a dependent load.  Child info word:
//   >= 0          interior child: index of ITS child pair
//   kLeafBit | count << 25 | start      leaf child, count in [1, 63]
//   kLeafBit | 0 << 25 | big           leaf child with > 63 prims: LeafBig[big]
// Leaves keep the reference's primitive order (triangles, then spheres).
struct alignas(16) Pair {
    float l_minx, l_miny, l_minz; int32_t l_info;    // left child  (node i+1)
    float l_maxx, l_maxy, l_maxz; int32_t axis;      // parent's split axis
    float r_minx, r_miny, r_minz; int32_t r_info;    // right child (rightIndex)
    float r_maxx, r_maxy, r_maxz; int32_t pad;
};
struct LeafBig { int32_t start, count; };

// Leaves of the wide trees are the reference BVH's leaves.  A leaf record is
// the leaf's header (its EXACT box, tested exactly before the primitives)
// followed by copies of its primitives, so the box and the first primitive
// arrive in one round trip:
//   LeafHead {lo.xyz, count} {hi.xyz, slot0}   slot0 = Prim[] index of the first primitive
//   count x Prim (48 B, same encoding and order as Prim[])
// Wide node, 128 B = one L2 line, up to kWideSlots = 6 children.  Two trees
// use it: the reference BVH collapsed in reference order (closest-hit walks,
// host_scene.cpp build_ref_wide) and the SAH occlusion tree collapsed
// (any-hit walks, build_shadow_tree).
//   dw 0-3    {origin.xyz, exps}  exps = ex | ey << 8 | ez << 16 | slot mask << 24, scale_a = 2^(e_a - 127)
//   dw 4-21   child planes as fp16 offsets, dword (side * 9 + axis * 3 + pair) holds slots 2*pair (low
//             half) and 2*pair+1 (high half) of side 0 = lo, 1 = hi; decoded plane = fma(h, scale_a,
//             origin_a) in f32 (h * scale exact, one rounding; the host verifies with the same fma that
//             every decoded box CONTAINS the child's exact box); a ray picks its near/far side per axis
//             by swapping whole dwords; an empty slot holds lo = +inf, hi = -inf (never hit)
//   dw 22-27  child codes (>= 0 wide-node index, < 0 kLeafBit | leaf-record offset; INT32_MAX empty)
//   dw 28-31  reference-order tree: for the octants o = 0..3 of the ray direction (bit a set iff
//             d[a] > 0; bit 2 clear), the rank of slot j in the reference's visiting order at bits
//             3j..3j+2; an octant o >= 4 visits in exactly the reverse order of o ^ 7 (every split
//             flips), rank n-1-r (empty slots hold n-1).  Zero in the occlusion tree.
constexpr int kWideSlots = 6;
struct alignas(128) Wide {
    float ox, oy, oz; uint32_t exps;
    uint32_t h[18];
    int32_t child[6];
    uint32_t rank[4];
};
static_assert(sizeof(Wide) == 128, "wide node size");

struct alignas(16) LeafHead {
    float minx, miny, minz; int32_t count;
    float maxx, maxy, maxz; int32_t slot0;
};
struct alignas(16) Vec4 { uint32_t v[4]; };   // 16-B unit of the leaf-record array
#ifndef RT_TOP_PAIRS
#define RT_TOP_PAIRS 256
#endif
constexpr int kTopPairs = RT_TOP_PAIRS;   // top-level pairs cached in LDS (64 B each, per workgroup)
constexpr int kLeafCountShift = 25;
constexpr int32_t kLeafStartMask = (1 << kLeafCountShift) - 1;
constexpr int kLeafMaxCount = 63;

static_assert(sizeof(Pair) == 64, "pair size");
static_assert(sizeof(LeafHead) == 32, "leaf head size");
static_assert(sizeof(Node) == 32, "node size");
static_assert(sizeof(Prim) == 48, "prim size");
static_assert(sizeof(Material) == 64, "material size");
static_assert(sizeof(Light) == 32, "light size");

}  // namespace dl
