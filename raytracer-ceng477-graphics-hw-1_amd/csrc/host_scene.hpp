// Host-side scene model, XML loader and BVH builder of librt_hip.
//
// The BVH must be *bit-identical* to the reference's (bvh.h:48-163): same
// boxes, same split rule/retries/depth cap, same pre-order flatten and the
// same per-leaf primitive order — closest-hit tie-breaking and t-pruning
// depend on it.  The flattened form here is the GPU
// layout (device_layout.hpp), not the reference's 104-byte AoS BVHNode.
#pragma once

#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "device_layout.hpp"

namespace rtx {

struct V3 { float x, y, z; };

inline float vget(const V3& v, int i) { return i == 1 ? v.y : (i == 2 ? v.z : v.x); }

struct CameraRec {
    V3 position, gaze, up;
    float near_plane[4];
    float near_distance;
    int width, height;
    std::string name;
};

struct LightRec { V3 position, intensity; };
struct MaterialRec { int is_mirror; V3 ambient, diffuse, specular, mirror; float phong; };
struct TriRec { int material_id, v0, v1, v2; V3 normal, center; };
struct SphereRec { int material_id, center_id; float radius; };

struct HostScene {
    int bg[3] = {0, 0, 0};
    float eps = 0.001f;
    int max_depth = 0;
    V3 ambient{0, 0, 0};
    std::vector<CameraRec> cameras;
    std::vector<LightRec> lights;
    std::vector<MaterialRec> materials;
    std::vector<V3> verts;
    std::vector<TriRec> tris;      // reference flattening order (raytracer.cpp:336-341)
    std::vector<SphereRec> spheres;
};

// A vector whose resize(n) leaves new elements of a trivial type uninitialized: the build writes every
// byte of the device arrays itself (in parallel), so the serial zero-fill and its first-touch page
// faults are not paid twice.
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = NoInitAlloc<U>; };
    NoInitAlloc() = default;
    template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
    template <class U> void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A> void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T> using DevVec = std::vector<T, NoInitAlloc<T>>;

// Flattened BVH in device layout.
struct FlatBVH {
    DevVec<dl::Node> nodes;             // pre-order, left child = i + 1
    DevVec<dl::Prim> prims;             // leaf primitive copies, leaf-contiguous
    DevVec<dl::TriShade> tri_shade;     // per triangle id: normal + material
    // child-pair layout of the same tree (device_layout.hpp dl::Pair)
    DevVec<dl::Pair> pairs;
    std::vector<dl::LeafBig> leaf_big;
    float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};
    int32_t root_info = 0;
    int top_pairs = 0;               // pairs [0, top_pairs) = the top levels, breadth-first
    // Occlusion tree: an SAH hierarchy over the SAME leaves (same prim ranges,
    // same exact leaf boxes) with union boxes above them (build_shadow_tree).
    DevVec<dl::Pair> spairs;
    float sroot_lo[3] = {0, 0, 0}, sroot_hi[3] = {0, 0, 0};
    int32_t sroot_info = 0;
    int smax_depth = 0;
    // leaf records (LeafHead + prims), 16-B units, one per reference leaf in
    // pre-order, + 3 units of tail pad; shared by both wide trees
    DevVec<dl::Vec4> lrec;
    std::vector<int32_t> pair_lrec;  // [2 * pair + side]: leaf record offset of a leaf child, else -1
    int32_t root_lrec = -1;          // the root's record when the root is a leaf
    // the occlusion tree collapsed to wide nodes (any-hit walks)
    DevVec<dl::Wide> swnodes;
    int32_t swroot = 0;              // >= 0 node index, < 0 kLeafBit | leaf-record offset
    int swmax_stack = 0;             // worst-case stack entries of a walk over them
    // the reference tree collapsed to wide nodes (closest-hit walks, reference order)
    DevVec<dl::Wide> wnodes;
    int32_t wroot = 0;
    int wmax_stack = 0;              // worst-case stack entries of a walk over them
    int leaves = 0, max_leaf = 0, max_depth = 0, max_stack = 0;
    double build_ms = 0;
    double ref_ms = 0, flat_ms = 0, stree_ms = 0, refwide_ms = 0;   // phases: reference tree, flatten (layout,
                                                                    // leaf records, pairs), occlusion tree,
                                                                    // reference-order wide tree
    int threads = 1;                 // host threads the build used   // phases of build_ms: reference tree, flatten, wide trees
};

// parser.cpp:6-218 semantics.  Returns empty string on success, else message.
// threads: for the large number lists (0: build_threads default, 1: serial).
std::string load_xml(const char* path, HostScene& out, int threads = 0);

// raytracer.cpp:342-348: per-triangle normal and centre.
void prepare_triangles(HostScene& s);

// bvh.h:48-163 + the GPU flatten + the wide trees. Returns empty string or an
// error message.  threads: host build threads (0: RT_BUILD_THREADS, else the
// hardware concurrency capped at 16; 1: serial).  The output does not depend
// on the thread count.
// on_flat (optional) is called once the flatten's arrays (nodes, prims, tri_shade, pairs, leaf_big,
// lrec) are final, while the wide trees are still being built (they only read those arrays).
std::string build_bvh(const HostScene& s, FlatBVH& out, int threads = 0,
                      const std::function<void()>* on_flat = nullptr);
int build_threads(int requested);

}  // namespace rtx
