/* ORACLE / TEST INFRASTRUCTURE ONLY — never linked into the product.
 *
 * Plain-C CPU restatement of the reference renderer's hot path
 * (lutfullaherkaya/raytracer-ceng477-graphics-hw-1): XML scene load
 * (parser.cpp:6-218), triangle flattening (raytracer.cpp:335-350), BVH build
 * (bvh.h:48-163), primary ray generation (raytracer.cpp:292-324), ordered-DFS
 * closest-hit and any-hit traversal (raytracer.cpp:177-280), Blinn-Phong +
 * shadow rays + mirror recursion (raytracer.cpp:385-452), SSAA box filter
 * (raytracer.cpp:459-484) and write_ppm (ppm.cpp:4-39).
 *
 * Pinned against the compiled reference (oracle/_ref/ref_harness) through the
 * golden fixtures in tests/golden/ (bit-exact RGB + primary hit-t samples).
 * Used only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ro_scene ro_scene;

typedef struct ro_counters {
    uint64_t primary_rays;     /* eye rays traced (W*H*F^2)                 */
    uint64_t shadow_rays;      /* any-hit queries (one per hit per light)   */
    uint64_t reflection_rays;  /* closest-hit traversals at depth >= 1      */
    uint64_t node_visits;      /* box tests (pops) in both traversals       */
    uint64_t tri_tests;        /* Cramer triangle tests                     */
    uint64_t sphere_tests;     /* analytic sphere tests                     */
} ro_counters;

/* Load an XML scene (same numeric semantics as parser.cpp). Returns NULL and
 * fills err on failure. Builds the BVH. */
ro_scene* ro_load(const char* path, char* err, int errlen);
void ro_free(ro_scene* s);

int ro_num_cameras(const ro_scene* s);
/* Output (post-AA) image size and name of camera i. */
int ro_camera_info(const ro_scene* s, int cam, int* width, int* height, char* name, int namelen);
int ro_bvh_info(const ro_scene* s, int* nodes, int* leaves, int* max_leaf, int* ntris, int* nspheres);

/* BVH nodes in pre-order, encoded like the product's 32-byte device node
 * (for BVH parity tests): {bmin.xyz, a} {bmax.xyz, b}; interior a = right
 * child index, b = axis; leaf a = first leaf-primitive slot,
 * b = 0x80000000 | nsph << 20 | ntri.  Returns the node count. */
int ro_export_nodes(const ro_scene* s, void* out, int capacity);

/* Render output rows [row_begin, row_end) of camera `cam` at SSAA factor `aa`
 * (internal resolution W*aa x H*aa, quantise per sample, integer box filter)
 * with `threads` threads (row-interleaved like raytracer.cpp:352-360).
 * out: caller-allocated (row_end-row_begin)*W*3 bytes. counters may be NULL.
 * max_depth_override < -999 keeps the scene's MaxRecursionDepth. */
int ro_render(const ro_scene* s, int cam, int aa, int threads, int row_begin, int row_end,
              int max_depth_override, uint8_t* out, ro_counters* counters);

/* Diagnostics: full-frame render that also records BVH node visits per
 * output pixel (all samples, all bounces, shadow rays included). */
int ro_work_map(const ro_scene* s, int cam, int aa, int threads, uint8_t* out, uint32_t* work);

/* Primary closest-hit at internal resolution (W*aa x H*aa): t (tSmall, -1 on
 * miss) and material id (0 on miss). Either pointer may be NULL. */
int ro_primary_hits(const ro_scene* s, int cam, int aa, float* t, int32_t* material);

/* Byte-identical to write_ppm (ppm.cpp:4-39). */
int ro_write_ppm(const char* path, const uint8_t* rgb, int width, int height);

#ifdef __cplusplus
}
#endif
#endif
