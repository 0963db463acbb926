/*
 * rt.h — C-ABI of the MI355X-native renderer (librt_hip.so).
 *
 * Drop-in boundary for the reference's hot path.  The reference has no FFI;
 * its operator boundary is the C++ class pair used by main()
 * (raytracer.cpp:487-525):
 *
 *   RayTracer::RayTracer(parser::Scene&)            raytracer.cpp:335-350
 *        -> rt_scene_create / rt_scene_load_xml     (flatten + BVH build + upload)
 *   Image RayTracer::render(Camera&)                raytracer.cpp:362-383
 *        -> rt_render (host buffer, synchronous) / rt_render_device (HBM, async)
 *   static Image ImageProcessor::downSample(...)    raytracer.cpp:459-484
 *        -> folded into rt_render* via aa_factor (and rt_downsample_host)
 *   void write_ppm(const char*, unsigned char*, int, int)   ppm.h:4, ppm.cpp:4-39
 *        -> rt_write_ppm (byte-identical P3)
 *   Scene::loadFromXml(const std::string&)          parser.cpp:6-218
 *        -> rt_scene_load_xml
 *
 * Conventions: plain pointers and sizes only; every function returns 0 on
 * success or a negative rt_status, with a message in rt_last_error()
 * (thread-local).  No exceptions cross this ABI (the reference throws
 * std::runtime_error from parser.cpp:14,20 and ppm.cpp:10 instead).
 * The library owns device copies of the scene until rt_scene_destroy; the
 * caller owns every host buffer.  One in-flight render per rt_scene.
 */
#ifndef RT_RT_H
#define RT_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 12

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_ARG = -1,        /* bad argument / shape                         */
    RT_ERR_IO = -2,         /* file cannot be read or written               */
    RT_ERR_PARSE = -3,      /* XML malformed / missing element              */
    RT_ERR_HIP = -4,        /* HIP runtime error (message has the HIP name) */
    RT_ERR_NO_DEVICE = -5,  /* no gfx950 device visible                     */
    RT_ERR_LIMIT = -6       /* scene exceeds an encoding limit, or a walk hit its
                               step bound (rt_scene_check)                   */
} rt_status;

/* ---- scene model: field names and meaning follow parser.h:170-251 ---- */
typedef struct rt_vec3f { float x, y, z; } rt_vec3f;

typedef struct rt_camera {          /* parser::Camera (parser.h:170-178)     */
    rt_vec3f position, gaze, up;
    float near_plane[4];            /* left right bottom top (Vec4f x y z w) */
    float near_distance;
    int image_width, image_height;  /* OUTPUT resolution (before SSAA)       */
} rt_camera;

typedef struct rt_point_light { rt_vec3f position, intensity; } rt_point_light;  /* parser.h:180-183 */

typedef struct rt_material {        /* parser::Material (parser.h:185-192)   */
    int is_mirror;
    rt_vec3f ambient, diffuse, specular, mirror;
    float phong_exponent;
} rt_material;

typedef struct rt_triangle { int material_id, v0_id, v1_id, v2_id; } rt_triangle;  /* 1-based ids */
typedef struct rt_sphere { int material_id, center_vertex_id; float radius; } rt_sphere;

/* Borrowed host arrays, read during rt_scene_create only.  `triangles` is the
 * reference's flattened order (raytracer.cpp:336-341): the scene's standalone
 * <Triangle>s, then each <Mesh>'s faces in file order with the mesh's
 * material id. */
typedef struct rt_scene_desc {
    int background_color[3];
    float shadow_ray_epsilon;
    int max_recursion_depth;
    rt_vec3f ambient_light;
    const rt_point_light* lights;   int num_lights;
    const rt_material* materials;   int num_materials;
    const rt_vec3f* vertices;       int num_vertices;
    const rt_triangle* triangles;   int num_triangles;
    const rt_sphere* spheres;       int num_spheres;
} rt_scene_desc;

#define RT_OPT_HOST_ONLY 1   /* load + BVH build only, no device upload (no GPU needed) */
/* The render path is the chain renderer (closest-hit chains, deferred any-hit
 * shadow walks, shading + fold + SSAA in one pass).  Bits 2, 4 and 16 named the
 * megakernel, wavefront and fused comparison paths up to ABI 10; they were
 * bit-identical and slower, and are accepted and ignored since ABI 11. */
#define RT_OPT_CHAIN 8       /* the chain path (the default; accepted for ABI <= 10 callers) */

typedef struct rt_options {
    int device;       /* HIP device ordinal; -1 = current device            */
    int flags;        /* RT_OPT_* bits                                       */
    int build_threads;/* host threads for the BVH build (bvh.h:48-163); 0 =
                         env RT_BUILD_THREADS or hardware concurrency (<= 16),
                         1 = serial.  The tree never depends on it.  (ABI 2) */
} rt_options;

typedef struct rt_stats {
    uint64_t primary_rays;      /* eye rays (W*H*F^2)                        */
    uint64_t shadow_rays;       /* any-hit queries (one per hit per light)   */
    uint64_t reflection_rays;   /* closest-hit traversals at depth >= 1      */
    uint64_t node_visits;       /* BVH box tests (stack pops), both walks    */
    uint64_t tri_tests;         /* Cramer triangle tests                     */
    uint64_t sphere_tests;      /* analytic sphere tests                     */
    double   kernel_ms;         /* device time of the render kernel(s)       */
    double   wall_ms;           /* host wall time of the call                */
    uint64_t shadow_rays_skipped;  /* of shadow_rays: not traced by the chain path's
                                      timed kernels because they cannot change the
                                      pixel (light behind the surface; ABI 6)   */
} rt_stats;

typedef struct rt_bvh_info {
    int nodes, leaves, max_leaf_prims, max_depth, max_stack;
    int triangles, spheres;
    double build_ms;         /* whole host build                                  */
    double ref_ms;           /* the reference tree (bvh.h:48-163) alone  (ABI 2) */
    double wide_ms;          /* the SAH occlusion tree + both wide trees (ABI 2) */
    int build_threads;       /* threads the build used                   (ABI 2) */
    int wide_nodes;          /* wide nodes of both wide trees (occlusion + reference order) */
    uint64_t wide_hash;      /* FNV-1a of both wide trees + leaf records (ABI 2) */
    /* device bytes of the structures the production walks read (ABI 7) */
    uint64_t ref_wide_bytes;     /* reference-order wide tree (closest hit)           */
    uint64_t occ_wide_bytes;     /* occlusion wide tree (any hit)                      */
    uint64_t leaf_record_bytes;  /* leaf records: exact leaf box + primitive copies    */
    uint64_t tri_shade_bytes;    /* per-triangle normal + material (hit epilogues)     */
    /* scene creation phases, host wall ms (ABI 10): XML read + parse (0 for
     * rt_scene_create), triangle normals/centres, flatten (device layout, leaf
     * records, child pairs), reference-order wide tree, occlusion tree (built
     * concurrently with the wide tree when threads allow), device upload */
    double xml_ms, prep_ms, flat_ms, refwide_ms, stree_ms, upload_ms;
} rt_bvh_info;

/* ---- errors / devices ---- */
const char* rt_last_error(void);
int rt_abi_version(void);
int rt_device_count(int* count);

/* ---- multi-GPU (ABI 4) ----
 * SURVEY.md §8(b) "N GPUs, one HIP stream each, one RCCL comm"; the
 * reference's row-interleaved threads (raytracer.cpp:352-383) become row
 * stripes over the GPUs of one node.  rt_set_devices(n), n >= 1: scenes
 * created afterwards (rt_scene_create / rt_scene_load_xml) hold a replica on
 * each of devices 0..n-1 and one RCCL communicator over them; rt_render and
 * rt_render_cameras then split every frame into stripe_rows-row stripes dealt
 * round-robin over the devices (env RT_GROUP_STRIPE, default 4), render them
 * concurrently (one HIP stream per device), gather the uint8 slabs to device 0
 * with ONE ncclGather over xGMI, un-interleave them there and copy the frame
 * to the caller's buffer -- designed to give the same bytes as one GPU; the
 * RCCL gather at n > 1 has not run on hardware yet (a group of one, and the
 * RT_GROUP_VIRTUAL=1 rehearsal -- n ranks on device 0, device copies in place
 * of RCCL -- are tested bit-exact).  rt_render_cameras on a group renders each
 * run of consecutive same-size cameras as one frame batch on every device
 * (frames in flight together) with one grouped gather (env RT_GROUP_BATCH:
 * at most that many frames per gather; 1 = one ncclGather per call, the
 * escape hatch while the grouped call is unrun at n > 1).  The asynchronous
 * device-buffer entry points (rt_render_device, rt_render_frames_device,
 * rt_render_cameras_device) keep using device 0 only: a one-process-per-GPU
 * caller shards with their stripe/rank arguments instead.  n = 1 runs the
 * same group path (RCCL communicator of one) on device 0; n = 0 (default):
 * no group, one device (rt_options.device).  RCCL is loaded on first use. */
int rt_set_devices(int n);
/* Devices a scene renders on (1 unless created after rt_set_devices(n >= 1)). */
int rt_scene_num_devices(const struct rt_scene* scene);

/* ---- scene lifetime ---- */
typedef struct rt_scene rt_scene;

/* RayTracer ctor (raytracer.cpp:335-350): per-triangle normal/centre, BVH
 * build bit-identical to bvh.h:48-163, SoA/AoS flatten and upload to HBM. */
int rt_scene_create(const rt_scene_desc* desc, const rt_options* opts, rt_scene** out);
/* Scene::loadFromXml (parser.cpp:6-218) + rt_scene_create. */
int rt_scene_load_xml(const char* path, const rt_options* opts, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

int rt_scene_num_cameras(const rt_scene* scene);
/* Camera i of an XML-loaded scene; name may be NULL. */
int rt_scene_get_camera(const rt_scene* scene, int index, rt_camera* cam, char* name, int name_len);
int rt_scene_bvh_info(const rt_scene* scene, rt_bvh_info* info);
/* Override MaxRecursionDepth (parser.cpp:48-57) for subsequent renders. */
int rt_scene_set_max_depth(rt_scene* scene, int max_recursion_depth);
/* Copy of the flattened BVH in device layout (32-byte nodes, pre-order, left
 * child = i+1; see csrc/device_layout.hpp).  Returns the node count; copies
 * min(count, capacity) nodes when out != NULL. */
int rt_scene_export_nodes(const rt_scene* scene, void* out, int capacity);

/* ---- rendering ---- */
/* RayTracer::render + ImageProcessor::downSample: renders `cam` at internal
 * resolution (W*aa) x (H*aa), quantises each sample (toPixel, parser.h:88-93),
 * box-filters with integer floor division.  out_rgb: caller-allocated
 * W*H*3 bytes, row-major, top row first.  Synchronous.  stats may be NULL;
 * when non-NULL the work counters are collected (slower counting kernel). */
int rt_render(rt_scene* scene, const rt_camera* cam, int aa_factor,
              uint8_t* out_rgb, rt_stats* stats);

#define RT_RENDER_COUNT 1   /* flags: accumulate work counters on device */

/* Asynchronous render into device memory on `stream` (a hipStream_t; NULL =
 * the null stream).  Output rows are split into stripes of `stripe_rows`
 * rows dealt round-robin over `nranks` ranks (the reference's row interleave,
 * raytracer.cpp:353, at stripe granularity); this call renders rank `rank`'s
 * stripes packed contiguously into out_dev, which must hold
 * rt_slab_rows(H, stripe_rows, nranks) * W * 3 bytes.  nranks = 1 renders the
 * full frame in row order.  With RT_RENDER_COUNT the counters accumulate
 * into the scene's device counter block (rt_counters_reset / _read). */
int rt_render_device(rt_scene* scene, const rt_camera* cam, int aa_factor,
                     int stripe_rows, int rank, int nranks,
                     void* out_dev, void* stream, int flags);
/* Multi-camera batching (raytracer.cpp:505-519 renders the cameras one after
 * another): renders cams[0..n) at SSAA factor `aa` with the frames running
 * concurrently on the device (chain path: up to 4 frames in flight, each on
 * its own stream and workspace, forked from and joined back into `stream`).
 * outs_dev[i] must hold cams[i] W*H*3 bytes; each image is identical to
 * rt_render of that camera.  (ABI 2) */
int rt_render_cameras_device(rt_scene* scene, const rt_camera* cams, int n, int aa_factor,
                             void* const* outs_dev, void* stream, int flags);
/* Sharded frame batch (ABI 3): rank `rank` of `nranks` renders its row
 * stripes (as rt_render_device) of n frames, the frames in flight together
 * exactly as in rt_render_cameras_device (each frame's slow mirror-chain tail
 * overlaps the other frames' bulk).  outs_dev[i] holds cams[i]'s slab,
 * rt_slab_rows(H, stripe_rows, nranks) * W * 3 bytes, identical to
 * rt_render_device of that camera.  The frame-sequence form of the
 * reference's per-camera render loop (raytracer.cpp:505-519) for a
 * multi-GPU serving loop. */
int rt_render_frames_device(rt_scene* scene, const rt_camera* cams, int n, int aa_factor,
                            int stripe_rows, int rank, int nranks,
                            void* const* outs_dev, void* stream, int flags);
/* The same into caller-allocated host buffers, synchronous (the drop-in main's
 * camera loop).  stats (nullable) sums the work counters over the cameras. */
int rt_render_cameras(rt_scene* scene, const rt_camera* cams, int n, int aa_factor,
                      uint8_t* const* outs, rt_stats* stats);
/* Diagnostics: dependent-step latency of closest-hit walks.  rays: n x
 * {o.xyz, dir.xyz}; one wave walks ray i with `lanes` lanes (1..64), `reps`
 * times; out[4i..4i+3] = {shader cycles of the last rep, steps, winner prim
 * slot or -1, cycles of the first rep}.  mode 0: the production walk, 1: the
 * reference tree (ABI 2). */
int rt_walk_timing(rt_scene* scene, const float* rays, int n, int lanes, int reps, int mode,
                   unsigned long long* out);
/* Diagnostics: out[i] = the device's specular power term for base[i],
 * exponent[i] -- (float)pow((double)base, (double)exponent) of the C library
 * (raytracer.cpp:414) -- on the current device (host arrays, synchronous;
 * ABI 5). */
int rt_phong_pow(const float* base, const float* exponent, float* out, int n);
/* Diagnostics: out[3i+j] = num[3i+j] / den[i] as the device's triangle test
 * (raytracer.cpp:147, 154, 161) evaluates its three Cramer quotients: one
 * shared reciprocal, the correctly rounded float quotients (host arrays,
 * synchronous; ABI 8). */
int rt_cramer_div(const float* den, const float* num, float* out, int n);
/* Diagnostics: q[j*nv + i] = v[i] / d[j] (unsigned 32-bit, d[j] > 0) as the
 * shadow walkers' task dealing divides by a wave-uniform divisor (pathchain.hip
 * UDiv: a scalar-register reciprocal, a high multiply and two corrections;
 * host arrays, synchronous; ABI 9). */
int rt_udiv(const uint32_t* v, int nv, const uint32_t* d, int nd, uint32_t* q);
/* HBM held by a scene on its (first) device (ABI 7): the uploaded scene (trees,
 * primitives, tables) and the render workspaces allocated so far (chain-path
 * arenas of every slot and their side tables, output staging).  The workspaces grow on demand up to
 * the scene's budget, env RT_WS_BUDGET_MB at scene creation (default 16384 MB
 * for all slots together); a frame batch or chunk is sized to fit it. */
int rt_scene_memory(const rt_scene* scene, uint64_t* scene_bytes, uint64_t* workspace_bytes);
/* Measured roofline denominators (ABI 7), on `device` (-1: the
 * current one), ~1 s, allocates 4 GiB + the tables temporarily:
 *   hbm_copy_gbps      streaming float4 copy of 2 GiB (read + write bytes / time)
 *   hbm_read_gbps      the same buffer read only
 *   l2_gather_gbps     the BVH walks' divergent fetch: every lane reads one random
 *                      128-B line (eight dwordx4) per dependent step from a table every
 *                      workgroup shares, best of 8..20 waves per CU; table of
 *                      l2_table_bytes (2 MiB, inside one XCD's 4 MiB L2)
 *   scene_gather_gbps  the same over a table of scene_table_bytes (the caller's
 *                      walk hot set; lines beyond L2 come from the Infinity Cache)
 *   l2_line_gbps,      the same bytes with 8 lanes reading the 8 pieces of one line
 *   scene_line_gbps    (full-line fetches: the L2's deliverable bandwidth) */
typedef struct rt_peaks {
    double hbm_copy_gbps, hbm_read_gbps;
    double l2_gather_gbps, l2_table_bytes;
    double scene_gather_gbps, scene_table_bytes;
    double l2_line_gbps, scene_line_gbps;
} rt_peaks;
int rt_measure_peaks(int device, uint64_t scene_table_bytes, rt_peaks* out);
/* Rows in one rank's slab (max over ranks, so all slabs have equal size). */
int rt_slab_rows(int height, int stripe_rows, int nranks);
/* Rank-0 reassembly: slabs[nranks][slab_rows][W][3] (gathered) -> image[H][W][3]. */
int rt_unshuffle_stripes(const void* slabs_dev, void* image_dev, int width, int height,
                         int stripe_rows, int nranks, void* stream);
int rt_counters_reset(rt_scene* scene, void* stream);
int rt_counters_read(rt_scene* scene, rt_stats* stats);   /* synchronises the device */
/* Diagnostics (ABI 7): the raw u64 counter block, n slots (returns the slots
 * copied).  0-6 as rt_stats; 8.. per kernel role of the chain path (pathchain.hpp
 * CounterSlot): phase-A / phase-B closest-hit walk bytes (or node visits), walks
 * and hits, continuations, and the shadow rays of A, of B's workgroup queue and
 * of B's overflow -- bytes and rays each.  Bytes when the scene was created with
 * RT_DEBUG=0x20 (the production walks' fetched bytes).  24..29 (every launch,
 * timed or counting; round 4): chain launches, continuations, continuations
 * beyond the phase-B record space (walked by k_fallback), deferred closest-hit
 * rays, deferred shadow rays, launches whose fallback shadow queue overflowed.
 * 30 (round 5): launches with compact 16-B phase-A records (RT_COMPACT). */
int rt_counters_read_raw(rt_scene* scene, uint64_t* out, int n);
/* Diagnostics (ABI 7): per-kernel device time of the chain path's launches
 * since the last reset, for a scene created with env RT_DEBUG=0x10 (each kernel's
 * own dispatch start / end timestamps, as rocprofv3 reports them -- ABI 12; each
 * launch then synchronises).  ms[k] for k =
 * k_chain, k_pack_a, k_mix, k_occlude (A's shadows, frame batches), k_pack_b,
 * k_occlude (B's overflow), k_finish, k_fallback.  Returns the launches timed. */
int rt_kernel_times(rt_scene* scene, double* ms, int n, int reset);
/* Synchronises the scene's device and reports a walk that was cut off since
 * the last check: every BVH walk has an always-on step bound (64 x the tree's
 * nodes; a DFS pops each node at most once), and a walk exceeding it ends
 * early and sets the scene's device error word -> RT_ERR_LIMIT (the frames
 * rendered since the last check are then invalid).  rt_render,
 * rt_render_cameras and rt_counters_read check it themselves; asynchronous
 * callers (rt_render_device, rt_render_frames_device) call this.  The word is
 * SCENE-WIDE, not per stream: a check reports (and clears) a walk cut off in
 * any render of the scene on any stream since the previous check, so callers
 * that render one scene on several streams should check after joining them.
 * (ABI 4) */
int rt_scene_check(rt_scene* scene);

/* Primary closest-hit per internal pixel ((W*aa) x (H*aa)): t (tSmall, -1 on
 * miss) and material id (0 on miss) into caller-allocated host arrays
 * (either may be NULL).  Debug / parity surface for Ray::getFirstIntersection
 * (raytracer.cpp:177-225). */
int rt_primary_hits(rt_scene* scene, const rt_camera* cam, int aa_factor,
                    float* t_out, int32_t* material_out);
/* The same dump from the TIMED walk (ABI 12): one whole frame through the
 * production kernels (k_chain's reference-order wide-tree walk, k_fallback
 * for the rays it defers), with each sample's level-0 tSmall and material
 * stored where the production kernel records its hit.  Unset entries (a
 * sample no kernel recorded) read back as NaN / -1.  Parity surface for
 * Ray::getFirstIntersection (raytracer.cpp:177-225) on the product path. */
int rt_primary_hits_production(rt_scene* scene, const rt_camera* cam, int aa_factor,
                               float* t_out, int32_t* material_out);

/* ---- host utilities ---- */
/* ImageProcessor::downSample (raytracer.cpp:459-484) on host buffers. */
int rt_downsample_host(const uint8_t* in, int width, int height, int factor, uint8_t* out);
/* write_ppm (ppm.cpp:4-39), byte-identical P3 output. */
int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height);

#ifdef __cplusplus
}
#endif
#endif /* RT_RT_H */
