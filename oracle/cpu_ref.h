/*
 * oracle/cpu_ref.h -- C API of the CPU restatement of the reference path tracer.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library or run the oracle binary; the product
 * (surf-path-tracer_amd/) never links it.
 *
 * Parity status: UNPINNED against a run of the reference itself.  The reference
 * (nemjit001/surf-path-tracer) is unbuildable in this image: its CPU sources
 * include glm, tinyobjloader and the Vulkan headers, none of which exist here,
 * and building it against stand-ins is not allowed.  The reference ships no
 * tests, fixtures or golden images.  What pins this oracle instead:
 *   - data facts of the bundled assets (triangle counts per OBJ file);
 *   - glibc sinf/cosf/expf used exactly as the reference calls them;
 *   - property checks (BVH closest hit == brute-force closest hit, etc.).
 * See DESIGN.md "Oracle".
 */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* Event counters of one render call (means per sample = value / samples). */
typedef struct {
    uint64_t samples;      /* camera samples (paths) */
    uint64_t n_ext;        /* extension rays traced (Scene::intersect calls) */
    uint64_t n_hit;        /* extension rays that hit geometry */
    uint64_t n_cont;       /* continuation rays spawned */
    uint64_t n_shadow;     /* shadow rays traced (Scene::intersectAny calls) */
    uint64_t n_acc;        /* radiance contributions added to a path's energy */
    uint64_t n_unocc;      /* unoccluded shadow rays */
    uint64_t max_segments; /* longest path, in extension rays */
} orc_counters;

/* variant 0: bundled indoor scene (reference main.cpp:161-346).
 * variant 1: C5 deep scene -- indoor scene + 648 Suzanne copies baked in one mesh. */
orc_scene* orc_scene_create(const char* assets_dir, int variant);
void orc_scene_destroy(orc_scene*);

/* Mesh facts: triangles per loaded mesh (susanne, cube, lens, plane[, lattice]). */
int orc_scene_mesh_tris(const orc_scene*, uint32_t* out, int max);
/* Instances and lights. */
uint32_t orc_scene_instance_count(const orc_scene*);
uint32_t orc_scene_light_count(const orc_scene*);

/* GPUScene::update(dt) (scene.cpp:267-282): rotate instance 3, refit the TLAS. */
void orc_scene_update(orc_scene*, float dt);

/* Camera of main.cpp:141-149 for a W x H render. */
void orc_scene_set_camera(orc_scene*, uint32_t width, uint32_t height);
/* Copy of the CameraUBO (128 B, camera.h:12-19) the camera produces. */
void orc_camera_ubo(const orc_scene*, void* out128);

/* GPUBatcher layout export (scene.cpp:61-157), materials in first-use order.
 * which: 0 triangles(64B) 1 triExt(80B) 2 blasIdx(u32) 3 blasNodes(48B)
 *        4 materials(64B) 5 instances(160B) 6 tlasIdx(u32) 7 tlasNodes(48B)
 *        8 lights(8B) 9 background(64B).  Returns bytes; copies when dst != NULL. */
uint64_t orc_scene_export(const orc_scene*, int which, void* dst);

/* Renders rows [row_begin,row_end) of a W x H image for `frames` frames, one
 * sample per pixel per frame, frame f seeded initSeed(p + 1799*(first_frame+f))
 * (renderer.cpp:169).  acc (rows*W*4 floats) accumulates (rgb,1) per sample
 * exactly as AccumulatorState does (renderer.cpp:180).  max_segments 0 =
 * unbounded (reference semantics); >0 caps the extension rays per path.
 * threads <= 0: OpenMP default.  Returns seconds spent in the render loop. */
double orc_render(orc_scene*, uint32_t width, uint32_t height,
                  uint32_t row_begin, uint32_t row_end,
                  uint32_t first_frame, uint32_t frames, uint32_t max_segments,
                  int threads, float* acc, orc_counters* counters);
/* The same over an arbitrary row list (acc: nrows x width RGBA, list order). */
double orc_render_rows(orc_scene*, uint32_t width, uint32_t height, const uint32_t* rows, uint32_t nrows,
                       uint32_t first_frame, uint32_t frames, uint32_t max_segments, int threads,
                       float* acc, orc_counters* out);
/* Multi-sample frames (Renderer::render with config().samplesPerFrame = spp,
 * renderer.cpp:160-188): frame f is seeded once per pixel with
 * initSeed(p + 1799*(first_sample + f*spp)) and its spp samples run in
 * sequence, each continuing the RNG state the previous sample's path left.
 * first_sample is the accumulator's totalSamples before the first frame
 * (= the frame index for spp 1). */
double orc_render_spp(orc_scene*, uint32_t width, uint32_t height, uint32_t row_begin, uint32_t row_end,
                      uint32_t first_sample, uint32_t frames, uint32_t spp, uint32_t max_segments, int threads,
                      float* acc, orc_counters* counters);
double orc_render_rows_spp(orc_scene*, uint32_t width, uint32_t height, const uint32_t* rows, uint32_t nrows,
                           uint32_t first_sample, uint32_t frames, uint32_t spp, uint32_t max_segments, int threads,
                           float* acc, orc_counters* out);

/* Closest hit of n world-space rays (o,d: 3 floats each, depth starts 1e30).
 * out_t, out_u, out_v (floats), out_inst, out_prim (u32, ~0 when missed). */
void orc_trace_closest(const orc_scene*, uint32_t n, const float* o, const float* d,
                       float* out_t, float* out_u, float* out_v,
                       uint32_t* out_inst, uint32_t* out_prim);
/* Any hit of n rays with depth tmax[i]. out[i] = 1 when occluded. */
void orc_trace_any(const orc_scene*, uint32_t n, const float* o, const float* d,
                   const float* tmax, uint8_t* out);
/* Closest-hit traversal statistics: per ray and instance (n x instance_count,
 * instance-id order) BLAS node visits and triangle tests.  Diagnostics. */
void orc_trace_visits(const orc_scene*, uint32_t n, const float* o, const float* d, uint32_t* nodes, uint32_t* tris);
/* Brute force closest hit over every instance triangle (no BVH): property check. */
void orc_trace_brute(const orc_scene*, uint32_t n, const float* o, const float* d,
                     float* out_t, uint32_t* out_inst, uint32_t* out_prim);

/* Records the extension and shadow rays of pixel paths for kernel-level tests.
 * For pixels [pix_begin, pix_end) of frame `frame` (whole image, W x H) it
 * stores every extension ray (o,d) and every shadow ray (o,d,tmax) the path
 * tracer issues, up to max_ext / max_shadow records.  Returns counts. */
void orc_record_rays(orc_scene*, uint32_t width, uint32_t height, uint32_t frame,
                     uint32_t pix_begin, uint32_t pix_end,
                     uint32_t max_ext, float* ext_o, float* ext_d, uint32_t* n_ext,
                     uint32_t max_shadow, float* sh_o, float* sh_d, float* sh_tmax,
                     uint32_t* n_shadow);

/* Extension rays of every pixel's path of one whole frame (W x H, row-major). Diagnostics. */
void orc_path_lengths(orc_scene*, uint32_t width, uint32_t height, uint32_t frame, uint32_t* out);

/* Deepest root-to-leaf edge count of the TLAS and of every BLAS. */
void orc_bvh_depths(const orc_scene*, uint32_t* tlas_depth, uint32_t* max_blas_depth);

/* Ends paths whose throughput is exactly zero (radiance-neutral; see cpu_ref.cpp).
 * Default off = reference semantics. */
void orc_set_zero_cutoff(int on);
/* tinyobj-semantics OBJ load (Mesh(path)); -1 if unreadable. */
long orc_obj_load(const char* path, float* tris_out, float* ext_out, uint64_t cap);
/* Sequential BvhBLAS::build over n 64-B Triangles; returns nodesUsed. */
uint32_t orc_bvh_build(const float* tris, uint32_t n, uint32_t* idx_out, float* nodes_out);

/* RNG of surf_math.cpp:31-95, for known-answer tests. */
uint32_t orc_init_seed(uint32_t seed);
uint32_t orc_random_u32(uint32_t* seed);
float orc_random_f32(uint32_t* seed);

/* RgbaToU32 (surf_math.cpp:13-29) over n pixels of acc/spp. */
void orc_finalize_rgba8(const float* acc, uint32_t n, float inv_samples, uint32_t* out);

#ifdef __cplusplus
}
#endif
