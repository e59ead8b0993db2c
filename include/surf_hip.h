/*
 * surf_hip.h -- C-ABI of the MI355X-native wavefront path tracer.
 *
 * This is the drop-in boundary for the reference's GPU path
 * (nemjit001/surf-path-tracer).  Each entry point names the reference
 * interface it replaces (paths relative to the reference repository root):
 *
 *   surf_create / surf_destroy      WaveFrontRenderer ctor/dtor (headers/renderer.h:211, sources/renderer.cpp:604-937)
 *   surf_upload_scene               GPUScene ctor: the 9 SSBOs + scene UBO (headers/scene.h:94-122, sources/scene.cpp:159-258)
 *   surf_update_instances           GPUScene::update re-upload (sources/scene.cpp:267-282)
 *   surf_set_camera                 CameraUBO upload (sources/renderer.cpp:971-979, headers/camera.h:12-19)
 *   surf_render                     WaveFrontRenderer::render dispatch loop (sources/renderer.cpp:1029-1118)
 *   surf_clear_accumulator          IRenderer::clearAccumulator (headers/renderer.h:91, sources/renderer.cpp:927-937)
 *   surf_read_accumulator           accumulator SSBO readback (headers/renderer.h:344-350)
 *   surf_finalize_rgba8             wavefront_finalize.comp:15-26 (+ RgbaToU32 rounding, sources/surf_math.cpp:13-29)
 *   surf_get_stats                  FrameInstrumentationData + Lumen energy (headers/renderer.h:30-34, sources/renderer.cpp:955-969)
 *   surf_trace_closest / _any       ray_extend.comp / ray_connect.comp traversal, exposed for hit-record tests
 *   surf_scene_build_indoor ...     host scene build of main.cpp:161-346 (Mesh/BvhBLAS/Instance/GPUBatcher)
 *
 * Conventions: every function returns 0 (SURF_OK) or a negative surf_status;
 * nothing aborts.  A context belongs to one HIP device and is driven from one
 * host thread.  Input records are byte-identical to the reference host structs
 * (sizes asserted below); the library re-lays them out internally (SoA queues,
 * child-box BVH nodes, BVH-ordered triangles).  Host buffers passed in are
 * copied; the caller keeps ownership.
 */
#ifndef SURF_HIP_H
#define SURF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SURF_ABI_VERSION 4

typedef enum {
    SURF_OK = 0,
    SURF_ERR_INVALID = -1,      /* bad argument / inconsistent scene */
    SURF_ERR_HIP = -2,          /* HIP runtime error (see surf_last_error) */
    SURF_ERR_NO_DEVICE = -3,    /* no gfx950 device at that index */
    SURF_ERR_NO_SCENE = -4,     /* render before upload */
    SURF_ERR_OOM = -5,          /* device allocation failed */
    SURF_ERR_IO = -6,           /* asset file unreadable */
    SURF_ERR_LIMIT = -7         /* scene exceeds a compiled limit (stack depth) */
} surf_status;

/* ---- reference record layouts (byte-identical; offsets in comments) ---- */

typedef struct { float x, y, z, _pad; } surf_float3_16;         /* ALIGN(16) Float3 slot */

typedef struct {                                                /* Triangle, mesh.h:14-25 (64 B) */
    surf_float3_16 v0, v1, v2, centroid;                        /* v0 = OBJ vertex 1, v1 = OBJ vertex 0 */
} surf_triangle;

typedef struct {                                                /* TriExtension, mesh.h:26-30 (80 B) */
    surf_float3_16 n0, n1, n2;                                  /* @0 @16 @32 */
    float uv0[2], uv1[2], uv2[2];                               /* @48 @56 @64 */
    float _pad[2];
} surf_tri_extension;

typedef struct {                                                /* BvhNode, bvh.h:36-46 (48 B) */
    uint32_t left_first, count, _pad[2];                        /* leaf iff count != 0 */
    surf_float3_16 bb_min, bb_max;                              /* @16 @32 */
} surf_bvh_node;

typedef struct {                                                /* Material, material.h:6-19 (64 B) */
    float emission_strength, reflectivity, refractivity, index_of_refraction;
    surf_float3_16 emission_color, albedo, absorption;          /* @16 @32 @48 */
} surf_material;

typedef struct {                                                /* GPUInstance, bvh.h:93-102 (160 B) */
    uint32_t tri_offset, bvh_idx_offset, bvh_node_offset, material_offset;
    float area;                                                 /* @16 */
    uint32_t _pad[3];
    float transform[16];                                        /* @32, glm column major */
    float inv_transform[16];                                    /* @96 */
} surf_gpu_instance;

typedef struct {                                                /* GPULightData, scene.h:67-71 (8 B) */
    uint32_t light_instance_idx, primitive_count;
} surf_light;

typedef struct {                                                /* SceneBackground, scene.h:18-26 (64 B) */
    uint32_t type;                                              /* 0 solid, 1 gradient */
    uint32_t _pad[3];
    surf_float3_16 color, gradient_a, gradient_b;               /* @16 @32 @48 */
} surf_background;

typedef struct {                                                /* CameraUBO, camera.h:12-19 (128 B) */
    surf_float3_16 position, up, fwd, right;                    /* @0 @16 @32 @48 */
    surf_float3_16 first_pixel, u_vector, v_vector;             /* @64 @80 @96 */
    float resolution[2];                                        /* @112 */
    float focal_length, defocus_angle;                          /* @120 @124 */
} surf_camera_ubo;

/* GPUScene's nine buffers + scene UBO (scene.h:113-122), host pointers. */
typedef struct {
    const surf_triangle* triangles;       uint32_t triangle_count;
    const surf_tri_extension* tri_ext;    /* triangle_count records */
    const uint32_t* blas_indices;         uint32_t blas_index_count;
    const surf_bvh_node* blas_nodes;      uint32_t blas_node_count;
    const surf_material* materials;       uint32_t material_count;
    const surf_gpu_instance* instances;   uint32_t instance_count;
    const uint32_t* tlas_indices;         /* instance_count records */
    const surf_bvh_node* tlas_nodes;      uint32_t tlas_node_count;
    const surf_light* lights;             uint32_t light_count;
    const surf_background* background;
} surf_scene_desc;

typedef struct {
    uint64_t samples;          /* camera samples rendered since the last clear (Mrays/s numerator, main.cpp:431) */
    uint64_t n_ext;            /* extension rays traced */
    uint64_t n_hit;            /* extension rays that hit geometry */
    uint64_t n_cont;           /* continuation rays */
    uint64_t n_shadow;         /* shadow rays traced */
    uint64_t n_acc;            /* radiance contributions */
    uint64_t n_unocc;          /* unoccluded shadow rays */
    uint64_t iterations;       /* wavefront iterations (extend->shade->connect->regen) */
    uint64_t tail_paths;       /* paths finished by the tail kernel */
    double   ms_total;         /* device time of render + drain calls since the last clear */
    double   ms_extend, ms_shade, ms_connect, ms_regen, ms_tail, ms_accum;  /* per-kernel (surf_set_profiling) */
    double   ms_sort;          /* the pool's ray-order sort (the shadow queue needs none), profiling mode */
    uint64_t launches_extend;  /* k_extend launches timed (profiling mode) */
    uint64_t n_ext_wavefront;  /* extension rays traced by k_extend (n_ext minus the drain's) */
    uint32_t stack_depth;      /* traversal stack entries reserved per ray */
    uint32_t pool_capacity;    /* paths in flight */
    float    energy;           /* sum of acc.rgb / samples over the shard ("Lumen", renderer.cpp:191-201) */
    uint32_t max_segments;     /* longest path seen (extension rays), diagnostics */
    uint64_t tail_survivors;   /* drain paths handed to the cooperative tail */
    uint32_t frame_window;     /* radiance ring slots (passes) of the current stream (surf_set_frame_batch), 0 before the first render */
} surf_stats;

typedef struct surf_ctx surf_ctx;       /* one per HIP device */
typedef struct surf_scene surf_scene;   /* host-side scene built by this library */

/* ---- version / device ---- */
int surf_abi_version(void);
int surf_device_count(int* count);

/* ---- context ----
 * Renders rows [row_begin, row_end) of a width x height frame (one shard). */
int surf_create(int hip_device, uint32_t width, uint32_t height,
                uint32_t row_begin, uint32_t row_end, surf_ctx** out);
/* Interleaved row blocks: block b = rows [b*row_block, (b+1)*row_block) goes to
 * shard b % shard_count. row_block 0 = contiguous split. */
int surf_create_sharded(int hip_device, uint32_t width, uint32_t height,
                        uint32_t shard_index, uint32_t shard_count, uint32_t row_block,
                        surf_ctx** out);
void surf_destroy(surf_ctx* ctx);
const char* surf_last_error(const surf_ctx* ctx);   /* ctx may be NULL: last global error */
/* Rows of this shard in shard order (row_count from surf_shard_rows(ctx, NULL, &n)). */
int surf_shard_rows(const surf_ctx* ctx, uint32_t* rows, uint32_t* row_count);
/* The HIP device the context was created on (the multi-GPU gather allocates
 * its buffers and streams there, whatever device the calling thread has set). */
int surf_get_device(const surf_ctx* ctx, int* hip_device);
/* The rows shard shard_index of shard_count owns under surf_create_sharded's
 * rule, in shard order (rows may be NULL to get the count).  Host only. */
int surf_shard_row_list(uint32_t height, uint32_t shard_index, uint32_t shard_count, uint32_t row_block, uint32_t* rows,
                        uint32_t* row_count);

/* Paths in flight (default: 5 full frames, W * H * 5, at most 16 M, whatever
 * the shard). Must be called before the first render. */
int surf_set_pool_capacity(surf_ctx* ctx, uint32_t paths);
/* Frame window: passes (samples per pixel; a frame of spp samples takes spp
 * consecutive passes) whose samples may be in flight at once -- a multiple of
 * the stream's samples_per_frame.  Default: the passes the stream being
 * started requests (one render call's frames x spp, rounded to a multiple of spp),
 * at least 256 -- 4096 for a stream opened by a one-frame request (a drop-in
 * loop extends its stream one frame per call) -- at most
 * 4096 and at most what min(64 GiB, a quarter of the free HBM) holds; a later
 * stream that requests more frames grows the ring (C3 at 1280x720: 256 frames
 * = 3.8 GB, a one-frame stream 4096 = 60 GB; C4 at 1920x1080: 1024 frames = 34 GB;
 * 64 GiB hold 2070 slots at 1080p).
 * Sample radiance is held per (frame slot, pixel) until a frame completes and
 * is accumulated in frame order; long Russian-roulette paths of old frames
 * overlap the bulk of newer ones.  A stream longer than the window issues
 * frame f only once frame f - window is accumulated.  Setting it fixes it
 * (must be called before the first render).  Several contexts on one device:
 * each sizes its default ring from the HBM free when its stream starts, so a
 * context started after another gets a smaller window (and, for a drop-in
 * loop, a lower throughput) -- fix the window here on each context for
 * predictable memory and throughput (memory: W * H * 16 B per slot). */
int surf_set_frame_batch(surf_ctx* ctx, uint32_t frames);
/* Throughput cutoff (enabled 1 / 0; -1 = automatic, the default: on for
 * streams of 1-sample frames, off for multi-sample frames, whose next sample
 * starts from the RNG state the reference's path ends with -- an early end
 * would change it, so there the cutoff is a deviation, not a neutral
 * shortcut): a path whose throughput T is below FLT_MIN
 * (1.17549435e-38) in every channel -- zero or denormal -- ends early.  The
 * reference's Russian roulette ends such a path with certainty at its next
 * diffuse bounce (p = max(T) < 2^-32, the smallest positive randomF32).  The
 * terms dropped are those the path would still add before that bounce: the
 * emitter hits along its chain of specular / dielectric bounces up to the next
 * diffuse bounce (any number of them), plus that bounce's NEE term -- each
 * below 1.2e-38 x (emission or light term):
 * radiance-neutral in f32 except for a pixel whose own energy is ~1e-38 (the
 * parity tests compare the GPU with the cutoff against the oracle without it,
 * bit for bit, on every tested image); n_ext/n_cont/... shrink.  It ends the
 * total-internal-reflection orbits in the glass lens that the reference traces
 * for up to millions of segments at a denormal throughput.
 * Stall risk with the cutoff off -- the automatic default for multi-sample
 * frames, e.g. a drop-in Renderer whose samplesPerFrame is above 1: such an
 * orbit runs to its end as in the reference (13,104,648 segments for one C3
 * path, frame 143, pixel 205912 at 1280x720 -- seconds of drain for the frame
 * holding it).  Bound it with max_segments (surf_render; a deviation, the
 * capped paths are counted and listed by surf_debug_capped) or enable the
 * cutoff (a deviation for multi-sample frames, see above). */
int surf_set_zero_cutoff(surf_ctx* ctx, int enabled);
/* Drain policy: when no new sample may be issued and at most `threshold_paths`
 * paths are in flight, the tail kernel finishes them in stages: each stage
 * runs `lanes_per_wave` paths per 64-lane wave for up to `stage_segments`
 * segments and hands the survivors to the next; once at most the
 * surf_set_tail_coop limit remain, the cooperative tail runs each on a whole
 * wave (0 = automatic for the first two; stage_segments 0 = a single lane
 * stage to the end; default 16).  Results do not depend on the policy.
 * Drains the context first. */
int surf_set_tail_policy(surf_ctx* ctx, uint32_t threshold_paths, uint32_t lanes_per_wave, uint32_t stage_segments);
/* Drain paths handed to the cooperative tail (default 150000, 0 = never): one
 * path per 64-lane wave with the lanes-as-planes traversal (any TLAS -- a
 * single-leaf TLAS walks its instances in a wave-uniform loop, any other the
 * TLAS DFS on the wave -- with a BVH stack of <= 64 entries; past 64
 * instances, materials or lights the tables are read from global memory), in
 * two-wave workgroups whose idle wave traces its sibling's shadow rays once
 * the path queue is empty (SURF_TAIL_PAIR=0 in the environment: one-wave
 * workgroups).  Identical results. */
int surf_set_tail_coop(surf_ctx* ctx, uint32_t max_paths);
/* Diagnostics: how many paths the segment cap ended in the current sample
 * stream, and the sample ids (frame slot * shard pixels + pixel) of up to
 * min(count, 64, max) of them (one per workgroup 0..63 that capped a path;
 * unused entries are 0xffffffff). */
int surf_debug_capped(surf_ctx* ctx, uint32_t* sample_ids, uint32_t max, uint64_t* count);
/* Diagnostics: shader-clock cycles of one drain segment's pieces on a lone
 * wave, each repeated `reps` times on the same path record path12 = (origin,
 * sample id bits), (direction, flag bits), (throughput, rng state bits):
 * cycles7[0] closest-hit wave walk, [1] shading, [2] the shadow ray's any-hit
 * walk, [3] the cosine sample alone, [4] the light sample alone, [5] the hit
 * normal alone (sums over reps); [6] a checksum; [7..14] with a walk-profile
 * build (SURF_WALK_PROFILE) the closest and any-hit walks' split: interior
 * cycles, leaf cycles, walks, leaves, triangles, two-level visits, prologue
 * cycles, instance-loop cycles (else 0).  No reference counterpart. */
int surf_debug_segment_cycles(surf_ctx* ctx, const float* path12, uint32_t reps, uint64_t* cycles15);
/* Diagnostics: the current sample stream's issue order.  permuted_frames is
 * the number of leading frames whose chain heads are issued heavy pixels
 * first (0: frame-major order throughout); heavy_pixels the size of that
 * heavy class (0 when permuted_frames is 0).  No reference counterpart. */
int surf_debug_issue_order(surf_ctx* ctx, uint32_t* heavy_pixels, uint32_t* permuted_frames);
/* Diagnostics: the emitters' BLAS staged in k_connect's LDS by the last phase
 * launched (blasAnyStaged): its compact interior records and its triangles,
 * both 0 when k_connect walked every BLAS from global memory.  No reference
 * counterpart. */
int surf_debug_connect_staging(surf_ctx* ctx, uint32_t* records, uint32_t* triangles);
/* Diagnostics: extension rays the capped lane walk left to k_extend_cont
 * (SURF_LANE_CAP) since the last surf_clear_accumulator.  No reference
 * counterpart. */
int surf_debug_lane_resumed(surf_ctx* ctx, uint64_t* rays);
/* When enabled, per-kernel device times are measured with HIP events on the
 * render stream (slower: disables the graph replay). */
int surf_set_profiling(surf_ctx* ctx, int enabled);

/* ---- scene / camera ---- */
int surf_upload_scene(surf_ctx* ctx, const surf_scene_desc* desc);
/* GPUScene::update's re-upload (scene.cpp:276-282): new instance records, TLAS
 * indices and nodes and lights for the uploaded BLASes/materials (same counts;
 * each instance must name a (node, index, triangle) offset triple of the
 * upload).  Drains the context first; geometry stays resident. */
int surf_update_instances(surf_ctx* ctx, const surf_gpu_instance* instances, uint32_t instance_count,
                          const uint32_t* tlas_indices, const surf_bvh_node* tlas_nodes, uint32_t tlas_node_count,
                          const surf_light* lights, uint32_t light_count);
int surf_set_camera(surf_ctx* ctx, const surf_camera_ubo* camera);

/* ---- rendering ----
 * Renders `frames` frames of samples_per_frame (spp) samples per pixel each,
 * as Renderer::render does per call (renderer.cpp:160-188): frame k is seeded
 * once per pixel with initSeed(pixel + 1799 * (first_sample_index + k * spp))
 * (renderer.cpp:169; first_sample_index = the accumulator's totalSamples
 * before this call, which is the frame index for spp 1), and its spp samples
 * run in sequence, sample j + 1's jitter, lens sample and path drawing from the
 * RNG state sample j's path left (renderer.cpp:171-181); (rgb, 1) is
 * accumulated per sample in sample order (renderer.cpp:180).  On the device a
 * frame's samples of one pixel form a chain: the kernel that ends sample j's
 * path (k_shade or a drain kernel) issues sample j + 1 in its place.
 * max_segments: 0 = unbounded + Russian roulette (reference semantics);
 * N > 0 caps each path at N extension rays.  Returns once every
 * sample is issued: consecutive calls form one sample stream, so the last long
 * paths of a call overlap the next call; any read (accumulator, stats,
 * finalize, synchronize) drains the stream first.  Scheduling only, identical
 * results (environment at surf_create, for A/B runs): a multi-frame call that
 * starts a stream issues every frame's samples of the pixels whose centre
 * camera ray first hits one of the largest BLASes first (SURF_REORDER=0:
 * frame-major); continuations are traced in the order of the large BLASes
 * they can reach, those reaching the most first (SURF_KEY=1: ascending,
 * 0: by start instance); each phase's shadow rays are
 * traced beside the next phase's extension (SURF_OVERLAP=0: serialized). */
int surf_render(surf_ctx* ctx, uint32_t frames, uint32_t first_sample_index,
                uint32_t max_segments, uint32_t samples_per_frame);
int surf_clear_accumulator(surf_ctx* ctx);
/* Float RGBA accumulator of this shard's rows, shard order, rows*width*4 floats. */
int surf_read_accumulator(surf_ctx* ctx, float* rgba_rows);
/* Device-to-device copy of the accumulator into dst (a device pointer on the
 * same device, rows*width*16 bytes): feeds the RCCL gather. */
int surf_copy_accumulator_device(surf_ctx* ctx, void* dst_device);
/* RGBA8 of acc / total samples with RgbaToU32 rounding, rows*width words. */
int surf_finalize_rgba8(surf_ctx* ctx, uint32_t* out_rgba8);
/* The displayed image: fs_quad.frag:22-24 (sqrt gamma) applied to the RGBA8
 * finalize image, written as 8-bit UNORM (round to nearest even), rows*width words. */
int surf_display_rgba8(surf_ctx* ctx, uint32_t* out_rgba8);
/* surf_finalize_rgba8 (display 0) / surf_display_rgba8 (display 1) of a host
 * accumulator, e.g. a frame assembled from row shards (surf_mgpu.h): n pixels
 * of RGBA floats times inv_samples, the same rounding as the kernels. */
int surf_pack_rgba8(const float* acc, uint32_t n, float inv_samples, int display, uint32_t* out_rgba8);
int surf_get_stats(surf_ctx* ctx, surf_stats* out);
int surf_synchronize(surf_ctx* ctx);

/* ---- traversal entry points (kernel-level parity tests) ----
 * n world-space rays, o/d 3 floats each.  closest: depth starts at 1e30;
 * writes t,u,v (floats) and inst,prim (u32, ~0 on miss).  any: tmax per ray,
 * occluded[i] = 1 when a hit is found. Host buffers. */
int surf_trace_closest(surf_ctx* ctx, uint32_t n, const float* o, const float* d,
                       float* out_t, float* out_u, float* out_v, uint32_t* out_inst, uint32_t* out_prim);
int surf_trace_any(surf_ctx* ctx, uint32_t n, const float* o, const float* d, const float* tmax,
                   uint8_t* occluded);
/* 0: one ray per lane (the wavefront kernels' traversal); 1: one ray per
 * 64-lane wave, lanes as the node record's planes (the drain's traversal; any
 * TLAS; needs a BVH stack of <= 64 entries).  Results are identical; selects
 * what surf_trace_* run. */
int surf_set_trace_mode(surf_ctx* ctx, int mode);

/* ---- host scene build (the reference's main.cpp scene, OBJ assets) ----
 * variant 0: bundled indoor scene; 1: C5 deep scene (+648 Suzannes in one mesh);
 * 2 / 3: general-TLAS test scenes (+40 / +80 scattered cube, Suzanne and lens
 * instances: 51 instances with the LDS tables, 91 with global tables). */
int surf_scene_build_indoor(const char* assets_dir, int variant, surf_scene** out);
int surf_scene_desc_get(const surf_scene* scene, surf_scene_desc* out);
/* GPUScene::update (sources/scene.cpp:267-282): rotate instance 3 by
 * 1.0*delta_time radians about WORLD_UP, refit the TLAS, re-batch.  Follow
 * with surf_update_instances (or surf_upload_scene) on each context. */
int surf_scene_update(surf_scene* scene, float delta_time);
/* Reference camera of main.cpp:141-149 for a width x height render. */
int surf_scene_camera(const surf_scene* scene, uint32_t width, uint32_t height, surf_camera_ubo* out);
/* Deepest root-to-leaf edge counts of the TLAS and of all BLASes. */
int surf_scene_bvh_depths(const surf_scene* scene, uint32_t* tlas_depth, uint32_t* max_blas_depth);
void surf_scene_destroy(surf_scene* scene);

/* Image files for an RGBA8 image (R in the low byte, as surf_finalize_rgba8 /
 * surf_display_rgba8 write it), rows top to bottom: binary PPM (P6, alpha
 * dropped) or PNG (8-bit RGBA, zlib).  The reference only presents to a
 * swapchain; these are its on-disk equivalent. */
int surf_write_ppm(const char* path, uint32_t width, uint32_t height, const uint32_t* rgba8);
int surf_write_png(const char* path, uint32_t width, uint32_t height, const uint32_t* rgba8);

/* Mesh::Mesh(path) (sources/mesh.cpp:69-154, tinyobjloader triangulate=true):
 * .obj or .obj.gz parsed in parallel chunks (threads = 0: default count).  The
 * triangles (64 B reference Triangle, OBJ corner 0 stored in v1) and
 * TriExtensions (80 B) are identical for every thread count. */
typedef struct surf_mesh surf_mesh;
int surf_obj_load(const char* path, uint32_t threads, surf_mesh** out);
int surf_mesh_data(const surf_mesh* mesh, const surf_triangle** triangles, const surf_tri_extension** tri_ext,
                   uint32_t* count);
void surf_mesh_destroy(surf_mesh* mesh);

/* BvhBLAS::build (sources/bvh.cpp:255-465: binned SAH, 8 bins, pre-order pair
 * allocation) over `count` reference Triangles, multi-threaded (threads = 0:
 * SURF_BUILD_THREADS / OMP_NUM_THREADS / hardware).  Writes the reference's
 * index permutation (count) and node pool (nodes_out needs 2*count records;
 * *nodes_used are written).  The arrays are identical for every thread count. */
int surf_bvh_build(const surf_triangle* triangles, uint32_t count, uint32_t threads, uint32_t* indices_out,
                   surf_bvh_node* nodes_out, uint32_t* nodes_used);

#ifdef __cplusplus
}  /* extern "C" */

static_assert(sizeof(surf_triangle) == 64, "Triangle is 64 B");
static_assert(sizeof(surf_tri_extension) == 80, "TriExtension is 80 B");
static_assert(sizeof(surf_bvh_node) == 48, "BvhNode is 48 B");
static_assert(sizeof(surf_material) == 64, "Material is 64 B");
static_assert(sizeof(surf_gpu_instance) == 160, "GPUInstance is 160 B");
static_assert(sizeof(surf_light) == 8, "GPULightData is 8 B");
static_assert(sizeof(surf_background) == 64, "SceneBackground is 64 B");
static_assert(sizeof(surf_camera_ubo) == 128, "CameraUBO is 128 B");
#endif

#endif /* SURF_HIP_H */
