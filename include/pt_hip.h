/*
 * pt_hip.h — C ABI of the MI355X path-tracing hot path (libpt_hip.so).
 *
 * This is the drop-in boundary for the per-pixel trace loop of the reference
 * (Blackgaurd/pathtracer-cpp). Every entry point below replaces one interface
 * of the reference; the replaced interface is cited as file:line into the
 * reference tree (pathtracer/...):
 *
 *   pt_render_f32 / pt_ctx_render   <- render_cpu()  render.h:62-104 (loop 80-88)
 *                                     render_gpu()  render.h:109-152 (tile loop 128-139)
 *                                     trace()       render.h:36-61
 *   pt_bvh_build                     <- BVH::build()  bvh.h:79-155 (find_best_axis 48-78)
 *   pt_camera_init                   <- Camera::Camera() camera.h:33-61
 *   pt_sample_seed                   <- rng.h:32 global LCG (stream policy, see below)
 *   pt_image_to_rgb8                 <- Image::gamma_correct + save_png quantisation
 *                                       image.h:41-62
 *
 * Plain C types only (no torch, no C++ types). All functions are synchronous
 * and must be called from one host thread per context. Return value: 0 on
 * success, a negative PT_E* code on failure; pt_last_error() describes it.
 *
 * Stream policy (the only intended behaviour change vs the reference): the
 * reference draws every random number from ONE global LCG (rng.h:32), which
 * makes pixel values depend on every earlier pixel and cannot be parallelised.
 * Here the same LCG (rng.h:14-20) is re-seeded before every sample with
 * pt_sample_seed(h*W + w, s, seed). trace()/get_ray()/the BVH are unchanged,
 * so with this seeding the GPU output is bit-identical to the reference's
 * render loop run with the same per-sample reseed (tests/golden).
 */
#ifndef PT_HIP_H
#define PT_HIP_H

#if !defined(__HIPCC_RTC__)  /* hipRTC (scene-specialised kernels) provides the fixed-width types */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define PT_ABI_VERSION 3

/* Reference constants (linalg.h:10-12, render.h:16, rng.h:3). */
#define PT_SEED 1u
#define PT_MAX_DEPTH 64          /* kernel limit on `depth` (reference GL path: 20, shader.h:35) */

/* Error codes. */
#define PT_OK 0
#define PT_E_ARG (-1)            /* invalid argument (null pointer, bad size, bad node graph) */
#define PT_E_EMPTY (-2)          /* no triangles in scene (render.h:64-67)                 */
#define PT_E_HIP (-3)            /* HIP runtime error (no device, launch failure, OOM)      */
#define PT_E_IO (-4)             /* file write failure (image.h:61)                         */
#define PT_E_RUNAWAY (-5)        /* specular rejection loop hit its bound   */

/* Material type values, identical to Material::Type (material.h:28-32). */
#define PT_MAT_EMIT 1
#define PT_MAT_DIFFUSE 2
#define PT_MAT_SPECULAR 3

/* BVHNode in the reference's own 40-byte AoS layout (bvh.h:12-16):
 * AABB {vec3 lb, rt} then int left, right, tri_start, tri_end.
 * Leaf <=> left == -1 && right == -1 (bvh.h:25-27). */
typedef struct pt_bvh_node {
    float lb[3];
    float rt[3];
    int32_t left, right;
    int32_t tri_start, tri_end;
} pt_bvh_node;

/* Material in the reference's 32-byte layout (material.h:27-37). */
typedef struct pt_material {
    int32_t type;                /* PT_MAT_* */
    float color[3];              /* albedo (surface_color, render.h:56) */
    float emit[3];               /* emit_color (render.h:45, 55)        */
    float roughness;             /* specular jitter scale (material.h:21) */
} pt_material;

/* A scene = the arrays a built BVH owns (bvh.h:32-34). Host pointers, caller-owned. */
typedef struct pt_scene {
    int32_t num_tris;
    const float* verts;          /* num_tris * 9 floats: v1, v2, v3 of triangle i (triangle.h:10) */
    const pt_material* materials;/* num_tris entries, material of triangle i                    */
    int32_t num_nodes;
    const pt_bvh_node* nodes;    /* num_nodes entries, root = 0                                 */
    const int32_t* tri_idx;      /* num_tris entries (bvh.h:33)                                  */
} pt_scene;

/* Camera parameters the ray generator reads (camera.h:19-25, get_ray 63-73),
 * precomputed on the host by pt_camera_init. transform holds the 3x3 rotation
 * rows right, up, -forward (camera.h:55-57). */
typedef struct pt_camera {
    float pos[3];
    int32_t res[2];              /* width, height */
    float v_res[2];
    float cell_size;
    float distance;
    float transform[9];          /* row-major 3x3 */
} pt_camera;

/* Progress of a render (optional, pt_params.progress): `done` of `total` pixel-samples
 * are complete. Called from the rendering call's own threads (one at a time, never
 * concurrently), with done increasing to total; the drop-in render_cpu / render_gpu turn
 * it into the reference's per-row / per-chunk console lines (render.h:87, 136). */
typedef void (*pt_progress_fn)(void* user, int64_t done, int64_t total);

/* Render parameters. */
typedef struct pt_params {
    int32_t spp;                 /* samples per pixel (render_*: `samples`) */
    int32_t depth;               /* max path segments (render_*: `depth`)   */
    uint32_t seed;               /* stream seed, PT_SEED for the reference  */
    int32_t part_index;          /* row partition for multi-GPU: this part  */
    int32_t part_count;          /*   number of parts (1 = whole image)     */
    int32_t band_rows;           /*   rows per band; row h belongs to part (h / band_rows) % part_count */
    int32_t batch_spp;           /* samples per accumulation batch (radiance slab of 12 B per
                                    sample and pixel), 0 = auto. With several batches two slabs
                                    alternate (fused accumulation) when both fit the slab budget;
                                    an explicit batch that does not fit twice is summed by a
                                    separate pass instead, never resized */
    int32_t samples_per_item;    /* samples per work item (lane-level scheduling unit), 0 = auto */
    pt_progress_fn progress;     /* NULL = no progress reports                */
    void* progress_user;         /*   its first argument                      */
} pt_params;

#define PT_MAX_DEVICES 16        /* devices of one pt_render_*_devices call */

/* Statistics of one render call. */
typedef struct pt_stats {
    uint64_t rays;               /* traced segments = BVH::intersect calls (bvh.h:156) */
    uint64_t paths;              /* camera samples */
    uint64_t runaway;            /* specular rejection loops that hit the bound (0 normally) */
    double kernel_ms;            /* sum of trace-kernel durations (HIP events); devices: the slowest part's */
    double reduce_ms;            /* sum of accumulate-kernel durations           */
    double total_ms;             /* end-to-end wall time of the call             */
    int32_t trace_launches;      /* number of trace-kernel launches              */
    int32_t rows;                /* rows rendered by this part                    */
    int32_t kernel_path;         /* PT_PATH_*: which trace kernel ran              */
    /* pt_render_*_devices only (zero otherwise): */
    int32_t n_devices;           /* parts = listed devices                                     */
    int32_t gather_path;         /* PT_GATHER_*: how the parts met                              */
    double gather_ms;            /* RCCL gather + row assembly on the first device (HIP events) */
    double device_kernel_ms[PT_MAX_DEVICES];  /* per part: trace-kernel time                  */
    double device_render_ms[PT_MAX_DEVICES];  /* per part: context + scene upload + render    */
    uint64_t device_rays[PT_MAX_DEVICES];     /* per part: traced segments                    */
} pt_stats;

/* pt_stats.gather_path values. */
#define PT_GATHER_NONE 0         /* single context                                          */
#define PT_GATHER_RCCL 1         /* RCCL send/recv group to the first device + device assembly */
#define PT_GATHER_HOST 2         /* parts copied to the host, rows placed there (a device listed
                                    twice, or PT_TEST_HOOKS=1 PT_GATHER=host) */
#define PT_GATHER_HOST_FALLBACK 3 /* as PT_GATHER_HOST, because RCCL was unavailable or its group
                                    failed (that set of communicators aborted and dropped; a
                                    line on stderr for every such frame) */

/* pt_stats.kernel_path values. */
#define PT_PATH_TREE_GLOBAL 0    /* child-pair tree walk, scene read through L1/L2 */
#define PT_PATH_TREE_LDS 1       /* child-pair tree walk, scene in LDS             */
#define PT_PATH_FLAT_TABLE 2     /* flat leaf list, generic kernel-argument table  */
#define PT_PATH_FLAT_RTC 3       /* flat leaf list, hipRTC scene-specialised kernel */
#define PT_PATH_WIDE 4           /* wide (4/8-child) tree walk, scene read through L1/L2 */
#define PT_PATH_FLAT_TABLE_FAST 5 /* flat leaf list, kernel-argument table with the scene's flags */

/* ---- stream policy ---------------------------------------------------- */
#if defined(__HIPCC__)
#define PT_INLINE static inline __host__ __device__
#else
#define PT_INLINE static inline
#endif
/* lowbias32 integer finaliser (public-domain constants). */
PT_INLINE uint32_t pt_mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
/* LCG state for sample `sample` of pixel `pixel` = h * W + w (h = 0 is the bottom
 * row, as Image::pixels, image.h:11). */
PT_INLINE uint32_t pt_sample_seed(uint32_t pixel, uint32_t sample, uint32_t seed) {
    return pt_mix32(pt_mix32(pt_mix32(seed) ^ pixel) + sample);
}

/* ---- library / errors ------------------------------------------------- */
int pt_abi_version(void);
const char* pt_last_error(void);
int pt_device_count(void);

/* ---- host-side scene preparation (replaces BVH::build, Camera ctor) ---- */
/* Build the reference's SAH BVH (bvh.h:79-155) over num_tris triangles.
 * nodes_out must hold 2*num_tris-1 entries, tri_idx_out num_tris entries.
 * Returns the node count (>0) or a negative error code. The output is
 * bit-identical to BVH::build (same nodes, order, boxes, tri_idx). */
int pt_bvh_build(int32_t num_tris, const float* verts, pt_bvh_node* nodes_out,
                 int32_t* tri_idx_out);

/* Camera ctor arithmetic (camera.h:33-61). fov in radians. Returns PT_E_ARG
 * when forward and up are nearly parallel (camera.h:41-45). */
int pt_camera_init(const float pos[3], const float forward[3], const float up[3],
                   int32_t res_x, int32_t res_y, float fov, float distance,
                   pt_camera* out);

/* Validate a scene's node graph and report how the kernel will traverse it
 * (no device needed). info (may be NULL) receives: [0] reachable nodes,
 * [1] tree depth, [2] leaves on the exact flat path (0 = tree traversal),
 * [3] reference LIFO stack bound. Same checks as pt_ctx_set_scene. */
int pt_scene_validate(const pt_scene* scene, int32_t info[4]);
/* Extended form: info[0..3] as pt_scene_validate, then [4] wide nodes (0 = no wide
 * tree), [5] wide width, [6] wide levels, [7] wide nodes staged in LDS, [8] triangles in
 * wide-leaf order, [9] bytes per wide triangle record (48: vertices only, the leaf box is
 * the triangle's AABB; 64: with the stored leaf box; 0 = no wide tree).
 * Writes min(n, PT_SCENE_INFO_N) entries; returns PT_SCENE_INFO_N. */
#define PT_SCENE_INFO_N 10
int pt_scene_info(const pt_scene* scene, int32_t* info, int32_t n);

/* ---- rendering --------------------------------------------------------- */
typedef struct pt_ctx pt_ctx;

/* Create a context bound to HIP device `device` (its own stream). */
int pt_ctx_create(int device, pt_ctx** out);
void pt_ctx_destroy(pt_ctx* ctx);

/* Pack the scene to the device layout (SoA, tri_idx order) and upload it. A flat
 * scene (<= 64 leaves) also starts compiling its scene-specialised kernel (hipRTC,
 * ~0.4 s) on a background thread: renders do not wait for it; their launches run the
 * generic flat kernel until it is ready and then switch to it (bit-identical images
 * either way). */
int pt_ctx_set_scene(pt_ctx* ctx, const pt_scene* scene);

/* Wait for the scene's background preparation (the hipRTC compile) and load its result,
 * so every later render runs the specialised kernel. Optional. */
int pt_ctx_prepare(pt_ctx* ctx);

/* Wait for every background scene-kernel compile of the process; returns how many were still
 * running. No compile is left running at exit either way (the library waits in an exit
 * handler), but a host whose own teardown changes signal handlers before the C exit handlers
 * run (Python's faulthandler is disabled in interpreter finalisation) calls it first: the
 * Python package does, at interpreter exit. */
int pt_rtc_wait(void);

/* Render this part's rows. Output is the linear per-pixel mean after /spp
 * (image.h:37-40), float32 RGB, rows of this part in increasing h, h = 0
 * first. `out` is a DEVICE pointer when out_is_device != 0 (e.g. a torch
 * tensor on the context's device), otherwise a host pointer. Size:
 * pt_part_rows(...) * res_x * 3 floats. The call returns after the result is
 * complete (the context's stream is synchronised). */
int pt_ctx_render(pt_ctx* ctx, const pt_camera* cam, const pt_params* params,
                  float* out, int out_is_device, pt_stats* stats);

/* Progressive rendering (render_realtime's frame accumulation, render.h:219-387, offscreen):
 * adds samples [s_first, s_first + s_count) of this part to the context's running sum and
 * writes the running mean. s_first == 0 starts a new sum; otherwise s_first must equal the
 * samples already summed with the same camera and depth/seed/partition (else PT_E_ARG).
 * After every call the image is bit-identical to pt_ctx_render with spp = s_first +
 * s_count (params->spp is ignored). Any other render on the context ends the sum. */
int pt_ctx_render_progressive(pt_ctx* ctx, const pt_camera* cam, const pt_params* params, int32_t s_first,
                              int32_t s_count, float* out, int out_is_device, pt_stats* stats);

/* pt_ctx_render followed by gamma_correct + save_png quantisation on the device
 * (image.h:41-55): out receives rows*W*3 bytes of this part (row order as pt_ctx_render;
 * flip != 0 reverses it: top row first, as the PNG of a whole image), equal to
 * pt_image_to_rgb8 of the linear image. Requires gamma > 0. */
int pt_ctx_render_rgb8(pt_ctx* ctx, const pt_camera* cam, const pt_params* params, float gamma, int flip,
                       uint8_t* out, int out_is_device, pt_stats* stats);

/* Number of rows of part `part_index` for the given partition. */
int32_t pt_part_rows(int32_t res_y, int32_t part_index, int32_t part_count, int32_t band_rows);

/* One-shot: create context on device params->... (device 0), upload, render
 * the whole image (part 0 of 1) into host out_rgb (res_x*res_y*3 floats). */
int pt_render_f32(const pt_scene* scene, const pt_camera* cam, const pt_params* params,
                  float* out_rgb, pt_stats* stats);

/* One-shot on several GPUs of this process: part p of the row partition (bands of
 * params->band_rows rows, default 1; row h -> part (h / band) % n_devices) renders on
 * devices[p] from its own host thread into device memory; with distinct devices the
 * parts are gathered to devices[0] by one RCCL group of ncclSend/ncclRecv (communicators
 * from ncclCommInitAll, cached per device list) and assembled there, then copied to
 * out_rgb (the whole image, as pt_render_f32). A device may be listed more than once
 * (then the rows are assembled on the host). The image is bit-identical for any device
 * list (per-sample seeding); stats: rays/paths summed, kernel_ms the slowest part's,
 * per-device times and rays, gather path and time. Replaces render_gpu's tile loop on
 * one GL context (render.h:109-152, tiles 128-139) with every visible GPU. */
int pt_render_f32_devices(const pt_scene* scene, const pt_camera* cam, const pt_params* params,
                          const int32_t* devices, int32_t n_devices, float* out_rgb, pt_stats* stats);
/* As pt_render_f32_devices, then gamma_correct + save_png quantisation (image.h:41-55) on
 * devices[0] after the gather: rgb8 receives res_x*res_y*3 bytes, top row first, equal to
 * pt_image_to_rgb8 of the linear image (a quarter of its device-to-host bytes). */
int pt_render_rgb8_devices(const pt_scene* scene, const pt_camera* cam, const pt_params* params,
                           const int32_t* devices, int32_t n_devices, float gamma, uint8_t* rgb8,
                           pt_stats* stats);

/* ---- post-process (image.h:41-62) -------------------------------------- */
/* gamma (powf(x, 1/gamma)), clamp to [0,1], *255, truncate, vertical flip:
 * rgb8 is top row first, as the PNG written by Image::save_png. */
int pt_image_to_rgb8(const float* linear_rgb, int32_t res_x, int32_t res_y, float gamma,
                     uint8_t* rgb8);
/* Thresholds of the device quantiser for gamma > 0: thr255[k-1] = the least float x >= 0
 * whose 8-bit value under pt_image_to_rgb8 (host powf) is >= k, k = 1..255; *neg_mode
 * (if non-NULL) = how a negative value quantises: 0 -> 255 (NaN power), 1 -> 0 (odd
 * integer exponent), 2 -> as |x| (even integer exponent). */
int pt_rgb8_thresholds(float gamma, float* thr255, int32_t* neg_mode);
/* ---- OBJ/MTL ingestion: BVH::load_obj (bvh.h:184-242) through the reference's
 * vendored tinyobjloader (triangulation, number parsing and MTL rules restated in
 * csrc/pt_obj.cpp). Triangles come out in the order load_obj adds them. */
typedef struct pt_obj pt_obj;
/* Parse `filename`; MTL files are searched in mtl_search_path (':'-separated; NULL or
 * "" = the OBJ file's directory, as ObjReader::ParseFromFile). PT_E_IO if the file
 * cannot be opened; PT_E_ARG for a malformed face line, a face without a material or
 * a vertex index past the end (the reference's undefined behaviour). */
int pt_obj_load(const char* filename, const char* mtl_search_path, pt_obj** out);
int32_t pt_obj_num_tris(const pt_obj* obj);
/* verts: 9 floats per triangle (v1, v2, v3); mats: the bvh.h:220-238 mapping
 * (illum 1 -> DIFFUSE(Kd), 2 -> EMIT(Ka), else DIFFUSE(0.5)); illum: the MTL value
 * behind each triangle (load_obj reports "Unknown material type" for the others).
 * Any output may be NULL. */
int pt_obj_triangles(const pt_obj* obj, float* verts, pt_material* mats, int32_t* illum);
/* tinyobjloader-style warnings collected while parsing ("" if none). */
const char* pt_obj_warnings(const pt_obj* obj);
void pt_obj_free(pt_obj* obj);

/* Write an 8-bit RGB PNG (top row first). */
int pt_write_png(const char* filename, const uint8_t* rgb8, int32_t res_x, int32_t res_y);

/* ---- cached multi-device contexts ------------------------------------- */
/* pt_render_*_devices keep one context per listed device (keyed by the device list) and
 * the scene last uploaded to it, so a process that renders several scenes or frames in a
 * row (the reference's modified_cornell.cc renders six, modified_cornell.cc:14, 107) pays
 * context creation once and re-uploads a scene only when its arrays change. This frees
 * every cached context and its device memory (radiance slabs, scene, part buffers). Safe
 * to call at any time; a later pt_render_*_devices call creates fresh contexts. */
void pt_devices_release(void);

#ifdef __cplusplus
}
#endif
#endif /* PT_HIP_H */
