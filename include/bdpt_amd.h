/*
 * bdpt_amd — MI355X-native bidirectional path tracer: the C-ABI drop-in
 * boundary for the reference's BDPT hot path.
 *
 * Reference (JackMinn/Bidirectional-Path-Tracing) interfaces these entry points
 * replace:
 *   bdpt_scene_load_obj      Scene::load                      src/core/renderer.cpp:235-315
 *                            (tinyobj LoadObj :249, BSDFs per illum :258-271,
 *                             emitters :279-305, AcceleratorBVH::build accel.h:115-123)
 *   bdpt_scene_create        the Scene the Integrator holds (core.h:352-358: worldData, bsdfs,
 *                            emitters, bvh) handed over from the caller's memory
 *   bdpt_camera_constants    camera set-up of Renderer::render renderer.cpp:140-153
 *                            and BDPTIntegrator bdpt.h:49-54, :485-489
 *   bdpt_ctx_create          Integrator::init (rgb allocation) src/core/integrator.cpp:16-20
 *                            + upload of the Scene the integrator holds by reference
 *   bdpt_render              the offline loop of Renderer::render renderer.cpp:130-214
 *                            calling BDPTIntegrator::render bdpt.h:219-241 for every
 *                            (pixel, sample), with camera splats (bdpt.h:295-371)
 *                            accumulated into the same framebuffer
 *   bdpt_render_sample_mt    virtual v3f Integrator::render(const Ray&, Sampler&) const
 *                            src/core/integrator.h:31, overridden at bdpt.h:219, with the
 *                            caller's Sampler (std::mt19937 state, src/core/math.h:63-76)
 *   bdpt_render_sample       the same, Sampler given as (seed, draws already taken)
 *   bdpt_bsdf_eval/pdf/sample  BSDF::eval / pdf / sample        src/core/core.h:308-310
 *                            (diffuse.h:35-61, perfectmirror.h:33-59, glass.h:55-108,
 *                             mixture.h:60-151, phong.h) of a scene material, batched
 *   bdpt_intersect           AcceleratorBVH::intersect / occlusion  src/core/accel.h:125-172,
 *                            externals/bvh.h:259-352 (as visibilityQuery calls it, bdpt.h:498-505)
 *   bdpt_splat_to_image_plane  BDPTIntegrator::splatToImagePlane   bdpt.h:485-496
 *   bdpt_ctx_destroy         Integrator/Renderer teardown (renderer.cpp:221-227)
 *   bdpt_config_load_toml    loadTOML                         src/main.cpp:22-116
 *   bdpt_save_exr            Integrator::save -> saveEXR      integrator.cpp:26-30, utils.h:95-156
 *   (CLI lib/tinyrender_amd) main / run                       src/main.cpp:121-181
 *   bdpt_render_path         PathTracerIntegrator::render     src/integrators/path.h:235-245 for every
 *                            (pixel, sample) of the offline loop (the reference's other offline
 *                            integrator, TOML type = "path"), on the same GPU substrate
 *   bdpt_render_direct       DirectIntegrator::render         src/integrators/direct.h:449-462 (TOML
 *                            type = "direct": area / solidAngle / cosineHemisphere / bsdf / mis)
 *
 * Conventions: plain C types only; status 0 = OK, < 0 = error (message from
 * bdpt_last_error(), thread-local). A context is bound to one HIP device and is
 * not thread-safe: callers that render from several threads (the reference's
 * parallel_for, renderer.cpp:157) keep one context per thread. Calls on one
 * context are ordered even across streams (each call waits for the previous
 * call's work on its stream before touching the context's buffers). Nothing
 * here falls back to the CPU: without a HIP device, bdpt_ctx_create fails with
 * BDPT_ERR_NO_DEVICE.
 *
 * Determinism: camera sample (pixel p, sample k) draws from
 * std::mt19937(seed_base + p*spp + k) exactly like the reference's Sampler
 * (src/core/math.h:63-76), and all arithmetic follows the reference's single-
 * precision operation order, so paths are identical to the CPU reference; only
 * the order of floating-point additions into the framebuffer differs.
 */
#ifndef BDPT_AMD_H
#define BDPT_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BDPT_OK 0
#define BDPT_ERR_INVALID -1
#define BDPT_ERR_IO -2
#define BDPT_ERR_NO_DEVICE -3
#define BDPT_ERR_HIP -4
#define BDPT_ERR_UNSUPPORTED -5

/* Strategy switches of the reference (bdpt.h:16-17, compile-time there). */
#define BDPT_STRATEGY_BDPT 0
#define BDPT_STRATEGY_LIGHT_TRACING 1
#define BDPT_STRATEGY_PATH_TRACING 2

/* bdpt_frame_params.flags */
#define BDPT_FLAG_COUNT 1u            /* counting pass: fill bdpt_stats.counters (slower) */
#define BDPT_FLAG_FULL_TRAVERSAL 2u   /* visit every box the reference visits (no t-culling) */
/* (bit 2, the round-1 wavefront schedule, was removed: the megakernel beat it ~5x; now BDPT_ERR_UNSUPPORTED) */

typedef struct bdpt_scene bdpt_scene; /* host-side ingested scene */
typedef struct bdpt_ctx bdpt_ctx;     /* device context (one HIP device) */

typedef struct {
    int64_t triangles, bvh_nodes, shapes, materials, emitters, bvh_max_depth;
    int64_t device_bytes; /* HBM bytes of the uploaded scene arrays */
    int64_t bvh_leaves;   /* reference BVH leaves (<= 4 triangles each) */
    int64_t wide_nodes;   /* 4-wide traversal nodes */
    int64_t wide_depth, wide_max_stack;
    int64_t wide_leaves;  /* leaves of the traversal tree */
    int64_t triangle_tree; /* 1: SAH tree over single triangles (default); 0: over the reference
                              leaves (environment BDPT_TRAV_TREE=refleaf at scene load) */
} bdpt_scene_info;

typedef struct {
    float eye[3], at[3], up[3]; /* [camera] eye / at / up (main.cpp:31-37) */
    float fov;                  /* degrees */
} bdpt_camera;

typedef struct {
    bdpt_camera camera;
    int32_t width, height; /* [film] (the global image; shards still splat into it) */
    int32_t spp;           /* [renderer] spp */
    int32_t rr_depth;      /* [renderer] rrDepth (bdpt.h:39): with russian_roulette 0 the hard path-depth
                              cap (NO_RR = 1, bdpt.h:18), else where Russian roulette starts; 1..1024 */
    int32_t strategy;      /* BDPT_STRATEGY_* (reference default: BDPT) */
    uint32_t seed_base;    /* 260450963 = the reference's Sampler seed (renderer.cpp:155) */
    int32_t row_offset;    /* shard: render rows row_offset, row_offset+row_stride, ... */
    int32_t row_stride;    /*        (1 = whole image)                                   */
    uint32_t flags;        /* BDPT_FLAG_* */
    int32_t russian_roulette; /* BDPT_RR_*: 0 = the reference as shipped (NO_RR 1, bdpt.h:18); 1 = its
                                 NO_RR 0 branch (bdpt.h:68, :129-132, :188, :201-204) */
} bdpt_frame_params;

/* bdpt_frame_params.russian_roulette */
#define BDPT_RR_NONE 0      /* NO_RR 1: every subpath stops at rrDepth (one draw at the cap) */
#define BDPT_RR_LUMINANCE 1 /* NO_RR 0: past rrDepth a subpath continues while sampler.next() < rr, with
                               rr = (luminance(throughput) < 0.01 ? 0.5 : 1) stored per vertex and entering
                               every pdf (rr * pdf); no depth cap (see bdpt_stats.capped_samples) */

#define BDPT_NUM_COUNTERS 32
/* counters: [0] closest-hit rays, [1] shadow rays, [2] interior-node visits,
 * [3] triangle tests, [4] light vertices stored, [5] light-vertex reads,
 * [6] camera splats, [7] RNG draws; SIMD-efficiency probes: [8] traversal
 * iterations summed over lanes, [9] the same counted once per wave, [10]
 * state-machine actions summed over lanes, [11] action executions per wave;
 * wave clocks (s_memtime, summed over waves): [12] in traversal, [13] in the
 * state advance, [14] whole persistent loop; [15] exact slab fallbacks;
 * traversal-stack depth probes (after each 4-wide node): [16] entries held
 * beyond depth 8, [17] beyond 12, [18] beyond 16; [19] stack entries culled on pop;
 * wave clocks per state-machine step (megakernel): [20] query resolve, [21] eye start,
 * [22] eye vertex, [23] emitter sample, [24] light start, [25] next-event estimation,
 * [26] light vertex + camera connection, [27] vertex connections, [28] BSDF continuation,
 * [29] light-walk loop test, [30] eye-walk loop test, [31] sample finish. */
typedef struct {
    double kernel_ms;      /* HIP-event time of the render kernel(s) of the last call */
    int64_t samples;       /* camera samples rendered by the last call */
    int64_t launches;      /* kernel launches of the last call */
    int64_t counters[BDPT_NUM_COUNTERS];
    int64_t capped_samples; /* Russian roulette: samples of the last call that met a bound the reference
                               does not have - more than max(255, rr_depth - 1) stored light vertices, or
                               2^25 bounces in one subpath (> 0 means the frame is not the reference's,
                               and bdpt_render_host fails) */
    double span_ms;         /* BDPT frame kernel, device clock: first wave start -> last wave exit */
    double tail_ms;         /* BDPT frame kernel, device clock: the frame's last 64-sample chunk claimed ->
                               last wave exit (the end tail a persistent grid pays per launch) */
    int64_t max_light_depth; /* counting pass (BDPT_FLAG_COUNT) maxima over the samples: light-subpath */
    int64_t max_eye_depth;   /* depth, eye-subpath depth, */
    int64_t max_queries;     /* ray queries of one sample */
    int64_t schedule_errors; /* MT19937 draws past the generated ring (or a ring left by another sample), a
                                continuation walk out of stack
                                (any non-zero count is a bug, and bdpt_render_host fails) */
    int64_t sched[4];        /* counting pass (BDPT_FLAG_COUNT), the connection tasks a wave holds when it
                                shades (connectVertices still to run, connectToLight + the connections of a
                                new eye vertex, connectToCamera of a new light vertex): summed over the
                                shading steps, the shading steps, steps with >= 32 and with >= 64 tasks.
                                Builds whose waiting lanes walk the shadow rays (BDPT_HELP): tasks pushed,
                                pushes refused (ring full), claim rounds, tasks claimed */
    int64_t parked_samples;  /* Russian roulette: walks handed to the continuation pass's chain kernel
                                (deeper than BDPT_PARK_DEPTH bounces; a sample may be handed over again) */
    int64_t rr_long_walks_max;  /* Russian roulette: the most subpaths deeper than 512 bounces one wave held
                                   at once (such a wave stops refilling: express mode) */
    int64_t rr_express_iters[3]; /* Russian roulette: loop iterations of express-mode waves holding 1, 2..4,
                                    more than 4 such subpaths (up to 4 are walked in turn by the whole wave) */
} bdpt_stats;

const char* bdpt_last_error(void);
const char* bdpt_version(void);

/* ---- host-side scene ingest (no GPU needed) ---- */
int bdpt_scene_load_obj(const char* obj_path, bdpt_scene** out);
int bdpt_scene_free(bdpt_scene* scene);
int bdpt_scene_get_info(const bdpt_scene* scene, bdpt_scene_info* out);
/* Reference-layout export (tests): tri_f32[ntri][18] = v0 v1 v2 n0 n1 n2 in BVH
 * leaf order, tri_i32[ntri][3] = shapeID primID matID, node_f32[nnodes][6] =
 * bbox min/max, node_u32[nnodes][3] = start nPrims rightOffset (flat preorder). */
int bdpt_scene_export(const bdpt_scene* scene, float* tri_f32, int32_t* tri_i32, float* node_f32, uint32_t* node_u32);
/* Traversal-tree export (tests; wide_bvh.hpp): wnodes[wide_nodes][32] (8 float4:
 * child lo.x hi.x lo.y hi.y lo.z hi.z link-bits unused), wtri[triangles][12]
 * (v0|ref index bits, e1|ref leaf id bits, e2|0), lbox[bvh_leaves][8] (lo|0 hi|0),
 * root_link. Any pointer may be NULL. */
int bdpt_scene_export_traversal(const bdpt_scene* scene, float* wnodes, float* wtri, float* lbox, uint32_t* root_link);

/* ---- scene hand-over from the caller's in-memory Scene (src/core/core.h:352-358) ----
 * What Scene::load built (renderer.cpp:235-315), as plain arrays: the caller
 * flattens WorldData, its bsdfs, emitters and the AcceleratorBVH it already has
 * (INTEGRATION.md §2 does it from the reference's own types); nothing is
 * re-parsed or rebuilt, and the result is the same bdpt_scene the OBJ path
 * gives for the same file (bit-identical device arrays, bdpt_scene_export_layout). */
typedef struct {
    int32_t illum;             /* tinyobj material_t::illum: 7 diffuse, 3 mirror, 6 glass, 8 mixture, 5 null,
                                  anything else Phong (renderer.cpp:258-271) */
    float kd[3], ks[3], ke[3], tf[3]; /* diffuse, specular, emission, transmittance */
    float ns, ni;              /* shininess, ior */
    float scale, spec_weight;  /* MixtureBSDF / PhongBSDF::scale, ::specularSamplingWeight as constructed
                                  (mixture.h:39-46, phong.h:40-47); unused by the other kinds */
    int32_t has_texture;       /* non-zero: a bitmap texture (diffuse_/specular_texname) — rejected */
} bdpt_material_desc;
typedef struct {
    int32_t shape;             /* Emitter::shapeID */
    float area;                /* Emitter::area */
    float radiance[3];         /* Emitter::radiance */
    int32_t ncdf;              /* faceAreaDistribution.cdf.size() (= the shape's faces + 1) */
    const float* cdf;          /* faceAreaDistribution.cdf, normalized */
} bdpt_emitter_desc;
typedef struct {
    float bmin[3], bmax[3];    /* BVHFlatNode::bbox.min / max (externals/bvh.h:102-105) */
    uint32_t start, nprims, right_offset;
} bdpt_bvh_node_desc;
typedef struct {
    int64_t triangles;         /* AcceleratorBVH::objects.size() */
    const float* positions;    /* [triangles][9] v0 v1 v2, shape by shape, faces in mesh.indices order
                                  (the order AcceleratorBVH::build creates its objects, accel.h:115-123) */
    const float* normals;      /* [triangles][9] the corners' normals (attrib.normals[normal_index]) */
    const int32_t* tri_shape;  /* [triangles] shapeID */
    const int32_t* tri_prim;   /* [triangles] primID = faceID / 3 */
    const int32_t* tri_mat;    /* [triangles] mesh.material_ids[primID] */
    int32_t shapes;            /* worldData.shapes.size() */
    int32_t materials;         /* worldData.materials.size() = bsdfs.size() */
    const bdpt_material_desc* material;
    int32_t emitters;          /* Scene::emitters.size() */
    const bdpt_emitter_desc* emitter;
    int64_t bvh_nodes;         /* nodes of BVH::flatTree reachable from the root (preorder) */
    const bdpt_bvh_node_desc* bvh;
    const int32_t* bvh_order;  /* [triangles]: the triangle (index into the arrays above) that
                                  AcceleratorBVH::objects[i] (= BVH::build_prims[i] after the build) is */
} bdpt_scene_desc;
/* Validates the descriptor (order, ranges, the BVH's layout and box nesting) and
 * copies it; the caller's arrays may be freed afterwards. BDPT_ERR_INVALID with a
 * message when it is inconsistent. */
int bdpt_scene_create(const bdpt_scene_desc* desc, bdpt_scene** out);
/* The scene's device arrays as uploaded by bdpt_ctx_create (the
 * same transforms: shade records widened with v0 and the triangle's near-cull
 * graze code in the shape word's top byte, mixture records with Ks = 0 as
 * diffuse, emitter faces with their graze code), for
 * checking that two ingest paths agree bit for bit: 0 tri, 1 shade, 2 nodes (the
 * reference's binary tree), 3 wnodes, 4 wtri, 5 lbox, 6 BSDF records, 7 emitter
 * records, 8 emitter faces, 9 emitter CDFs, 10 shape -> emitter, 11 roots / tree
 * sizes (uint32 root_link, wroot_link, wmax_stack, wdepth), 12 the BSDF records
 * as ingested (before the upload's mixture -> diffuse rewrite). *bytes = the
 * array's size; dst may be NULL (size only), else it must hold *bytes on entry. */
#define BDPT_LAYOUT_ARRAYS 13
int bdpt_scene_export_layout(const bdpt_scene* scene, int32_t array, void* dst, int64_t* bytes);
/* Camera constants: worldToCamera, cameraToWorld, cameraToClip, NDCToScreen
 * (column-major) then invWidth, invHeight, tan(fov/2), aspect, forward.xyz,
 * virtual near-plane distance — 72 floats. */
int bdpt_camera_constants(const bdpt_camera* cam, int32_t width, int32_t height, float out[72]);

/* ---- device ---- */
int bdpt_device_count(int32_t* count);
int bdpt_ctx_create(const bdpt_scene* scene, int32_t hip_device, bdpt_ctx** out);
int bdpt_ctx_destroy(bdpt_ctx* ctx);

/* Renders every (pixel, sample) of the shard and ADDS the result to fb_device
 * (device pointer, width*height*3 floats, pixel-major RGB, row 0 = top): eye
 * estimates acc/spp per pixel plus every light-path camera splat (which may land
 * on rows outside the shard). Asynchronous on `hip_stream` (hipStream_t; NULL =
 * the context's own stream); timing is read with bdpt_get_stats after a sync. */
int bdpt_render(bdpt_ctx* ctx, const bdpt_frame_params* params, float* fb_device, void* hip_stream);
/* Same, with a host framebuffer (copied to the device, accumulated, copied back). Synchronous. */
int bdpt_render_host(bdpt_ctx* ctx, const bdpt_frame_params* params, float* fb_host);
/* ---- Integrator::render(const Ray&, Sampler&): one camera sample ---- */
/* The reference's Sampler (math.h:63-76) is a std::mt19937 plus a stateless
 * uniform_real_distribution<float>. Its state crosses the ABI as libstdc++ streams
 * it (operator<< / operator>> of std::mersenne_twister_engine): the 624 state words
 * _M_x, then the position _M_p (0..624). */
#define BDPT_MT19937_WORDS 625
typedef struct {
    int32_t pixel; /* index into the W*H framebuffer (row-major, row 0 = top) */
    float rgb[3];  /* radiance * misWeight, added as rgb[pixel] += ... (bdpt.h:363-370) */
} bdpt_splat;
/* The state of std::mt19937(seed) after `draws` outputs (host only). */
int bdpt_sampler_state(uint32_t seed, int64_t draws, uint32_t state[BDPT_MT19937_WORDS]);
/* BDPTIntegrator::render(ray, sampler) (bdpt.h:219-241): ray = o.xyz d.xyz min_t max_t;
 * `state` is the caller's sampler, advanced in place exactly as the reference
 * advances it. Returns Li; the camera splats of the sample's light subpath are
 * returned in order in splats[0 .. *nsplats) for the caller to add to its image
 * (at most rr_depth without Russian roulette). If `capacity` is smaller than the
 * count: BDPT_ERR_INVALID, *nsplats = the count, `state` unchanged (call again
 * with a larger list).
 * Any rr_depth in [1, 1024]. Synchronous. */
int bdpt_render_sample_mt(bdpt_ctx* ctx, const bdpt_frame_params* params, const float ray[8],
                          uint32_t state[BDPT_MT19937_WORDS], float Li[3], bdpt_splat* splats, int32_t capacity,
                          int32_t* nsplats);
/* The same with the sampler given as std::mt19937(sampler_seed) after
 * *sampler_draws draws (updated on return); splats are added to fb_host
 * (W*H*3 floats) in order. Synchronous. */
int bdpt_render_sample(bdpt_ctx* ctx, const bdpt_frame_params* params, const float ray[8], uint32_t sampler_seed,
                       int32_t* sampler_draws, float Li[3], float* fb_host);
int bdpt_get_stats(bdpt_ctx* ctx, bdpt_stats* out);
/* (new) The frame-kernel build the context's last bdpt_render launched: "bdpt_frame_kernel",
 * "_split" (rrDepth <= 3: no deferred shading step between the subpaths), "_deep" (rrDepth > 28),
 * "_rr" (Russian roulette), "_rrc" (Russian roulette in a scene with glass: a lone subpath trapped by
 * total internal reflection bounces inline) or "_hbm" (BSDF records in HBM); "" before the first render. For
 * matching profiler records to the kernel that ran. */
const char* bdpt_last_kernel(const bdpt_ctx* ctx);
/* Waits for all work queued by this context (on every stream it was given). */
int bdpt_synchronize(bdpt_ctx* ctx);
/* (new) Claim order of the shard's rows for the context's later bdpt_render calls: order[i]
 * is the i-th row claimed (a permutation of the shard's local rows 0..n-1, local row r =
 * image row row_offset + r * row_stride); n = 0 restores top-to-bottom. The reference's
 * offline loop hands rows to its threads in order (parallel_for over rows,
 * renderer.cpp:157, parallelfor.h:25-65); the order changes no sample (each keeps its
 * (pixel, sample) seed) and so no result beyond the float addition order, only which
 * samples run last: a render whose shard has a different row count fails
 * (BDPT_ERR_INVALID). Costly rows first leaves cheap samples in flight when the work runs
 * out, which shortens the persistent grid's end tail (each of N ranks pays it once). */
int bdpt_set_row_order(bdpt_ctx* ctx, const int32_t* order, int32_t n);
/* (new) Per local row of the last BDPT_FLAG_COUNT render's shard, the ray queries its
 * samples issued (a cost estimate for bdpt_set_row_order). Returns BDPT_ERR_INVALID when
 * n differs from that shard's row count. Synchronous. */
int bdpt_get_row_costs(bdpt_ctx* ctx, int64_t* costs, int32_t n);

/* ---- the reference's path tracer on the same substrate (src/integrators/path.h) ---- */
typedef struct {
    int32_t is_explicit;     /* [renderer] isExplicit (default true): renderExplicit / renderImplicit */
    int32_t max_depth;       /* maxDepth (default -1 = Russian roulette past rr_depth) */
    int32_t rr_depth;        /* rrDepth (default 5) */
    float rr_prob;           /* rrProb (default 0.95) */
    int32_t emitter_samples; /* emitterSamples (default 1) */
    int32_t bsdf_samples;    /* bsdfSamples (default 0) */
} bdpt_path_params;
/* Renders every (pixel, sample) of the shard with PathTracerIntegrator::render
 * and ADDS acc/spp per pixel to fb_device (same framebuffer, camera, seeding and
 * shard conventions as bdpt_render; params->rr_depth / strategy are not used).
 * Asynchronous. bdpt_get_stats().counters: [1] samples that outgrew the
 * 512-level recursion stack (then the call's result is not the reference's;
 * bdpt_render_path_host fails with BDPT_ERR_UNSUPPORTED), [2] / [3] samples
 * that drew more than 227 / 624 random numbers; with BDPT_FLAG_COUNT also
 * [0] closest-hit rays and [7] random numbers drawn. */
int bdpt_render_path(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_path_params* path, float* fb_device,
                     void* hip_stream);
int bdpt_render_path_host(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_path_params* path,
                          float* fb_host);
/* One PathTracerIntegrator::render(ray, sampler) call (path.h:235-245) with the
 * caller's sampler state (advanced in place, as bdpt_render_sample_mt). Synchronous. */
int bdpt_render_path_sample_mt(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_path_params* path,
                               const float ray[8], uint32_t state[BDPT_MT19937_WORDS], float Li[3]);
/* The same with the sampler given as std::mt19937(sampler_seed) after
 * *sampler_draws draws, updated on return. */
int bdpt_render_path_sample(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_path_params* path,
                            const float ray[8], uint32_t sampler_seed, int32_t* sampler_draws, float Li[3]);

/* ---- the reference's direct-light integrator (src/integrators/direct.h) ---- */
#define BDPT_DIRECT_AREA 1              /* samplingStrategy "area"             renderArea :143-195 */
#define BDPT_DIRECT_SOLID_ANGLE 2       /* "solidAngle"                        renderSolidAngle :244-311 */
#define BDPT_DIRECT_COSINE_HEMISPHERE 3 /* "cosineHemisphere"                  renderCosineHemisphere :198-233 */
#define BDPT_DIRECT_BSDF 4              /* "bsdf"                              renderBSDF :235-264 */
#define BDPT_DIRECT_MIS 5               /* "mis"                               renderMIS :313-447 */
typedef struct {
    int32_t sampling_strategy; /* BDPT_DIRECT_*; 0 = an unknown samplingStrategy string (rejected) */
    int32_t emitter_samples;   /* [renderer] emitterSamples (default 1) */
    int32_t bsdf_samples;      /* bsdfSamples (default 1) */
} bdpt_direct_params;
/* Renders every (pixel, sample) of the shard with DirectIntegrator::render and ADDS
 * acc/spp per pixel to fb_device (conventions of bdpt_render_path). Emitters are the
 * spheres the reference makes of them (center = the shape's vertex mean, radius =
 * AABB max.x - center.x, renderer.cpp:295-304 / :349-358). An unknown strategy fails
 * with BDPT_ERR_INVALID (the reference prints "Error: wrong strategy" and exits,
 * direct.h:460-461). Asynchronous. */
int bdpt_render_direct(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_direct_params* direct,
                       float* fb_device, void* hip_stream);
int bdpt_render_direct_host(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_direct_params* direct,
                            float* fb_host);
/* One DirectIntegrator::render(ray, sampler) call (direct.h:449-462), as
 * bdpt_render_path_sample_mt / bdpt_render_path_sample. */
int bdpt_render_direct_sample_mt(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_direct_params* direct,
                                 const float ray[8], uint32_t state[BDPT_MT19937_WORDS], float Li[3]);
int bdpt_render_direct_sample(bdpt_ctx* ctx, const bdpt_frame_params* params, const bdpt_direct_params* direct,
                              const float ray[8], uint32_t sampler_seed, int32_t* sampler_draws, float Li[3]);
/* samplingStrategy string -> BDPT_DIRECT_* (0 when unknown). */
int32_t bdpt_direct_strategy(const char* name);

/* ---- several HIP devices in one process ---- */
/* The reference fans the offline loop out over host threads (parallel_for,
 * src/core/parallelfor.h:25-65, renderer.cpp:157); here every device gets one
 * context, one stream and one full-frame buffer. Device i renders the
 * interleaved row shard i, i + N, ... of the image; one RCCL sum-reduce
 * (ncclReduce over communicators from ncclCommInitAll, librccl loaded at first
 * use) brings the frames to devices[0]. A device list naming one device more than
 * once (a single-GPU rehearsal) sums on that device without RCCL. */
#define BDPT_MAX_DEVICES 16
typedef struct bdpt_multi bdpt_multi;
typedef struct {
    int32_t devices;   /* N */
    int32_t rccl;      /* 1: the reduce ran over RCCL */
    double wall_ms;    /* host wall time of the last bdpt_multi_render_host */
    double render_ms;  /* root-device events: start .. every device's render done */
    double reduce_ms;  /* root-device events: the reduce */
    int64_t samples;   /* camera samples over all devices */
    double kernel_ms[BDPT_MAX_DEVICES];      /* per device, HIP events of its render kernel */
    int64_t device_samples[BDPT_MAX_DEVICES];
    int64_t capped_samples;  /* Russian roulette: bdpt_stats.capped_samples summed over the devices; a
                                non-zero sum fails bdpt_multi_render_host as it fails bdpt_render_host */
    int64_t schedule_errors; /* bdpt_stats.schedule_errors summed over the devices; a non-zero sum fails
                                bdpt_multi_render_host (BDPT_ERR_HIP) as it fails bdpt_render_host */
} bdpt_multi_stats;
int bdpt_multi_create(const bdpt_scene* scene, int32_t ndevices, const int32_t* devices, bdpt_multi** out);
int bdpt_multi_destroy(bdpt_multi* multi);
/* The whole image (params->row_offset 0, row_stride 1) over all devices; the frame
 * is ADDED to fb_host (W*H*3 floats) as bdpt_render_host does. path / direct:
 * NULL for BDPT, else the PathTracerIntegrator / DirectIntegrator settings (at most
 * one). Synchronous. */
int bdpt_multi_render_host(bdpt_multi* multi, const bdpt_frame_params* params, const bdpt_path_params* path,
                           const bdpt_direct_params* direct, float* fb_host);
int bdpt_multi_get_stats(bdpt_multi* multi, bdpt_multi_stats* out);

/* ---- the BSDF plugin contract and the path's building blocks, batched on the device ---- */
/* All arrays are host arrays of n elements; directions are in the local shading
 * frame (z = the shading normal) as SurfaceInteraction::wo / wi. Synchronous. */
/* BSDF::eval(i) of material mat[k]: f * cos(wi) (core.h:308). f: n x 3. */
int bdpt_bsdf_eval(bdpt_ctx* ctx, int64_t n, const int32_t* mat, const float* wo, const float* wi, float* f);
/* BSDF::pdf(i): the solid-angle pdf of wi (core.h:309). */
int bdpt_bsdf_pdf(bdpt_ctx* ctx, int64_t n, const int32_t* mat, const float* wo, const float* wi, float* pdf);
/* BSDF::sample(i, u, &pdf) (core.h:310): u = n x 2 samples in [0, 1); returns f * cos
 * (f: n x 3), the sampled wi (n x 3) and *pdf. */
int bdpt_bsdf_sample(bdpt_ctx* ctx, int64_t n, const int32_t* mat, const float* wo, const float* u, float* f,
                     float* wi, float* pdf);
/* BSDF::getType() (core.h:311) of a scene material, and this build's kind
 * (1 diffuse, 2 mirror, 3 glass, 4 mixture, 5 phong, 0 the null BSDF of illum 5). */
int bdpt_bsdf_type(const bdpt_scene* scene, int32_t mat, uint32_t* type, int32_t* kind);

/* A closest hit as AcceleratorBVH::intersect fills SurfaceInteraction (accel.h:125-172). */
typedef struct {
    int32_t hit;               /* closest hit accepted (min_t <= t <= max_t) / occluded */
    float t, u, v;             /* t is the search result even when not accepted (accel.h:132) */
    int32_t shape_id, prim_id, mat_id;
    float p[3], ns[3], ng[3];  /* hit point, frameNs.n, frameNg.n */
    float wo[3];               /* frameNs.toLocal(-ray.d) */
    int32_t tri;               /* this build's triangle index (reference BVH leaf order) */
} bdpt_hit;
/* rays: n x 8 (o.xyz d.xyz min_t max_t). occlusion = 0: closest hit (accel.h:125);
 * 1: the any-hit query of visibilityQuery (bvh.h:259-352 with occlusion = true),
 * result in hit only. The traversal is the frame kernels' (culled 4-wide tree,
 * reference-leaf check; origins beyond 100 scene diagonals walk the reference's
 * tree unculled), with the interior-box test a frame would use for the batch's
 * origins: without the ambiguity slack when all lie within 100 scene diagonals
 * and, like the scene box, within 300 diagonals of 0 (the slack-free test's
 * fma planes), with it otherwise. */
int bdpt_intersect(bdpt_ctx* ctx, int64_t n, const float* rays, int32_t occlusion, bdpt_hit* out);
/* The same with the frame kernels' near-cull rule: origin_normals (n x 3) is the
 * normal of the surface each ray leaves (a path vertex's interpolated shading
 * normal, the emitter point's normal), zero for a camera origin; origin_tris
 * (n, may be NULL = all -1) the triangle that surface is (bdpt_hit.tri order),
 * -1 for none. bdpt_intersect (origin_normals NULL) culls no box for lying close
 * to the origin; the frames skip such boxes unless the query leaves its surface
 * at |cos| < 0.02 to the triangle's geometric plane, tested as |dot(d, n_s)| <
 * 0.02 + the triangle's normal-cone margin. */
int bdpt_intersect_from(bdpt_ctx* ctx, int64_t n, const float* rays, const float* origin_normals,
                        const int32_t* origin_tris, int32_t occlusion, bdpt_hit* out);
/* BDPTIntegrator::splatToImagePlane (bdpt.h:485-496) of points p (n x 3) for the
 * camera and image of params: xy = n x 2 (the reference's int truncation). */
int bdpt_splat_to_image_plane(bdpt_ctx* ctx, const bdpt_frame_params* params, int64_t n, const float* p,
                              int32_t* xy);

/* ---- diagnostics ---- */
/* GlassBSDF::FresnelDielectric (glass.h:40-53): in = n x (eta_i, eta_t, cos_i, cos_t). */
int bdpt_debug_fresnel(int32_t device, int64_t n, const float* in, float* out);
/* rayTriangleIntersect (core.h:379-400): rays n x 8, verts n x 9 (v0 v1 v2);
 * out = n x (hit, t, u, v). */
int bdpt_debug_triangle(int32_t device, int64_t n, const float* rays, const float* verts, float* out);
/* The device restatements of glibc's transcendental functions the path uses
 * (std::sinf / cosf / powf in src/core/math.h:125-242, mixture.h:70), element-wise
 * on device `device`: fn 0 sinf(x), 1 cosf(x), 2 powf(x, y), 3 / 4 the sin / cos
 * of the fused sincos the warps call. Host arrays of n floats; synchronous. */
int bdpt_debug_math(int32_t device, int32_t fn, const float* x, const float* y, float* out, int64_t n);

/* ---- scene configuration and image output (host only, no GPU needed) ---- */

/* The settings loadTOML (src/main.cpp:22-116) reads from a scene .toml, with its
 * defaults and cpptoml's typed-read rules. obj_file is resolved against the
 * TOML's directory as Scene::load does (renderer.cpp:236-241). */
typedef struct {
    char toml_file[4096];
    char obj_file_raw[4096]; /* [input] objfile as written */
    char obj_file[4096];     /* resolved path */
    bdpt_camera camera;      /* [camera] eye / at / up / fov (defaults 1,1,0 / 0,0,0 / 0,1,0 / 30) */
    int32_t width, height;   /* [film] (defaults 768 x 576) */
    int32_t realtime;        /* [renderer] realtime (default false) */
    char integrator[32];     /* [renderer] type (default "normal") */
    int32_t rr_depth;        /* [renderer] rrDepth (bdpt/path, default 5) */
    float rr_prob;           /* [renderer] rrProb (bdpt default 0; unused: NO_RR, bdpt.h:18) */
    int32_t spp;             /* [renderer] spp (default 1) */
    bdpt_path_params path;   /* type = "path": isExplicit, maxDepth, rrDepth, rrProb, emitterSamples,
                                bsdfSamples (main.cpp:96-101); defaults otherwise */
    bdpt_direct_params direct;       /* type = "direct": emitterSamples, bsdfSamples (main.cpp:88-92) */
    char sampling_strategy[32];      /* type = "direct": samplingStrategy as written (default "emitter") */
} bdpt_config;

/* loadTOML (main.cpp:22-116). BDPT_ERR_INVALID with the parse error otherwise. */
int bdpt_config_load_toml(const char* toml_path, bdpt_config* out);
/* Integrator::save -> saveEXR (integrator.cpp:26-30, utils.h:95-156): the
 * W*H*3 float framebuffer (pixel-major RGB, row 0 = top) as an uncompressed
 * scanline OpenEXR with half-float channels B, G, R — byte-identical to the
 * reference's tinyexr output. bdpt_encode_exr writes into `out` (capacity
 * bytes; out = NULL only reports *size). */
int bdpt_encode_exr(const float* rgb, int32_t width, int32_t height, unsigned char* out, int64_t capacity,
                    int64_t* size);
int bdpt_save_exr(const float* rgb, int32_t width, int32_t height, const char* path);

#ifdef __cplusplus
}
#endif
#endif
