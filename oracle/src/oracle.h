/* TEST INFRASTRUCTURE ONLY — the CPU oracle for the BDPT hot path.
 *
 * A plain-C restatement of the reference's algorithm
 * (JackMinn/Bidirectional-Path-Tracing: src/integrators/bdpt.h and the BSDFs,
 * BVH traversal, sampler, warps and scene ingest it calls). Each function in
 * each oracle/src C file cites the reference file:line it restates.
 *
 * Who may use it: tests/ (as the checker), __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg. The product library under
 * bidirectional-path-tracing_amd/ never includes, links or calls this code.
 *
 * Parity is pinned by tests/golden/ (framebuffers rendered by the unmodified
 * reference compiled by oracle/ref/Makefile) — see tests/test_oracle_golden.py.
 */
#ifndef TR_ORACLE_H
#define TR_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tro_scene tro_scene;

typedef struct {
    float eye[3], at[3], up[3], fov;
    int width, height, spp, rr_depth;
    int strategy; /* 0 BDPT, 1 LIGHT_TRACING, 2 PATH_TRACING (the reference's compile-time
                     switches, bdpt.h:16-17, as a run-time parameter) */
    /* integrator: 0 BDPTIntegrator (bdpt.h), 1 PathTracerIntegrator (path.h)
     * with the [renderer] settings of main.cpp:96-101 */
    int integrator;
    int pt_explicit, pt_max_depth, pt_rr_depth;
    float pt_rr_prob;
    int pt_emitter_samples, pt_bsdf_samples;
    /* integrator 2: DirectIntegrator (direct.h), samplingStrategy 1 area, 2 solidAngle,
     * 3 cosineHemisphere, 4 bsdf, 5 mis (main.cpp:88-92) */
    int di_strategy, di_emitter_samples, di_bsdf_samples;
    /* per-(pixel, sample) seeds are seed_base + pixel*spp + k; the reference's
     * Sampler seed 260450963 (renderer.cpp:155) unless a test varies it */
    uint32_t seed_base;
    /* 0: NO_RR = 1 (bdpt.h:18, the reference as shipped); 1: its NO_RR = 0 branch
     * (Russian roulette past rrDepth, bdpt.h:68, :129-132, :188, :201-204) */
    int russian_roulette;
} tro_params;

/* Loads an OBJ (+ MTL) exactly as Scene::load does (reference
 * src/core/renderer.cpp:235-315): tinyobj v1.2.0 parse + ear-clip
 * triangulation, BSDF per illum, emitters with face-area CDFs, Fast-BVH build.
 * Returns NULL on error (message via tro_last_error). */
tro_scene* tro_scene_load(const char* obj_path);
void tro_scene_free(tro_scene* s);
const char* tro_last_error(void);

/* Scene statistics: out[0]=triangles, out[1]=BVH nodes, out[2]=shapes,
 * out[3]=materials, out[4]=emitters, out[5]=max BVH depth. */
void tro_scene_stats(const tro_scene* s, int64_t out[6]);

/* Dumps in the same layouts as oracle/ref/ref_driver.cpp `dump`:
 * tri_f32 [ntri][18] (v0 v1 v2 n0 n1 n2, BVH leaf order), tri_i32 [ntri][3]
 * (shapeID, primID, matID), node_f32 [nnodes][6], node_u32 [nnodes][3]. */
void tro_scene_dump(const tro_scene* s, float* tri_f32, int32_t* tri_i32, float* node_f32, uint32_t* node_u32);

/* Camera constants as renderer.cpp:140-153 / bdpt.h:49-54 compute them:
 * 4 column-major mat4 (worldToCamera, cameraToWorld, cameraToClip,
 * NDCToScreen) then invWidth, invHeight, angle, aspect, fwd.xyz, vnear. */
void tro_camera(const tro_params* p, float out[72]);

/* Renders rows [row_begin, row_end) (stride row_stride) with the
 * deterministic per-(pixel, sample) seeding of SURVEY.md §8(c) and ADDS into
 * fb (W*H*3 floats): eye estimates acc*(1/spp) per pixel plus every camera
 * splat. Single-threaded. Returns the number of camera samples rendered. */
int64_t tro_render(const tro_scene* s, const tro_params* p, float* fb, int row_begin, int row_end, int row_stride);

/* One (pixel, k) camera sample: Li (3 floats) and its splats into fb. */
void tro_sample(const tro_scene* s, const tro_params* p, int pixel, int k, float Li[3], float* fb);

/* Work counters accumulated by tro_render on this thread (for the algorithmic
 * byte model of SURVEY.md §8(d)): [0] closest-hit rays, [1] shadow rays,
 * [2] interior-node visits, [3] triangle tests, [4] light vertices stored,
 * [5] light-vertex reads in connections, [6] splats, [7] RNG draws. */
#define TRO_NUM_COUNTERS 9
void tro_counters(int64_t out[TRO_NUM_COUNTERS], int reset);

/* Light vertices dropped because a subpath outgrew the oracle's 1024-vertex
 * store (Russian roulette only; always 0 in practice). */
int64_t tro_rr_overflow(int reset);
/* Deepest light / eye subpath (depth when its walk ended) and most stored light
 * vertices of one sample since the last reset, on this thread. */
void tro_walk_stats(int64_t out[3], int reset);

/* Unit-level hooks for KAT tests. */
uint32_t tro_mt19937_nth(uint32_t seed, int n);   /* n-th raw output */
float tro_sampler_nth(uint32_t seed, int n);      /* n-th Sampler::next() */
float tro_sinf(float x);
float tro_cosf(float x);
float tro_powf(float x, float y);

#ifdef __cplusplus
}
#endif
#endif
