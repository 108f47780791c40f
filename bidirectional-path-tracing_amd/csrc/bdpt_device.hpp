// Device-side BDPT building blocks: sampler, warps, frames, BVH traversal,
// BSDFs and the vertex connections. Each function cites the reference code
// (JackMinn/Bidirectional-Path-Tracing) whose arithmetic it reproduces.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bdpt_types.h"
#include "device_math.hpp"

namespace bdpt {
namespace dev {

constexpr float kPi = 3.14159265358979323846f;        // platform.h:50 (float M_PI)
constexpr float kInvPi = 0.31830988618379067154f;     // platform.h:51
constexpr float kInvTwoPi = 0.15915494309189533577f;  // platform.h:52
constexpr float kEpsilon = 1e-8f;                     // platform.h:56
constexpr float kTriMinT = 0x1.0624dep-10f;           // smallest float t with (double)t > 1e-3 (accel.h:43)
constexpr int kCounters = 32;
#ifndef BDPT_HELP_CLOCKS
#define BDPT_HELP_CLOCKS 0  // (bdpt_kernels.hip) the stack-depth probe words carry other clocks
#endif

#ifndef BDPT_TRAV_WHILE_WHILE
#define BDPT_TRAV_WHILE_WHILE 1  // megakernel traversal loop shape (0: one node or leaf per iteration)
#endif

// ------------------------------------------------------------------ inputs
// Loads through an address-space-1 pointer compile to global_load (SGPR/VGPR
// addressing, vmcnt only) instead of flat_load: the scene pointers arrive via
// a parameter block, so the compiler cannot infer their address space itself.
typedef float v4f_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 gld4(const float4* p) {
    const v4f_t v = *(const __attribute__((address_space(1))) v4f_t*)(p);
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float gld1(const float* p) { return *(const __attribute__((address_space(1))) float*)(p); }
__device__ __forceinline__ void gst1(float* p, float x) { *(__attribute__((address_space(1))) float*)(p) = x; }
__device__ __forceinline__ void gst4(float4* p, float4 x) {
    *(__attribute__((address_space(1))) v4f_t*)(p) = v4f_t{x.x, x.y, x.z, x.w};
}

struct DevScene {
    const float4* __restrict__ tri;
    const float4* __restrict__ shade;
    const float4* __restrict__ nodes;   // the reference's binary tree (2 child boxes per record)
    const float4* __restrict__ wnodes;  // 4-wide traversal nodes (wide_bvh.hpp)
    const float4* __restrict__ qnodes;  // the same nodes compressed to 64 B (quantize_wide_nodes), or null
    const float4* __restrict__ wtri;    // traversal triangles, that tree's leaf order (v0|ref index, e1|ref leaf, e2)
    const float4* __restrict__ lbox;    // exact box of every reference leaf (lo, hi)
    const BsdfRecord* __restrict__ bsdf;
    const EmitterRecord* __restrict__ emit;
    const float4* __restrict__ emit_tri;
    const float* __restrict__ emit_cdf;
    const int32_t* __restrict__ shape_emitter;
    uint32_t root_link, wroot_link;
    // 1: the interior boxes of the traversal tree are tested with slab_fast's
    // ambiguity slack; 0 (host decision per render, node_slack_needed in
    // bdpt_capi.cpp): the padded boxes make a plain tn <= tf conservative
    uint32_t node_slack;
    int32_t nemit, nbsdf, nshapes;
    float inv_nemit;  // 1 / nemit (the host's IEEE division): selectEmitter's pdf (core.h emitter selection)
    // LDS copy of the small tables (scene_tables_to_lds): word offsets of the
    // emitter records and the shape->emitter map, total words (16-byte rounded)
    uint32_t lds_emit_off, lds_shape_off, lds_words;
    uint32_t lds_bsdf_off;  // kLdsHdr, or kNoLds: the BSDF records stay in HBM (too many materials)
    // emitter faces (5 float4 each) and CDFs, also in LDS when they fit without
    // costing a resident block (host decision); kNoLds otherwise
    uint32_t lds_etri_off, lds_ecdf_off;
    int32_t n_etri, n_ecdf;
    // MT19937 continuation ring of the megakernel's lanes (rrDepth > 28, Russian
    // roulette): word k of lane slot s at mt_ring[s * kMtRingSlotWords + k] (one 2.5 KB block per
    // slot: a lane's draws touch one page, not 624 pages a slot-count stride apart —
    // a Russian-roulette subpath trapped in glass draws millions of them alone);
    // mt_ring_stride is the word stride within a block (1); null otherwise
    uint32_t* mt_ring;
    uint32_t mt_ring_stride;
    // The scene box grown by 100 scene diagonals: a query whose origin lies
    // outside (far_origin) walks the reference's own binary tree unculled. Far
    // from the scene Moller-Trumbore's arithmetic loses the hit point (cancellation
    // in o - v0), so the reference can accept a triangle the ray's line misses by
    // more than the traversal tree's padding.
    float near_lo[3], near_hi[3];
    uint32_t q_ok;  // qnodes present: the BDPT_QNODES kernels walk the 4-wide tree (else the binary one)
    uint32_t gdepth;  // traversal-stack overflow entries per lane slot (beyond the LDS ones)
};
constexpr uint32_t kNoLds = 0xffffffffu;
constexpr uint32_t kLdsHdr = 4;  // LDS header words: mt_ring (2 words), mt_ring_stride, the block's first lane slot

// Small per-scene tables — BSDF records, emitter records, shape -> emitter
// map — live in the kernels' dynamic LDS: the divergent shading code reads
// them with ds_read instead of chains of dependent global loads. Layout (words):
// [0, kLdsHdr) header, [kLdsHdr, emit_off) BsdfRecord[nbsdf], [emit_off, shape_off) EmitterRecord[nemit],
// [shape_off, ...) int32 shape_emitter[nshapes] (unless kNoLds); anything a kernel keeps in
// dynamic LDS besides goes at lds_words.
extern __shared__ uint32_t g_scene_lds[];
// Where the BSDF records are read: 0 = the LDS table only (the frame kernels'
// default build), 1 = HBM only (bdpt_kernels_hbm.hip: scenes whose records do not
// fit the LDS budget), 2 = chosen per launch by sc.lds_bsdf_off (the single-
// sample and per-function kernels: a generic pointer, flat loads — measured 8 %
// slower in the frame kernel, irrelevant for one wave).
#ifndef BDPT_BSDF_TABLE
#define BDPT_BSDF_TABLE 2
#endif
__device__ __forceinline__ const BsdfRecord& bsdf_of(const DevScene& sc, int m) {
#if BDPT_BSDF_TABLE == 1
    return sc.bsdf[m];
#else
#if BDPT_BSDF_TABLE == 2
    if (sc.lds_bsdf_off == kNoLds) return sc.bsdf[m];
#endif
    return reinterpret_cast<const BsdfRecord*>(g_scene_lds + kLdsHdr)[m];
#endif
}
__device__ __forceinline__ const EmitterRecord& emitter_of(const DevScene& sc, int i) {
    return reinterpret_cast<const EmitterRecord*>(g_scene_lds + sc.lds_emit_off)[i];
}
// The shape -> emitter map stays in global memory when a scene has too many
// shapes for the LDS budget (lds_shape_off == kNoLds; read on emitter hits only).
__device__ __forceinline__ int shape_emitter_of(const DevScene& sc, int shape) {
    if (sc.lds_shape_off == kNoLds) return *(const __attribute__((address_space(1))) int32_t*)(sc.shape_emitter + shape);
    return static_cast<int>(g_scene_lds[sc.lds_shape_off + shape]);
}
// Cooperative copy by the whole block, then a barrier.
__device__ __forceinline__ void scene_tables_to_lds(const DevScene& sc) {
    const uint32_t nb = static_cast<uint32_t>(sc.nbsdf) * (sizeof(BsdfRecord) / 4);
    const uint32_t ne = static_cast<uint32_t>(sc.nemit) * (sizeof(EmitterRecord) / 4);
    const uint32_t* b = reinterpret_cast<const uint32_t*>(sc.bsdf);
    const uint32_t* e = reinterpret_cast<const uint32_t*>(sc.emit);
    const uint32_t* m = reinterpret_cast<const uint32_t*>(sc.shape_emitter);
    if (threadIdx.x == 0) {
        const uint64_t ring = reinterpret_cast<uint64_t>(sc.mt_ring);
        g_scene_lds[0] = static_cast<uint32_t>(ring);
        g_scene_lds[1] = static_cast<uint32_t>(ring >> 32);
        g_scene_lds[2] = sc.mt_ring_stride;
        g_scene_lds[3] = blockIdx.x * blockDim.x;  // the block's first lane slot (mt_ring_slot)
    }
    if (sc.lds_bsdf_off != kNoLds)
        for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) g_scene_lds[kLdsHdr + i] = b[i];
    for (uint32_t i = threadIdx.x; i < ne; i += blockDim.x) g_scene_lds[sc.lds_emit_off + i] = e[i];
    if (sc.lds_shape_off != kNoLds)
        for (uint32_t i = threadIdx.x; i < static_cast<uint32_t>(sc.nshapes); i += blockDim.x)
            g_scene_lds[sc.lds_shape_off + i] = m[i];
    if (sc.lds_etri_off != kNoLds) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(sc.emit_tri);
        const uint32_t* c = reinterpret_cast<const uint32_t*>(sc.emit_cdf);
        for (uint32_t i = threadIdx.x; i < 20u * static_cast<uint32_t>(sc.n_etri); i += blockDim.x)
            g_scene_lds[sc.lds_etri_off + i] = t[i];
        for (uint32_t i = threadIdx.x; i < static_cast<uint32_t>(sc.n_ecdf); i += blockDim.x)
            g_scene_lds[sc.lds_ecdf_off + i] = c[i];
    }
    __syncthreads();
}

struct DevFrame {
    CameraConstants cam;
    float cam_o[3];
    int32_t W, H, spp, rr_depth, strategy;
    uint32_t seed_base;
    int32_t row_offset, row_stride, nrows;
    uint32_t flags;
    uint64_t total_samples;  // nrows * W * spp
    int32_t rr_mode;    // 1: NO_RR = 0 (Russian roulette past rr_depth; the bdpt_kernels_rr.hip build)
    int32_t depth_cap;  // subpath depth bound: rr_depth under NO_RR; with RR a guard (2^25 bounces)
    int32_t lv_max;     // light vertices a lane slot stores: rr_depth - 1 under NO_RR, more with RR
    uint32_t* capped;   // RR: samples that hit depth_cap or lv_max (the frame is then not the reference's)
    // frame-kernel timeline (s_memrealtime ticks): [0] first wave start (min), [1]
    // the claim of the last 64-sample chunk, [2] last wave exit (max) — the end
    // tail a row shard pays is [2] - [1] (kDiag*)
    unsigned long long* diag;
    // 1 / spp and 1 / (W * H) as the host's IEEE divisions, the bits the device's correctly
    // rounded reciprocal (rcp_cr) and division give: per-frame constants the shading bodies
    // would otherwise recompute (~10 instructions each) per splat and per sample
    float inv_spp, inv_pixels;
    // Russian-roulette continuation pass (bdpt_kernels.hip): per lane slot a
    // kParkWords record, then the list of parked slots ([0] count); null: off.
    // park_flags: kParkOn (park walks deeper than park_depth), kParkResume (this
    // launch resumes the records the chain kernel returned instead of claiming)
    uint32_t* park;
    int32_t park_depth;
    uint32_t park_flags;
    // lanes with a finished query that trigger a wave's shading step (the frame
    // kernels; chosen per render by the host: 0 = the build's BDPT_SHADE_READY)
    int32_t shade_ready;
    // Russian-roulette build: a subpath deeper than express_depth bounces puts its
    // wave in express mode (bdpt_kernels.hip); sched_flags kSchedNoCoopGroups walks
    // express waves' 2-4 long walks in turn instead of in lane groups. Schedule
    // only: the same per-sample arithmetic either way (tests/test_gpu_express.py).
    int32_t express_depth;
    uint32_t sched_flags;
    // Shadow-ray task rings of the BDPT_HELP build (bdpt_path.hpp task_push): per
    // wave task_cap records of 48 bytes (3 float4), wave w's at tasks + 3 * task_cap * w
    float4* tasks;
    uint32_t task_cap;
    // the shard's row claim order (bdpt_set_row_order; null: top to bottom) and, in a
    // counting pass, the queries issued per local row (null otherwise)
    const int32_t* row_order;
    unsigned long long* row_cost;
};
enum : uint32_t { kParkOn = 1u, kParkResume = 2u };
enum : uint32_t { kSchedNoCoopGroups = 1u };

struct Ray {
    f3 o, d;
    float min_t, max_t;
};

// Hit record = the parts of SurfaceInteraction (core.h:173-180) the path reads.
struct Hit {
    f3 p, wo;
    f3 n;  // frameNs.n; s and t are recomputed from it (Frame(n) is a pure function of n)
    float dist;
    int mat, shape;
};

// ------------------------------------------------------------------ sampler
// std::mt19937(seed) + uniform_real_distribution<float> (math.h:63-76). A BDPT
// sample draws at most 10 + 8 (rrDepth - 1) numbers (< 227 for rrDepth <= 28),
// all from the first twist, so output n is computed lazily from the seeding
// recurrence: out_n = temper(x[n+397] ^ twist(x[n], x[n+1])). State: x[n],
// x[n+1], x[n+397] and n. Draws past 226 continue from a per-lane ring of 624
// untempered outputs in HBM (mt_ring_step), which only deeper rrDepth needs.
struct LazyMT {
    uint32_t a0, a1, b, n;
};

__device__ __forceinline__ uint32_t mt_init_step(uint32_t x, uint32_t i) { return 1812433253u * (x ^ (x >> 30)) + i; }

// x[397] of the seeding recurrence: the 397 dependent steps (each with a
// quarter-rate 32-bit multiply) that dominate seeding.
__device__ __forceinline__ uint32_t mt_x397(uint32_t seed) {
    uint32_t x = seed;
#pragma unroll 4
    for (uint32_t i = 1; i <= 397; i++) x = mt_init_step(x, i);
    return x;
}
// Seeds from a precomputed x[397] (mt_x397(seed)).
__device__ __forceinline__ void mt_seed_with(LazyMT& r, uint32_t seed, uint32_t x397) {
    r.a0 = seed;
    r.a1 = mt_init_step(seed, 1);
    r.b = x397;
    r.n = 0;
}
__device__ __forceinline__ void mt_seed(LazyMT& r, uint32_t seed) { mt_seed_with(r, seed, mt_x397(seed)); }

// Positions the generator after `skip` draws (for Sampler objects that were
// already advanced, e.g. by the camera jitter of the driver).
__device__ __forceinline__ void mt_seed_skip(LazyMT& r, uint32_t seed, uint32_t skip) {
    uint32_t x = seed, i = 0;
    for (; i < skip; i++) x = mt_init_step(x, i + 1);
    r.a0 = x;
    x = mt_init_step(x, ++i);
    r.a1 = x;
    for (; i < skip + 397; i++) x = mt_init_step(x, i + 1);
    r.b = x;
    r.n = skip;
}

__device__ __forceinline__ uint32_t mt_next_u32(LazyMT& r) {
    uint32_t y = (r.a0 & 0x80000000u) | (r.a1 & 0x7fffffffu);
    uint32_t v = r.b ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    r.a0 = r.a1;
    r.a1 = mt_init_step(r.a1, r.n + 2);
    r.b = mt_init_step(r.b, r.n + 398);
    r.n++;
    v ^= (v >> 11);
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= (v >> 18);
    return v;
}

__device__ __forceinline__ uint32_t mt_temper(uint32_t v) {
    v ^= (v >> 11);
    v ^= (v << 7) & 0x9d2c5680u;
    v ^= (v << 15) & 0xefc60000u;
    v ^= (v >> 18);
    return v;
}
__device__ __forceinline__ uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t c) {  // c ^ twist(a, b)
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return c ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// Output n >= 227 of std::mt19937(seed): u[n] = u[n-227] ^ twist(u[n-624],
// u[n-623]) (with the seeding values x[n], x[n+1] while n + 1 < 624), kept in a
// 624-word ring (word k at ring[k * st]). The first call materialises outputs
// 0..226 (the seed is needed then only).
__device__ __forceinline__ uint32_t mt_ring_step(LazyMT& m, uint32_t seed, uint32_t* ring, uint32_t st) {
    const uint32_t n = m.n;
    if (n == 227) {
        LazyMT t;
        t.a0 = seed;
        t.a1 = mt_init_step(seed, 1);
        t.b = seed;
        for (uint32_t i = 1; i <= 397; i++) t.b = mt_init_step(t.b, i);
        for (uint32_t k = 0; k < 227; k++) {
            ring[k * st] = mt_twist(t.a0, t.a1, t.b);
            t.a0 = t.a1;
            t.a1 = mt_init_step(t.a1, k + 2);
            t.b = mt_init_step(t.b, k + 398);
        }
    }
    uint32_t un, un1;
    if (n < 623) un = m.a0, un1 = m.a1;
    else if (n == 623) un = m.a0, un1 = ring[0];
    else un = ring[((n - 624) % 624) * st], un1 = ring[((n - 623) % 624) * st];
    const uint32_t v = mt_twist(un, un1, ring[((n - 227) % 624) * st]);
    ring[(n % 624) * st] = v;
    if (n + 2 <= 623) {
        m.a0 = m.a1;
        m.a1 = mt_init_step(m.a1, n + 2);
    } else if (n + 1 <= 623) {
        m.a0 = m.a1;
    }
    m.n = n + 1;
    return mt_temper(v);
}

#ifndef BDPT_SAMPLER_STATE
#define BDPT_SAMPLER_STATE 0  // 1: the single-sample build (sample_state.hip): draws from a caller's std::mt19937
#endif
#if BDPT_SAMPLER_STATE
// The single-sample entry points (Integrator::render(const Ray&, Sampler&),
// integrator.h:31) take the caller's whole std::mt19937 (Sampler::g, math.h:63-76):
// libstdc++'s _M_x[624] then _M_p, in the order its operator<< writes them. It is
// advanced exactly as mersenne_twister_engine::operator() does (random.tcc:
// _M_gen_rand when _M_p reaches 624, then tempering). One lane uses it; the
// state lives in global memory, its address in LDS header words 0-1.
__device__ BDPT_NOINLINE uint32_t mt_state_u32() {
    const uint64_t base = (static_cast<uint64_t>(g_scene_lds[1]) << 32) | g_scene_lds[0];
    uint32_t* const x = reinterpret_cast<uint32_t*>(base);
    uint32_t p = x[624];
    if (p >= 624u) {
        for (int k = 0; k < 227; k++) x[k] = mt_twist(x[k], x[k + 1], x[k + 397]);
        for (int k = 227; k < 623; k++) x[k] = mt_twist(x[k], x[k + 1], x[k - 227]);
        x[623] = mt_twist(x[623], x[0], x[396]);
        p = 0;
    }
    x[624] = p + 1;
    return mt_temper(x[p]);
}
#endif

// x[0] (the seed) from x[i]: the seeding step x -> 1812433253 (x ^ x >> 30) + i
// is a bijection (odd multiplier; a 30-bit xorshift undoes itself).
__device__ __forceinline__ uint32_t mt_seed_from(uint32_t x, uint32_t i) {
    constexpr uint32_t kInv = 0x9638806du;  // 1812433253^-1 mod 2^32
    for (; i >= 1; i--) {
        x = (x - i) * kInv;
        x ^= x >> 30;
    }
    return x;
}

#ifndef BDPT_DEEP_RNG
#define BDPT_DEEP_RNG 0  // 1: the deep-path build of the megakernel (bdpt_kernels_deep.hip)
#endif
#if BDPT_DEEP_RNG
// BDPT draw n >= 227 (rrDepth > 28: the deep build of the megakernel; the
// host refuses such depths elsewhere). The ring of this lane slot is found
// through the LDS header. Only this build carries the branch and the call at
// every draw site: in the default build they cost ~30 % of the throughput.
#ifndef BDPT_RING_AHEAD
#define BDPT_RING_AHEAD 32  // draws generated ahead into the ring at one call site per shading step (0: per draw)
#endif
#if BDPT_RING_AHEAD
// The ring, generated ahead: outputs n >= 227 are produced by mt_ring_ahead,
// called once per shading step (before the sweep) for lanes within
// BDPT_RING_AHEAD draws of the ring, so every draw site reads
// ring[n mod 624] (one load, no call: an out-of-line call at each of the ~20
// draw sites made the caller keep its live registers in scratch). A sweep draws
// far fewer than BDPT_RING_AHEAD numbers (the action DAG's draw sites sum to
// < 20). Per lane slot kMtRingWords words: the 624-word ring, then the
// generator's cursor (x[g], x[g+1] of the seeding sequence while g < 623, g,
// the seed whose outputs the ring holds, and that seed's x[227] — the value a
// lane's LazyMT::a0 keeps from draw 227 on, so a lane past 227 checks on every
// call that the ring is its own).
constexpr uint32_t kMtRingWords = kMtRingSlotWords;
// The lane's slot: header word 3 (the block's first slot; the Russian-roulette
// chain kernel stores the slot of the sample it continues there) + threadIdx.x.
__device__ __forceinline__ uint32_t* mt_ring_slot() {
    const uint64_t base = (static_cast<uint64_t>(g_scene_lds[1]) << 32) | g_scene_lds[0];
    return reinterpret_cast<uint32_t*>(base) + static_cast<size_t>(g_scene_lds[3] + threadIdx.x) * kMtRingWords;
}
// Generates outputs up to r.n + BDPT_RING_AHEAD - 1; false if the lane had
// already drawn past what was generated (a schedule error: the caller reports it).
__device__ BDPT_NOINLINE bool mt_ring_ahead(const LazyMT& r) {
    uint32_t* const ring = mt_ring_slot();
    uint32_t xa0 = ring[624], xa1 = ring[625], g = ring[626];
    const uint32_t want = r.n + BDPT_RING_AHEAD;
    bool moved = false;  // the cursor changed: store it
    if (r.n < 227) {  // (x[n], x[n+1], x[n+397]) still in registers: the seed is recoverable
        const uint32_t seed = mt_seed_from(r.a0, r.n);
        // another seed's outputs, or this seed's past the window that still holds
        // output 227 (g > 851): outputs 0..226 again
        if (ring[627] != seed || g < 227 || g > 851) {
            uint32_t a0 = seed, a1 = mt_init_step(seed, 1), b = seed;
            for (uint32_t i = 1; i <= 397; i++) b = mt_init_step(b, i);
            for (uint32_t k = 0; k < 227; k++) {
                ring[k] = mt_twist(a0, a1, b);
                a0 = a1;
                a1 = mt_init_step(a1, k + 2);
                b = mt_init_step(b, k + 398);
            }
            xa0 = a0, xa1 = a1, g = 227;  // x[227], x[228]
            ring[627] = seed;
            ring[628] = a0;  // x[227]: the ring's tag for lanes past draw 227
            moved = true;
        }
    } else if (ring[628] != r.a0 || g < r.n) {
        // another sample's ring (a stale cursor or tag), or this lane drew past
        // what was generated: a schedule error the caller reports
        return false;
    }
    for (; g < want; g++) {
        moved = true;
        uint32_t un, un1;
        if (g < 623) un = xa0, un1 = xa1;
        else if (g == 623) un = xa0, un1 = ring[0];
        else un = ring[(g - 624) % 624], un1 = ring[(g - 623) % 624];
        ring[g % 624] = mt_twist(un, un1, ring[(g - 227) % 624]);
        if (g + 2 <= 623) {
            xa0 = xa1;
            xa1 = mt_init_step(xa1, g + 2);
        } else if (g + 1 <= 623) {
            xa0 = xa1;
        }
    }
    // (also after outputs 0..226 alone: a cursor left from the slot's previous seed
    // next to this seed's ring[627] would read as this seed's outputs)
    if (moved) ring[624] = xa0, ring[625] = xa1, ring[626] = g;
    return true;
}
// The wave generates lane b's ring ahead (the Russian-roulette build's inline
// chain: one lane draws while 63 wait): outputs g .. n + 63, lane j computing
// output g + j from the three words it reads. Every lane reads before any lane
// writes (each store waits on the wave's loads), and fewer than 227 consecutive
// outputs never read one another, so the words are mt_ring_ahead's; only once
// output 624 is past (no seeding values left). n and a0 are lane b's (wave-
// uniform). Returns the outputs generated so far, or 0 when lane b's ring is not
// its own or not that far (lane b then calls mt_ring_ahead, which reports it).
__device__ __forceinline__ uint32_t mt_ring_ahead_wave(int b, uint32_t n, uint32_t a0) {
    const uint64_t base = (static_cast<uint64_t>(g_scene_lds[1]) << 32) | g_scene_lds[0];
    uint32_t* const ring =
        reinterpret_cast<uint32_t*>(base) + static_cast<size_t>(g_scene_lds[3] + (threadIdx.x & ~63u) + b) * kMtRingWords;
    const uint32_t g = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ring[626])));
    const uint32_t tag = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(ring[628])));
    if (tag != a0 || g < n || g < 624) return 0;
    const uint32_t want = n + 64;
    if (g >= want) return g;
    const uint32_t gj = g + __lane_id();
    uint32_t v = 0;
    if (gj < want) v = mt_twist(ring[(gj - 624) % 624], ring[(gj - 623) % 624], ring[(gj - 227) % 624]);
    if (gj < want) ring[gj % 624] = v;
    if (__lane_id() == 0) ring[626] = want;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // (the stores done before lane b reads them)
    return want;
}
__device__ __forceinline__ uint32_t mt_u32_long(LazyMT& r) {
    const uint32_t v = mt_ring_slot()[r.n % 624];
    r.n++;
    return mt_temper(v);
}
#else
constexpr uint32_t kMtRingWords = 624;
__device__ BDPT_NOINLINE uint32_t mt_u32_long(LazyMT& r) {
    const uint64_t base = (static_cast<uint64_t>(g_scene_lds[1]) << 32) | g_scene_lds[0];
    uint32_t* const ring = reinterpret_cast<uint32_t*>(base);
    if (!ring) return mt_next_u32(r);  // unreachable (host check)
    const uint32_t st = g_scene_lds[2];
    const uint32_t seed = r.n == 227 ? mt_seed_from(r.a0, 227) : 0u;
    return mt_ring_step(r, seed, ring + static_cast<size_t>(blockIdx.x * blockDim.x + threadIdx.x) * kMtRingWords, st);
}
#endif  // BDPT_RING_AHEAD
#endif  // BDPT_DEEP_RNG

// generate_canonical<float, 24> (libstdc++ 11 random.tcc:3348-3380).
__device__ __forceinline__ float next1(LazyMT& r) {
#if BDPT_SAMPLER_STATE
    const uint32_t u = mt_state_u32();
    r.n++;
#elif BDPT_DEEP_RNG
    const uint32_t u = r.n < 227 ? mt_next_u32(r) : mt_u32_long(r);
#else
    const uint32_t u = mt_next_u32(r);
#endif
    float f = static_cast<float>(u) / 4294967296.0f;
    return f >= 1.0f ? 0x1.fffffep-1f : f;
}
struct F2 {
    float x, y;
};
__device__ __forceinline__ F2 next2(LazyMT& r) {
    F2 o;
    o.x = next1(r);
    o.y = next1(r);
    return o;
}

// -------------------------------------------------------------------- warps
// squareToUniformHemisphere (math.h:136-144)
__device__ __forceinline__ f3 uniform_hemisphere(F2 u) {
    float phi = u.x * kPi * 2.0f;
    float cosTheta = u.y;
    float sinTheta = sqrt_cr(glibc_fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    const SinCos sc = glibc_sincosf2(phi);
    return mk(sinTheta * sc.c, sinTheta * sc.s, cosTheta);
}
// squareToUniformDiskConcentric + squareToCosineHemisphere (math.h:153-192)
__device__ __forceinline__ f3 cosine_hemisphere(F2 u) {
    float rx = (2.f * u.x) - 1.f;
    float ry = (2.f * u.y) - 1.f;
#ifndef BDPT_DISK_SELECT
#define BDPT_DISK_SELECT 1
#endif
#if BDPT_DISK_SELECT
    // Both branches of the reference as selects (one division, one sincos per
    // lane, same operations and bits); the (0, 0) sample keeps dx = dy = 0.
    const bool zero = rx == 0 && ry == 0;
    const bool xb = (rx * rx) > (ry * ry);
    const float radius = xb ? rx : ry;
    const float q = (kPi * 0.25f) * ((xb ? ry : rx) * rcp_cr(xb ? rx : ry));
    const float phi = zero ? 0.f : (xb ? q : (kPi * 0.5f) - q);
    const SinCos sc = glibc_sincosf2(phi);
    const float dx = zero ? 0.f : radius * sc.c;
    const float dy = zero ? 0.f : radius * sc.s;
#else
    float dx = 0.f, dy = 0.f;
    if (!(rx == 0 && ry == 0)) {
        float radius, phi;
        if ((rx * rx) > (ry * ry)) {
            radius = rx;
            phi = (kPi * 0.25f) * (ry * rcp_cr(rx));
        } else {
            radius = ry;
            phi = (kPi * 0.5f) - ((kPi * 0.25f) * (rx * rcp_cr(ry)));
        }
        const SinCos sc = glibc_sincosf2(phi);
        dx = radius * sc.c;
        dy = radius * sc.s;
    }
#endif
    float z = 1.0f - (dx * dx + dy * dy);
    z = glibc_fmaxf(z, 0.f);
    return mk(dx, dy, sqrt_cr(z));
}
__device__ __forceinline__ float cosine_hemisphere_pdf(f3 v) { return v.z >= 0.f ? v.z * kInvPi : 0.f; }
// squareToPhongLobe / Pdf (math.h:210-227)
__device__ __forceinline__ f3 phong_lobe(F2 u, float ex) {
    float cosTheta = glibc_powf(u.x, 1.f / (ex + 2));
    float sinTheta = sqrt_cr(glibc_fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    float phi = u.y * 2.f * kPi;
    const SinCos sc = glibc_sincosf2(phi);
    return mk(sinTheta * sc.c, sinTheta * sc.s, cosTheta);
}
// EXACT: glibc's powf even in the fast-weight builds (the BSDF sampler, below)
template <bool EXACT = false>
__device__ __forceinline__ float phong_lobe_pdf(f3 v, float ex) {
    return v.z >= 0.f ? (ex + 2) * kInvTwoPi * (EXACT ? glibc_powf(v.z, ex) : pow_w(v.z, ex)) : 0.f;
}
// squareToUniformTriangle (math.h:229-234)
__device__ __forceinline__ F2 uniform_triangle(F2 s) {
    float u = sqrt_cr(1.f - s.x);
    return F2{1 - u, u * s.y};
}

// -------------------------------------------------------------------- frame
// Frame(n) with coordinateSystem (core.h:155-157, math.h:42-51): t = c, s = cross(c, n).
#ifndef BDPT_FRAME_SELECT
#define BDPT_FRAME_SELECT 0  // 1: the operand selected first, one sqrt + division per lane
#endif
__device__ __forceinline__ void make_frame(f3 a, f3& s, f3& t) {
#if BDPT_FRAME_SELECT
    const bool xb = fabsf(a.x) > fabsf(a.y);
    const float u = xb ? a.x : a.y;
    const float inv = rcp_cr(sqrt_cr(u * u + a.z * a.z));
    const float w = a.z * inv, m = -u * inv;
    t = xb ? mk(w, 0.f, m) : mk(0.f, w, m);
#else
    if (fabsf(a.x) > fabsf(a.y)) {
        float inv = rcp_cr(sqrt_cr(a.x * a.x + a.z * a.z));
        t = mk(a.z * inv, 0.f, -a.x * inv);
    } else {
        float inv = rcp_cr(sqrt_cr(a.y * a.y + a.z * a.z));
        t = mk(0.f, a.z * inv, -a.y * inv);
    }
#endif
    s = cross(t, a);
}
__device__ __forceinline__ f3 to_local(f3 s, f3 t, f3 n, f3 v) { return mk(dot(v, s), dot(v, t), dot(v, n)); }
__device__ __forceinline__ f3 to_world(f3 s, f3 t, f3 n, f3 v) { return (s * v.x + t * v.y) + n * v.z; }
__device__ __forceinline__ f3 reflect_z(f3 d) { return mk(-d.x, -d.y, d.z); }
// Shading-frame conversions at a vertex with shading normal n (the frame is
// rebuilt on use rather than kept live in registers between queries).
__device__ __forceinline__ f3 local_at(f3 n, f3 v) {
    f3 s, t;
    make_frame(n, s, t);
    return to_local(s, t, n, v);
}
__device__ __forceinline__ f3 world_at(f3 n, f3 v) {
    f3 s, t;
    make_frame(n, s, t);
    return to_world(s, t, n, v);
}

// ---------------------------------------------------------------- traversal
// BBox::intersect (bvh.h:33-69): the reference's slab test, bit for bit (true
// divisions, same swaps and comparisons), also returning the clipped interval.
__device__ __forceinline__ bool slab(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r,
                                     float& tn, float& tf) {
    float tmin = (lx - r.o.x) / r.d.x, tmax = (hx - r.o.x) / r.d.x;
    if (tmin > tmax) { float q = tmin; tmin = tmax; tmax = q; }
    float tymin = (ly - r.o.y) / r.d.y, tymax = (hy - r.o.y) / r.d.y;
    if (tymin > tymax) { float q = tymin; tymin = tymax; tymax = q; }
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (lz - r.o.z) / r.d.z, tzmax = (hz - r.o.z) / r.d.z;
    if (tzmin > tzmax) { float q = tzmin; tzmin = tzmax; tzmax = q; }
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    tn = tmin;
    tf = tmax;
    return true;
}

// Fast form of the same decision. The reference's test (after its swaps every
// per-axis interval is [lo_i, hi_i]) hits exactly when max_i lo_i <= min_j hi_j.
// Here t = (l - o) * RN(1/d) differs from the reference's RN((l - o) / d) by at
// most ~1.8e-7 |t| (three roundings instead of one), so tf - tn differs from the
// reference's by < 3e-7 (|tn| + |tf|). Decisions within a slack of
// 1e-6 (|tn| + |tf|) + 1e-30 of the boundary defer to slab() above, so the
// hit / miss outcome is always the reference's. Rays whose reciprocal
// direction or origin is not finite (where 0 * inf = NaN could arise) take
// slab() for every box (RayInv::fast == false).
#ifndef BDPT_CULL_NEAR
#define BDPT_CULL_NEAR 1  // 0: no box is culled for lying before t = 5e-4 (only the far cull remains)
#endif
constexpr float kCullNear = BDPT_CULL_NEAR ? 5e-4f : -__builtin_huge_valf();
// The near cull assumes Moller-Trumbore puts a hit where the ray meets its
// triangle. For a ray nearly parallel to a triangle's plane whose origin lies on
// that plane (a grazing ray leaving a surface) the computed t, u, v are rounding
// noise the reference still accepts (t > 1e-3), so such queries walk without the
// near cull: every query leaving a surface (a path vertex or the emitter) at
// |cos| < kGrazeCos to its triangle's plane. Below it the
// t error of a coplanar triangle, ~1.2e-7 |o - v0| / (|cos| sin(corner)), can
// pass 1e-3 only for triangles with a corner under ~0.35 degrees.
constexpr float kGrazeCos = 0.02f;
// The rule is about the origin triangle's geometric plane; the path only holds
// the interpolated shading normal n_s, so each triangle carries a graze code (top
// byte of its shading record's shape word, bdpt_capi.cpp graze_code): n_s lies
// within code / 64 of the geometric normal's direction, and |dot(d, n_s)| <
// kGrazeCos + code / 64 covers every |dot(d, n_g)| < kGrazeCos. Code 0 (flat
// triangles: n_s is n_g) leaves the plain test.
__device__ __forceinline__ int shape_id(int packed) { return packed & 0xffffff; }
#ifndef BDPT_GRAZE
#define BDPT_GRAZE 1  // 0: the plain |cos| < kGrazeCos test (A/B only; not exact on smooth meshes)
#endif
__device__ __forceinline__ float graze_threshold(int packed) {
    return BDPT_GRAZE ? kGrazeCos + static_cast<float>(static_cast<uint32_t>(packed) >> 24) * 0.015625f : kGrazeCos;
}
__device__ __forceinline__ bool graze_exempt(f3 d, f3 n, int packed) { return fabsf(dot(d, n)) < graze_threshold(packed); }
#ifndef BDPT_SLAB_FMA
#define BDPT_SLAB_FMA 2  // slack-free interior boxes by one fma per plane (slab_fma; 1: o inv formed per node step; 0: slab_fast)
#endif
enum : int { kSlabMiss = 0, kSlabHit = 1, kSlabAmbiguous = 2 };
struct RayInv {
    f3 inv;
    bool fast;
    float near;  // boxes left before t = near are culled (kCullNear, or -inf: no near cull, see cull_near_for)
};
#ifndef BDPT_QNODES
#define BDPT_QNODES 0  // 1: the walk reads the 64-byte compressed node records (wide_bvh.hpp quantize_wide_nodes)
#endif
__device__ __forceinline__ bool far_origin(const DevScene& sc, f3 o) {
#if BDPT_QNODES
    if (!sc.q_ok) return true;  // no compressed records: every query walks the reference's tree
#endif
    return !(o.x >= sc.near_lo[0] && o.x <= sc.near_hi[0] && o.y >= sc.near_lo[1] && o.y <= sc.near_hi[1] &&
             o.z >= sc.near_lo[2] && o.z <= sc.near_hi[2]);
}
constexpr float kNoCullNear = -__builtin_huge_valf();
__device__ __forceinline__ RayInv ray_inv(const Ray& r, float near);
__device__ __forceinline__ RayInv ray_inv(const Ray& r, float near) {
    RayInv ri;
    ri.near = near;
    ri.inv = mk(rcp_cr(r.d.x), rcp_cr(r.d.y), rcp_cr(r.d.z));
#if BDPT_SLAB_FMA
    // slab_fma's o inv must be finite too
    const float probe = (ri.inv.x + ri.inv.y + ri.inv.z) * 0.f + ((r.o.x + r.o.y + r.o.z) * 0.f) +
                        ((r.o.x * ri.inv.x + r.o.y * ri.inv.y + r.o.z * ri.inv.z) * 0.f);
#else
    const float probe = (ri.inv.x + ri.inv.y + ri.inv.z) * 0.f + ((r.o.x + r.o.y + r.o.z) * 0.f);
#endif
    ri.fast = (probe == 0.f);  // false iff some component is +-inf or NaN
#if BDPT_QNODES
    // the compressed records' 2^e / d must stay normal and finite (wide_bvh.hpp kQuantExpMin/Max)
    const float m = fmaxf(fmaxf(fabsf(ri.inv.x), fabsf(ri.inv.y)), fabsf(ri.inv.z));
    const float n = fminf(fminf(fabsf(ri.inv.x), fabsf(ri.inv.y)), fabsf(ri.inv.z));
    ri.fast = ri.fast && m <= 0x1p96f && n >= 0x1p-40f;
#endif
    return ri;
}
__device__ __forceinline__ int slab_planes(float x0, float x1, float y0, float y1, float z0, float z1, float& tn,
                                           float& tf) {
    tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    const float d = tf - tn, s = fmaf(fabsf(tn) + fabsf(tf), 1e-6f, 1e-30f);
    return d > s ? kSlabHit : (d < -s ? kSlabMiss : kSlabAmbiguous);  // inf operands: ambiguous
}
__device__ __forceinline__ int slab_fast(float lx, float ly, float lz, float hx, float hy, float hz, f3 o, f3 inv,
                                         float& tn, float& tf) {
    const float x0 = (lx - o.x) * inv.x, x1 = (hx - o.x) * inv.x;
    const float y0 = (ly - o.y) * inv.y, y1 = (hy - o.y) * inv.y;
    const float z0 = (lz - o.z) * inv.z, z1 = (hz - o.z) * inv.z;
    return slab_planes(x0, x1, y0, y1, z0, z1, tn, tf);
}
// The slack-free interior test's plane distances as one fma each,
// fma(l, inv, -RN(o inv)) instead of a subtraction and a product (24 VALU
// instead of 48 per 4-wide node; Caustic +1.1 %, HardLight +1.0 %, synth1m
// +1.3 %). Against the exact (l - o) / d the error is at most
// 2^-23 |t| + 2^-24 |o_i inv_i| per plane, i.e. 2^-23 |l_i - o_i| + 2^-24 |o_i| in
// scene units along axis i: node_slack_needed admits it only while every origin
// and the scene box lie within kFmaCoordDiags diagonals of 0 (bdpt_capi.cpp), where
// it stays below slab_fast's own bound and inside the boxes' padding.
__device__ __forceinline__ f3 slab_fma_origin(f3 o, f3 inv) {
    f3 oi = mk(-(o.x * inv.x), -(o.y * inv.y), -(o.z * inv.z));
#if BDPT_SLAB_FMA == 1
    asm volatile("" : "+v"(oi.x), "+v"(oi.y), "+v"(oi.z));  // formed per node step, not held across the walk
#endif
    return oi;
}
__device__ __forceinline__ void slab_fma(float lx, float ly, float lz, float hx, float hy, float hz, f3 oi, f3 inv,
                                         float& tn, float& tf) {
    const float x0 = fmaf(lx, inv.x, oi.x), x1 = fmaf(hx, inv.x, oi.x);
    const float y0 = fmaf(ly, inv.y, oi.y), y1 = fmaf(hy, inv.y, oi.y);
    const float z0 = fmaf(lz, inv.z, oi.z), z1 = fmaf(hz, inv.z, oi.z);
    tn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    tf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
}

__device__ __forceinline__ int cross_le(float a, float b) {  // a <= b with the same slack
    const float d = b - a, s = fmaf(fabsf(a) + fabsf(b), 1e-6f, 1e-30f);
    return d > s ? kSlabHit : (d < -s ? kSlabMiss : kSlabAmbiguous);
}
// Second chance for an ambiguous max-lo vs min-hi decision: the reference's
// test is the six cross pairs lo_i <= hi_j (i != j) — the pair of a flat
// (zero-thickness) box axis, tn == tf on a planar wall, never enters it.
__device__ __forceinline__ int slab_cross(float lx, float ly, float lz, float hx, float hy, float hz, f3 o,
                                          f3 inv) {
    const float x0 = (lx - o.x) * inv.x, x1 = (hx - o.x) * inv.x;
    const float y0 = (ly - o.y) * inv.y, y1 = (hy - o.y) * inv.y;
    const float z0 = (lz - o.z) * inv.z, z1 = (hz - o.z) * inv.z;
    const float lox = fminf(x0, x1), hix = fmaxf(x0, x1);
    const float loy = fminf(y0, y1), hiy = fmaxf(y0, y1);
    const float loz = fminf(z0, z1), hiz = fmaxf(z0, z1);
    const int a = cross_le(lox, fminf(hiy, hiz)), b = cross_le(loy, fminf(hix, hiz)),
              c = cross_le(loz, fminf(hix, hiy));
    if (a == kSlabMiss || b == kSlabMiss || c == kSlabMiss) return kSlabMiss;
    return (a & b & c) == kSlabHit ? kSlabHit : kSlabAmbiguous;
}

template <bool COUNT>
__device__ __forceinline__ bool box_test(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r,
                                         const RayInv& ri, float& tn, float& tf, uint32_t& fallbacks) {
    if (ri.fast) {
        int f = slab_fast(lx, ly, lz, hx, hy, hz, r.o, ri.inv, tn, tf);
        if (f == kSlabAmbiguous) f = slab_cross(lx, ly, lz, hx, hy, hz, r.o, ri.inv);
        if (f != kSlabAmbiguous) return f == kSlabHit;
    }
    if (COUNT) fallbacks++;
    return slab(lx, ly, lz, hx, hy, hz, r, tn, tf);
}

// rayTriangleIntersect (core.h:379-400) + accel.h:43's t > 1e-3, on the
// triangle's v0 and edges (e1 = v1 - v0, e2 = v2 - v0 rounded as the
// reference rounds them).
__device__ __forceinline__ bool tri_test_raw(f3 v0, f3 e1, f3 e2, const Ray& r, float& t, float& u, float& v) {
    const f3 pvec = cross(r.d, e2);
    const float det = dot(e1, pvec);
    if (fabsf(det) < kEpsilon) return false;
    const float invDet = rcp_det(det);  // |det| >= kEpsilon here
    const f3 tvec = r.o - v0;
    u = dot(tvec, pvec) * invDet;
    if (u < 0.f || u > 1.f) return false;
    const f3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * invDet;
    if (v < 0.f || u + v > 1.f) return false;
    t = dot(e2, qvec) * invDet;
    return true;
}
__device__ __forceinline__ bool tri_test_edges(f3 v0, f3 e1, f3 e2, const Ray& r, float& t, float& u, float& v) {
    return tri_test_raw(v0, e1, e2, r, t, u, v) && t >= kTriMinT;
}
__device__ __forceinline__ bool tri_test(const float4* __restrict__ tri, uint32_t i, const Ray& r, float& t, float& u,
                                         float& v) {
    return tri_test_edges(xyz(gld4(tri + 3 * i)), xyz(gld4(tri + 3 * i + 1)), xyz(gld4(tri + 3 * i + 2)), r, t, u, v);
}

// Traversal stack of (link, t_near) entries: the first kLdsStack entries of a
// lane live in LDS (entry k of thread x at lds[k * stride + x]: 8-byte lanes,
// conflict-free), deeper ones spill to a per-lane HBM column (rare; the host
// sizes it to the scene's worst case).
#ifndef BDPT_LDS_STACK
#define BDPT_LDS_STACK 7  // traversal-stack entries per lane in LDS (deeper ones spill to HBM, rare); 7 leaves the LDS room for the root nodes
#endif
constexpr int kLdsStack = BDPT_LDS_STACK;
constexpr uint32_t kEmptyLinkDev = 0xffffffffu;  // unused 4-wide child slot
// The accesses name their address space (LDS: ds_*, HBM: global_*): through
// the generic pointers the compiler merged the two branches into one FLAT
// access, and every FLAT load waits for vmcnt(0) and lgkmcnt(0) together —
// each pop then also waited for all of the wave's outstanding global loads.
#ifndef BDPT_STACK_AS
#define BDPT_STACK_AS 1
#endif
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#if BDPT_STACK_AS
typedef __attribute__((address_space(3))) u32x2 lds_uint2;
typedef __attribute__((address_space(1))) u32x2 gbl_uint2;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) uint32_t gbl_u32;
typedef __attribute__((address_space(1))) int32_t gbl_i32;
#else
typedef u32x2 lds_uint2;
typedef u32x2 gbl_uint2;
typedef uint32_t lds_u32;
typedef uint32_t gbl_u32;
typedef int32_t gbl_i32;
#endif
// threadIdx.x, re-read at each use (opaque to the optimiser): per-lane
// addresses derived from it at their use are not held in registers across the
// persistent loop (only threadIdx.x itself is).
__device__ __forceinline__ uint32_t opaque_tid() {
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

struct Stack {
    uint2* lds;
    int stride;
    int nlds;    // entries held in LDS
    uint2* gbl;  // entry k >= nlds at gbl[(k - nlds) * nslots + slot] (the frame kernels: the slot's block, nslots 1)
    uint32_t nslots, slot;
    bool tid_rel = false;  // lds and slot are the block's bases; the lane adds threadIdx.x at each access
    __device__ __forceinline__ uint32_t lane_off() const { return tid_rel ? opaque_tid() : 0u; }
    __device__ __forceinline__ void put(int k, uint32_t link, float tn) const {
        const u32x2 e = {link, __float_as_uint(tn)};
        const uint32_t t = lane_off();
        if (k < nlds) ((lds_uint2*)lds)[t + k * stride] = e;
        else ((gbl_uint2*)gbl)[static_cast<size_t>(k - nlds) * nslots + slot + t] = e;
    }
    __device__ __forceinline__ uint2 get(int k) const {
        const uint32_t t = lane_off();
        const u32x2 e = k < nlds ? ((const lds_uint2*)lds)[t + k * stride]
                                 : ((const gbl_uint2*)gbl)[static_cast<size_t>(k - nlds) * nslots + slot + t];
        return make_uint2(e.x, e.y);
    }
};

// Link-only stack for the binary reference traversal in kernels that keep a
// deeper LDS column of 4-byte entries (entry k of thread x at lds[k * stride]).
struct LinkStack {
    uint32_t* lds;
    int stride;
    int nlds;
    uint32_t* gbl;  // entry k >= nlds at gbl[(k - nlds) * nslots + slot]
    uint32_t nslots, slot;
    __device__ __forceinline__ void put(int k, uint32_t link, float) const {
        if (k < nlds) ((lds_u32*)lds)[k * stride] = link;
        else ((gbl_u32*)gbl)[static_cast<size_t>(k - nlds) * nslots + slot] = link;
    }
    __device__ __forceinline__ uint2 get(int k) const {
        if (k < nlds) return make_uint2(((const lds_u32*)lds)[k * stride], 0u);
        return make_uint2(((const gbl_u32*)gbl)[static_cast<size_t>(k - nlds) * nslots + slot], 0u);
    }
};

// Conservative distance culling. The reference never culls by distance
// (bbhits stay 0, bvh.h:265-337): its result is the minimum-t triangle among
// ALL reachable leaves, first-found (= lowest leaf index) on ties. Boxes
// entered beyond best + margin, or exited before t = 5e-4, cannot hold a
// triangle that changes that result.
#ifndef BDPT_CULL_FMA
#define BDPT_CULL_FMA 1  // the margin's product and sum as one fma (the same bound within an ulp; the margin is 1e-3 relative)
#endif
__device__ __forceinline__ float cull_far(float best) {
    return BDPT_CULL_FMA ? fmaf(fabsf(best), 1e-3f, best) + 1e-4f : best + fabsf(best) * 1e-3f + 1e-4f;
}
// The far bound of a walk in progress. An occlusion query's best_t stays its
// max_t (trav_begin; wleaf_tests returns at its first hit without lowering it),
// so ts.best_t serves both kinds of query.
#ifndef BDPT_FAR_BEST
#define BDPT_FAR_BEST 1  // 0: the select on the query kind (with CULL_FMA and ROOT_NF: Caustic +0.65 %, HardLight +0.65 %, synth1m +0.6 %)
#endif
#define BDPT_WALK_FAR(any, r, ts) cull_far(BDPT_FAR_BEST ? (ts).best_t : ((any) ? (r).max_t : (ts).best_t))

struct Counts {
    uint32_t c[kCounters];
    uint32_t m[3];  // maxima (counting pass): light-subpath depth, eye-subpath depth, queries per sample
    // connection-task histogram of the shading steps (frame kernels' counting pass): the
    // tasks a wave holds when it shades — connectVertices still to run (nl - ci at A_CONN),
    // connectToLight + all connections of a new eye vertex, connectToCamera of a new light
    // vertex — summed over steps, the steps, steps with >= 32 and >= 64 tasks. The
    // BDPT_HELP builds count their task rings here instead: tasks pushed, pushes
    // refused (ring full: the owner traces the ray), claim rounds, tasks claimed.
    uint32_t q[4];
    uint32_t t_step;  // this lane's tasks in the current shading step
};
// [5..8] Russian-roulette build: the most walks past BDPT_EXPRESS_DEPTH bounces one wave
// held at once, and the express-mode loop iterations of waves holding 1, 2..BDPT_COOP_MAX,
// more such walks
enum : int { kDiagStart = 0, kDiagLastClaim = 1, kDiagEnd = 2, kDiagErrors = 3, kDiagParked = 4, kDiagLongMax = 5,
             kDiagExpress1 = 6, kDiagExpressCoop = 7, kDiagExpressMore = 8, kDiagWords = 9 };

// Set bits of a wave mask as an int. (HIP's __popcll is typed unsigned long long
// here: mixed with int in min / max it selected the double overloads, and the
// refill and shade-threshold arithmetic ran in f64.)
__device__ __forceinline__ int popc64(uint64_t m) { return __builtin_popcountll(m); }
// The lane's rank among the set lanes of m below it (mbcnt: no per-lane mask
// held across the loop).
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}

// Lane i's value in every lane, for a wave-uniform i: v_readlane (a scalar
// result, a few cycles) where __shfl's ds_bpermute takes an LDS round trip
// (BDPT_READLANE; 0 keeps the shuffles). The value is the lane's register whether
// or not it is active.
#ifndef BDPT_READLANE
#define BDPT_READLANE 1
#endif
#if BDPT_READLANE
__device__ __forceinline__ int lane_val(int x, int i) { return __builtin_amdgcn_readlane(x, i); }
__device__ __forceinline__ float lane_val(float x, int i) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), i));
}
#else
__device__ __forceinline__ int lane_val(int x, int i) { return __shfl(x, i); }
__device__ __forceinline__ float lane_val(float x, int i) { return __shfl(x, i); }
#endif

// SIMD-efficiency probe: true on the lowest active lane of the wave only.
__device__ __forceinline__ bool first_active_lane() {
    return (__lane_id()) == static_cast<unsigned>(__ffsll(static_cast<unsigned long long>(__ballot(1))) - 1);
}

// Triangle tests of one reference leaf (bvh.h:291-309). Closest: keeps the
// minimum t, ties to the lowest index (the reference's strict `<` in its
// left-first DFS = leaf order). Any: true on a hit with t <= max_t — the
// reference's occlusion query returns at a hit inside [min_t, max_t] and
// otherwise reports any hit closer than max_t it kept (bvh.h:298-305, :350).
// The triangles are fetched BDPT_LEAF_GROUP at a time with all their loads in
// flight together (one memory round trip per group instead of two per
// triangle); indices past the leaf's count are clamped and their results unused.
#ifndef BDPT_LEAF_GROUP
#define BDPT_LEAF_GROUP 1
#endif
#ifndef BDPT_LEAF_PIPELINE
#define BDPT_LEAF_PIPELINE 0  // 1: fetch triangle k + 1 while testing triangle k
#endif
template <bool COUNT>
__device__ __forceinline__ bool leaf_tests(const float4* __restrict__ tri, uint32_t link, const Ray& r, bool any, float& best_t,
                                           int& best, float& best_u, float& best_v, uint32_t& tri_count) {
    constexpr uint32_t G = BDPT_LEAF_GROUP;
    const uint32_t start = (link >> 3) & 0x0fffffffu, count = link & 7u;
#if BDPT_LEAF_PIPELINE
    float4 n0 = gld4(tri + 3 * start), n1 = gld4(tri + 3 * start + 1), n2 = gld4(tri + 3 * start + 2);
    for (uint32_t k = 0; k < count; k++) {
        const float4 a0 = n0, a1 = n1, a2 = n2;
        const uint32_t nx = start + (k + 1 < count ? k + 1 : k);
        n0 = gld4(tri + 3 * nx), n1 = gld4(tri + 3 * nx + 1), n2 = gld4(tri + 3 * nx + 2);
        asm volatile("" ::"v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a2.x), "v"(a2.y),
                     "v"(a2.z));
        const uint32_t i = start + k;
        float t, u, v;
        if (COUNT) tri_count++;
        if (tri_test_edges(xyz(a0), xyz(a1), xyz(a2), r, t, u, v)) {
            if (any) {
                if (t <= r.max_t && t >= r.min_t) {
                    best = 1;
                    return true;
                }
            } else if (t < best_t || (t == best_t && best >= 0 && static_cast<int>(i) < best)) {
                best_t = t, best = static_cast<int>(i), best_u = u, best_v = v;
            }
        }
    }
    return false;
#endif
    for (uint32_t k0 = 0; k0 < count; k0 += G) {
        float4 q[G][3];
#pragma unroll
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t i = start + (k0 + g < count ? k0 + g : count - 1);
            q[g][0] = gld4(tri + 3 * i), q[g][1] = gld4(tri + 3 * i + 1), q[g][2] = gld4(tri + 3 * i + 2);
        }
#pragma unroll
        for (uint32_t g = 0; g < G; g++)
#pragma unroll
            for (int j = 0; j < 3; j++) asm volatile("" ::"v"(q[g][j].x), "v"(q[g][j].y), "v"(q[g][j].z));
#pragma unroll
        for (uint32_t g = 0; g < G; g++) {
            const uint32_t k = k0 + g;
            if (k >= count) break;
            const uint32_t i = start + k;
            float t, u, v;
            if (COUNT) tri_count++;
            if (tri_test_edges(xyz(q[g][0]), xyz(q[g][1]), xyz(q[g][2]), r, t, u, v)) {
                if (any) {
                    if (t <= r.max_t) {
                        best = 1;
                        return true;
                    }
                } else if (t < best_t || (t == best_t && best >= 0 && static_cast<int>(i) < best)) {
                    best_t = t, best = static_cast<int>(i), best_u = u, best_v = v;
                }
            }
        }
    }
    return false;
}

struct TravResult {
    int best;
    float t, u, v;
    uint32_t nodes, tris, exact;  // counting pass only
};

// BVH::getIntersection (bvh.h:259-352) over the reference's own binary tree:
// every box decided exactly as the reference decides it. Used for rays the
// 4-wide hierarchy cannot serve (zero / non-finite reciprocal direction, where
// the slab test is not monotone) and for BDPT_FLAG_FULL_TRAVERSAL (cull =
// false: every box the reference visits). Out of line, arguments by value
// (nothing of the caller's lives in scratch).
template <bool COUNT, typename StackT>
__device__ BDPT_NOINLINE TravResult traverse_binary(const DevScene& sc, Ray r, bool any, bool cull, StackT stk) {
    TravResult res{-1, r.max_t, 0.f, 0.f, 0u, 0u, 0u};
    uint32_t link = sc.root_link;
    int sp = 0;
    for (;;) {
        if (link & kLeafBit) {
            if (leaf_tests<COUNT>(sc.tri, link, r, any, res.t, res.best, res.u, res.v, res.tris)) break;
        } else {
            if (COUNT) res.nodes++, res.exact += 2;
            const float4* nd = sc.nodes + 4 * static_cast<size_t>(link);
            const float4 q0 = gld4(nd), q1 = gld4(nd + 1), q2 = gld4(nd + 2), q3 = gld4(nd + 3);
            float tn0, tf0, tn1, tf1;
            bool h0 = slab(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, r, tn0, tf0);
            bool h1 = slab(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r, tn1, tf1);
            const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
            if (cull) {
                const float far = cull_far(any ? r.max_t : res.t);
                h0 = h0 && !(tn0 > far) && !(tf0 < kCullNear);
                h1 = h1 && !(tn1 > far) && !(tf1 < kCullNear);
            }
            if (h0 && h1) {
                stk.put(sp++, l1, 0.f);
                link = l0;
                continue;
            }
            if (h0) { link = l0; continue; }
            if (h1) { link = l1; continue; }
        }
        if (sp == 0) break;
        link = stk.get(--sp).x;
    }
    return res;
}

// Fast, conservative box decision for one child of a 4-wide node: the slab
// intervals from RN(1/d), then tn/tf and the max-lo <= min-hi decision with the
// slack of slab_fast (kSlabAmbiguous when too close to call).
__device__ __forceinline__ int child_fast(float lx, float hx, float ly, float hy, float lz, float hz, f3 o, f3 inv,
                                          float& tn, float& tf) {
    return slab_fast(lx, ly, lz, hx, hy, hz, o, inv, tn, tf);
}

// Closest-hit / occlusion query over the 4-wide hierarchy (wide_bvh.hpp),
// written as a resumable step so persistent kernels can refill finished lanes.
// Every child box is tested conservatively (an ambiguous fast test counts as a
// hit): the boxes bound the (padded) triangles below them. Whether a triangle
// is a candidate of the reference's search at all is decided per triangle hit,
// by the exact test of its reference leaf box (wleaf_tests). Children are
// visited near-first; stacked entries carry their entry distance and are
// dropped on pop once a closer hit exists.
// The scene pointers a walk needs, copied once per query into registers: the
// DevScene lives in a parameter block in global memory, and reading a field
// through it inside the node loop would put a dependent load in front of
// every node fetch (the compiler must assume the block may change).
struct TravScene {
    const float4* __restrict__ wtri;
    const float4* __restrict__ lbox;
    const float4* __restrict__ wnodes;  // the records the walk reads (qnodes in the BDPT_QNODES build)
    uint32_t wroot_link;
    uint32_t node_slack;  // 0: interior boxes tested without the ambiguity slack (DevScene::node_slack)
};
__device__ __forceinline__ const float4* uniform_ptr(const float4* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v & 0xffffffffu)));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)));
    return reinterpret_cast<const float4*>((static_cast<uint64_t>(hi) << 32) | lo);
}
__device__ __forceinline__ TravScene trav_scene(const DevScene& sc) {
    return TravScene{uniform_ptr(sc.wtri), uniform_ptr(sc.lbox), uniform_ptr(BDPT_QNODES ? sc.qnodes : sc.wnodes),
                     static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sc.wroot_link))),
                     static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(sc.node_slack)))};
}

// Triangle tests of one traversal leaf (wtri records). A hit is a candidate of
// the reference's search iff the triangle's reference leaf box passes
// BBox::intersect (bvh.h:33-69; wide_bvh.hpp) — checked exactly (fast test,
// cross pairs, the reference's divisions) and only for a hit that would become
// the closest (minimum t, ties to the lowest reference index = the reference's
// strict `<` in its left-first DFS) or that ends an occlusion query (t <= max_t,
// see leaf_tests).
template <bool COUNT>
__device__ __forceinline__ bool ref_leaf_passes(const float4* __restrict__ lbox, uint32_t leaf, const Ray& r,
                                                const RayInv& ri, Counts& cnt) {
    const float4 lo = gld4(lbox + 2 * static_cast<size_t>(leaf)), hi = gld4(lbox + 2 * static_cast<size_t>(leaf) + 1);
    float tn, tf;
    uint32_t fb = 0;
    const bool pass = box_test<COUNT>(lo.x, lo.y, lo.z, hi.x, hi.y, hi.z, r, ri, tn, tf, fb);
    if (COUNT) cnt.c[15] += fb;
    return pass;
}
template <bool COUNT>
__device__ __forceinline__ bool wleaf_tests(const float4* __restrict__ wtri, const float4* __restrict__ lbox,
                                            uint32_t link, const Ray& r, const RayInv& ri, bool any, float& best_t,
                                            int& best, float& best_u, float& best_v, Counts& cnt) {
    const uint32_t start = (link >> 3) & 0x0fffffffu, count = link & 7u;
    for (uint32_t k = 0; k < count; k++) {
        const size_t i = static_cast<size_t>(start + k);
        const float4 q0 = gld4(wtri + 3 * i), q1 = gld4(wtri + 3 * i + 1), q2 = gld4(wtri + 3 * i + 2);
        float t, u, v;
        if (COUNT) cnt.c[3]++;
        if (!tri_test_edges(xyz(q0), xyz(q1), xyz(q2), r, t, u, v)) continue;
        const int idx = __float_as_int(q0.w);
        if (any) {
            if (t <= r.max_t && ref_leaf_passes<COUNT>(lbox, __float_as_uint(q1.w), r, ri, cnt)) {
                best = idx;
                return true;
            }
        } else if ((t < best_t || (t == best_t && best >= 0 && idx < best)) &&
                   ref_leaf_passes<COUNT>(lbox, __float_as_uint(q1.w), r, ri, cnt)) {
            best_t = t, best = idx, best_u = u, best_v = v;
        }
    }
    return false;
}

struct TravState {
    uint32_t link;
    int sp;
    int best;
    float best_t, best_u, best_v;
};

__device__ __forceinline__ TravState trav_begin(const TravScene& sc, const Ray& r) {
    return TravState{sc.wroot_link, 0, -1, r.max_t, 0.f, 0.f};
}

// Pops the nearest pending entry that can still hold a closer hit; false when
// the traversal is complete.
__device__ __forceinline__ bool trav_pop(const Ray& r, bool any, TravState& ts, const Stack& stk,
                                         uint32_t* culled = nullptr) {
    while (ts.sp > 0) {
        const uint2 e = stk.get(--ts.sp);
        if (!(__uint_as_float(e.y) > BDPT_WALK_FAR(any, r, ts))) {
            ts.link = e.x;
            return true;
        }
        if (culled) (*culled)++;
    }
    return false;
}

// A 4-wide node record as the walk reads it: the 128-byte float record
// (wide_bvh.hpp; v[0..5] = lo.x hi.x lo.y hi.y lo.z hi.z, v[6] = links) or, in
// the BDPT_QNODES build, the 64-byte compressed one (v[0] = grid origin and
// exponents, v[1..2] = 8-bit child bounds, v[3] = links).
#if BDPT_QNODES
constexpr int kNodeVecs = 4, kNodeStride = 4, kNodeLinks = 3;
#else
constexpr int kNodeVecs = 7, kNodeStride = 8, kNodeLinks = 6;
#endif
struct WNode {
    float4 v[kNodeVecs];
};
__device__ __forceinline__ WNode load_wnode(const float4* __restrict__ base, uint32_t link) {
    const float4* nd = base + kNodeStride * static_cast<size_t>(link);
    WNode n;
#pragma unroll
    for (int j = 0; j < kNodeVecs; j++) n.v[j] = gld4(nd + j);
    return n;
}
#ifndef BDPT_SLAB_SIGN
#define BDPT_SLAB_SIGN 2  // slack-free interior test: each axis's near / far planes picked by the ray's sign at the load (1: the offsets formed per node step; 0: off)
#endif
#ifndef BDPT_HIT_MERGE
#define BDPT_HIT_MERGE 1  // that test's culls as one comparison, max(tn, near) <= min(tf, far)
#endif
#if !BDPT_QNODES && BDPT_SLAB_SIGN
// The node as the slack-free test reads it (NF): v[0] / v[1] the near / far x
// planes of the four children for this ray — lo.x / hi.x when d.x > 0, hi.x /
// lo.x otherwise (RayInv::fast: inv is finite and nonzero) — likewise v[2..5] for
// y and z, v[6] the links. Each pair is one 128-byte record's 16-byte vectors at
// offsets (s, s ^ 16) from the axis's base with s = 16 for a negative direction:
// per-lane 32-bit offsets from the uniform base (the host keeps the node array
// under 4 GiB for this test, node_slack_needed). With inv > 0, l <= h gives
// fma(l, inv, oi) <= fma(h, inv, oi) (rounding is monotone), so max3 / min3 of
// the picked planes are the entry / exit distances slab_fma's six min / max form
// (one max3 and one min3 per child instead of eight operations; with the merged
// culls below: Caustic +2.3 %, HardLight +3.4 %, synth1m +3.7 %).
__device__ __forceinline__ uint32_t plane_sel(float inv) { return (__float_as_uint(inv) >> 27) & 16u; }
__device__ __forceinline__ WNode load_wnode_nf(const float4* __restrict__ base, uint32_t link, f3 inv) {
    const char* b = reinterpret_cast<const char*>(base);
    const uint32_t off = link << 7;
    uint32_t sx = plane_sel(inv.x), sy = plane_sel(inv.y), sz = plane_sel(inv.z);
#if BDPT_SLAB_SIGN == 1
    asm volatile("" : "+v"(sx), "+v"(sy), "+v"(sz));  // formed per node step, not held across the walk
#endif
    const uint32_t ax = off | sx, ay = off | sy, az = off | sz;
    WNode n;
    n.v[0] = gld4(reinterpret_cast<const float4*>(b + ax));
    n.v[1] = gld4(reinterpret_cast<const float4*>(b + (ax ^ 16u)));
    n.v[2] = gld4(reinterpret_cast<const float4*>(b + ay + 32));
    n.v[3] = gld4(reinterpret_cast<const float4*>(b + (ay ^ 16u) + 32));
    n.v[4] = gld4(reinterpret_cast<const float4*>(b + az + 64));
    n.v[5] = gld4(reinterpret_cast<const float4*>(b + (az ^ 16u) + 64));
    n.v[6] = gld4(reinterpret_cast<const float4*>(b + off + 96));
    return n;
}
#endif
__device__ __forceinline__ float qbyte(float w, int c) {  // byte c of the word, as a float (v_cvt_f32_ubyteN)
    return static_cast<float>((__float_as_uint(w) >> (8 * c)) & 0xffu);
}

// Interior 4-wide node ts.link: tests the four children, descends into the
// nearest hit child (true) and stacks the others far-to-near; false when no
// child is hit (the caller pops).
template <bool COUNT, bool SLACK, bool NF = false>
__device__ __forceinline__ bool trav_node_vals(const WNode& n, const Ray& r, const RayInv& ri, bool any,
                                               TravState& ts, const Stack& stk, Counts& cnt);
template <bool COUNT, bool SLACK>
__device__ __forceinline__ bool trav_node(const TravScene& sc, const Ray& r, const RayInv& ri, bool any, TravState& ts,
                                          const Stack& stk, Counts& cnt) {
#if !BDPT_QNODES && BDPT_SLAB_SIGN
    if (!SLACK) return trav_node_vals<COUNT, false, true>(load_wnode_nf(sc.wnodes, ts.link, ri.inv), r, ri, any, ts, stk, cnt);
#endif
    return trav_node_vals<COUNT, SLACK>(load_wnode(sc.wnodes, ts.link), r, ri, any, ts, stk, cnt);
}
// The four children of a 4-wide node: key = entry distance of each child the
// walk must visit (box hit, entered before `far`, left after the near cull), +inf
// otherwise, sorted near-first together with the links (kEmptyLinkDev for none).
template <bool SLACK, bool NF = false>
__device__ __forceinline__ void node_child_keys(const WNode& n, const Ray& r, const RayInv& ri, float far, float (&key)[4],
                                                uint32_t (&lnk)[4]) {
    const float4 lk = n.v[kNodeLinks];
#if BDPT_QNODES
    // plane distance of bound org + q 2^e: fma(q, 2^e / d, (org - o) / d); 2^e / d is exact
    const uint32_t eb = __float_as_uint(n.v[0].w);
    const float ax = __uint_as_float((eb & 0xffu) << 23) * ri.inv.x;
    const float ay = __uint_as_float(((eb >> 8) & 0xffu) << 23) * ri.inv.y;
    const float az = __uint_as_float(((eb >> 16) & 0xffu) << 23) * ri.inv.z;
    const float bx = (n.v[0].x - r.o.x) * ri.inv.x, by = (n.v[0].y - r.o.y) * ri.inv.y,
                bz = (n.v[0].z - r.o.z) * ri.inv.z;
#else
    const f3 oi = SLACK || !(BDPT_SLAB_FMA || NF) ? mk(0.f, 0.f, 0.f) : slab_fma_origin(r.o, ri.inv);
#endif
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const uint32_t l = __float_as_uint((&lk.x)[c]);
        float tn, tf;
#if BDPT_QNODES
        const int d = slab_planes(fmaf(qbyte(n.v[1].x, c), ax, bx), fmaf(qbyte(n.v[1].y, c), ax, bx),
                                  fmaf(qbyte(n.v[1].z, c), ay, by), fmaf(qbyte(n.v[1].w, c), ay, by),
                                  fmaf(qbyte(n.v[2].x, c), az, bz), fmaf(qbyte(n.v[2].y, c), az, bz), tn, tf);
#else
        const float clx = (&n.v[0].x)[c], chx = (&n.v[1].x)[c], cly = (&n.v[2].x)[c], chy = (&n.v[3].x)[c],
                    clz = (&n.v[4].x)[c], chz = (&n.v[5].x)[c];
        int d = kSlabHit;
        if (NF) {  // v[0], v[2], v[4]: near planes; v[1], v[3], v[5]: far planes (load_wnode_nf)
            tn = fmaxf(fmaxf(fmaf(clx, ri.inv.x, oi.x), fmaf(cly, ri.inv.y, oi.y)), fmaf(clz, ri.inv.z, oi.z));
            tf = fminf(fminf(fmaf(chx, ri.inv.x, oi.x), fmaf(chy, ri.inv.y, oi.y)), fmaf(chz, ri.inv.z, oi.z));
        } else if (SLACK || !BDPT_SLAB_FMA) {
            d = slab_fast(clx, cly, clz, chx, chy, chz, r.o, ri.inv, tn, tf);
        } else {
            slab_fma(clx, cly, clz, chx, chy, chz, oi, ri.inv, tn, tf);
        }
#endif
        const bool pass = SLACK ? d != kSlabMiss : !(tn > tf);
#if BDPT_HIT_MERGE
        // !(tn > tf), !(tn > far) and !(tf < near) as one comparison: it also drops the
        // boxes when far < near, where no hit can be accepted (the query's max_t or
        // best hit lies below kTriMinT); tn, tf are finite here (RayInv::fast)
        const bool hit = NF ? l != kEmptyLinkDev && !(fmaxf(tn, ri.near) > fminf(tf, far))
                            : l != kEmptyLinkDev && pass && !(tn > far) && !(tf < ri.near);
#else
        const bool hit = l != kEmptyLinkDev && pass && !(tn > far) && !(tf < ri.near);
#endif
        key[c] = hit ? tn : __builtin_inff();
        lnk[c] = hit ? l : kEmptyLinkDev;
    }
    // near-first order: sorting network on (key, link)
#define BDPT_CE(a, b)                                                       \
    {                                                                       \
        const bool sw = key[b] < key[a];                                    \
        const float k0 = sw ? key[b] : key[a], k1 = sw ? key[a] : key[b];   \
        const uint32_t l0 = sw ? lnk[b] : lnk[a], l1 = sw ? lnk[a] : lnk[b]; \
        key[a] = k0, key[b] = k1, lnk[a] = l0, lnk[b] = l1;                 \
    }
    BDPT_CE(0, 1) BDPT_CE(2, 3) BDPT_CE(0, 2) BDPT_CE(1, 3) BDPT_CE(1, 2)
#undef BDPT_CE
}
template <bool COUNT, bool SLACK, bool NF>
__device__ __forceinline__ bool trav_node_vals(const WNode& n, const Ray& r, const RayInv& ri, bool any,
                                               TravState& ts, const Stack& stk, Counts& cnt) {
    if (COUNT) cnt.c[2]++;
    float key[4];
    uint32_t lnk[4];
    node_child_keys<SLACK, NF>(n, r, ri, BDPT_WALK_FAR(any, r, ts), key, lnk);
    if (lnk[0] == kEmptyLinkDev) return false;
    if (lnk[3] != kEmptyLinkDev) stk.put(ts.sp++, lnk[3], key[3]);
    if (lnk[2] != kEmptyLinkDev) stk.put(ts.sp++, lnk[2], key[2]);
    if (lnk[1] != kEmptyLinkDev) stk.put(ts.sp++, lnk[1], key[1]);
    if (COUNT && !BDPT_HELP_CLOCKS) {  // stack-depth probe: entries held at depth >= 8, >= 12, >= 16
        cnt.c[16] += ts.sp > 8 ? ts.sp - 8 : 0;
        cnt.c[17] += ts.sp > 12 ? ts.sp - 12 : 0;
        cnt.c[18] += ts.sp > 16 ? ts.sp - 16 : 0;
    }
    ts.link = lnk[0];
    return true;
}

// The traversal tree's root node and its interior children (slot k = the
// root's child k) in LDS, copied by each block at kernel start (before the
// barrier of scene_tables_to_lds). Every walk starts at the root, so a query's
// first two node tests run when the lane issues it — with the other lanes of
// the shading step, from broadcast LDS reads — instead of as the first two
// global-memory steps of the walk loop (walk_begin_lds).
struct RootLds {
    WNode root;
    WNode kid[4];
};
#ifndef BDPT_COOP_ROOT_LDS
#define BDPT_COOP_ROOT_LDS 0  // cooperative walks read the root and its children from the block's LDS copy
#endif
__device__ __forceinline__ bool root_lds_usable(const DevScene& sc) { return !(sc.wroot_link & kLeafBit); }
__device__ __forceinline__ WNode coop_node(const TravScene& sc, uint32_t link, const RootLds* rl) {
    if (BDPT_COOP_ROOT_LDS && rl) {
        if (link == sc.wroot_link) return rl->root;
        const float4 lk = rl->root.v[kNodeLinks];
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (link == __float_as_uint((&lk.x)[k])) return rl->kid[k];  // (a leaf link never reaches here)
    }
    return load_wnode(sc.wnodes, link);
}
__device__ __forceinline__ void root_lds_fill(RootLds& m, const DevScene& sc) {
    if (!root_lds_usable(sc)) return;
    const float4* const base = BDPT_QNODES ? sc.qnodes : sc.wnodes;
    const float4* rn = base + kNodeStride * static_cast<size_t>(sc.wroot_link);
    if (threadIdx.x < kNodeVecs) {
        m.root.v[threadIdx.x] = gld4(rn + threadIdx.x);
    } else if (threadIdx.x >= 64 && threadIdx.x < 64 + 4 * kNodeVecs) {
        const int k = (threadIdx.x - 64) / kNodeVecs, j = (threadIdx.x - 64) % kNodeVecs;
        const float4 lk = gld4(rn + kNodeLinks);
        const uint32_t l = __float_as_uint((&lk.x)[k]);
        if (l != kEmptyLinkDev && !(l & kLeafBit)) m.kid[k].v[j] = gld4(base + kNodeStride * static_cast<size_t>(l) + j);
    }
}
// The root and (when the walk descends into an interior child) that child;
// false when the query is already complete (a miss: nothing below was hit).
#ifndef BDPT_ROOT_NF
#define BDPT_ROOT_NF 1  // the LDS root and children through the sign-picked planes too (lds_wnode_nf)
#endif
#if !BDPT_QNODES && BDPT_SLAB_SIGN && BDPT_ROOT_NF
// load_wnode_nf's plane vectors from an LDS copy of a node (the same 16-byte
// vectors at the same offsets: the copy is the record's first 112 bytes)
__device__ __forceinline__ WNode lds_wnode_nf(const WNode& m, f3 inv) {
    const char* b = reinterpret_cast<const char*>(&m);
    const uint32_t sx = plane_sel(inv.x), sy = plane_sel(inv.y), sz = plane_sel(inv.z);
    WNode n;
    n.v[0] = *reinterpret_cast<const float4*>(b + sx);
    n.v[1] = *reinterpret_cast<const float4*>(b + (sx ^ 16u));
    n.v[2] = *reinterpret_cast<const float4*>(b + 32 + sy);
    n.v[3] = *reinterpret_cast<const float4*>(b + 32 + (sy ^ 16u));
    n.v[4] = *reinterpret_cast<const float4*>(b + 64 + sz);
    n.v[5] = *reinterpret_cast<const float4*>(b + 64 + (sz ^ 16u));
    n.v[6] = m.v[6];
    return n;
}
#endif
template <bool COUNT, bool SLACK>
__device__ __forceinline__ bool root_node_vals(const WNode& m, const Ray& r, const RayInv& ri, bool any, TravState& ts,
                                               const Stack& stk, Counts& cnt) {
#if !BDPT_QNODES && BDPT_SLAB_SIGN && BDPT_ROOT_NF
    if (!SLACK) return trav_node_vals<COUNT, false, true>(lds_wnode_nf(m, ri.inv), r, ri, any, ts, stk, cnt);
#endif
    return trav_node_vals<COUNT, SLACK>(m, r, ri, any, ts, stk, cnt);
}
template <bool COUNT, bool SLACK>
__device__ __forceinline__ bool walk_begin_lds(const RootLds& m, const Ray& r, const RayInv& ri, bool any,
                                               TravState& ts, const Stack& stk, Counts& cnt) {
    if (COUNT) cnt.c[8]++;
    bool live = root_node_vals<COUNT, SLACK>(m.root, r, ri, any, ts, stk, cnt);
    if (live && !(ts.link & kLeafBit)) {
        const float4 lk = m.root.v[kNodeLinks];
        const int k = ts.link == __float_as_uint(lk.x) ? 0
                      : ts.link == __float_as_uint(lk.y) ? 1
                      : ts.link == __float_as_uint(lk.z) ? 2 : 3;
        if (COUNT) cnt.c[8]++;
        live = root_node_vals<COUNT, SLACK>(m.kid[k], r, ri, any, ts, stk, cnt) || trav_pop(r, any, ts, stk);
    }
    return live;
}

// One loop iteration (a 4-wide node or a leaf, then the pop). Returns true
// when the query is complete (result in ts.best / best_t / best_u / best_v).
template <bool COUNT, bool SLACK = true>
__device__ __forceinline__ bool trav_step(const TravScene& sc, const Ray& r, const RayInv& ri, bool any, TravState& ts,
                                          const Stack& stk, Counts& cnt) {
    if (COUNT) {
        cnt.c[8]++;
        if (first_active_lane()) cnt.c[9]++;
    }
    if (ts.link & kLeafBit) {
        if (wleaf_tests<COUNT>(sc.wtri, sc.lbox, ts.link, r, ri, any, ts.best_t, ts.best, ts.best_u, ts.best_v, cnt))
            return true;
    } else if (trav_node<COUNT, SLACK>(sc, r, ri, any, ts, stk, cnt)) {
        return false;
    }
    return !trav_pop(r, any, ts, stk, COUNT ? &cnt.c[19] : nullptr);
}

// The same walk as a while-while loop (Aila & Laine 2009): lanes descend
// through interior nodes together until each holds a leaf (or is done), then
// the leaves are tested together — a wave iteration runs one kind of work.
template <bool COUNT>
__device__ __forceinline__ void trav_while_while(const TravScene& sc, const Ray& r, const RayInv& ri, bool any,
                                                 TravState& ts, const Stack& stk, Counts& cnt) {
    for (;;) {
        bool live = true;
        while (!(ts.link & kLeafBit)) {
            if (COUNT) {
                cnt.c[8]++;
                if (first_active_lane()) cnt.c[9]++;
            }
            if (!trav_node<COUNT, true>(sc, r, ri, any, ts, stk, cnt) && !trav_pop(r, any, ts, stk)) {
                live = false;
                break;
            }
        }
        if (!live) return;
        if (COUNT) {
            cnt.c[8]++;
            if (first_active_lane()) cnt.c[9]++;
        }
        if (wleaf_tests<COUNT>(sc.wtri, sc.lbox, ts.link, r, ri, any, ts.best_t, ts.best, ts.best_u, ts.best_v, cnt))
            return;
        if (!trav_pop(r, any, ts, stk)) return;
    }
}

template <bool FULL, bool COUNT>
__device__ __forceinline__ int traverse(const DevScene& sc, const Ray& r, bool any, const Stack& stk, float& bt,
                                        float& bu, float& bv, Counts& cnt, float near = kNoCullNear) {
    if (r.min_t > r.max_t) return -1;  // the root's entry mint is min_t (bvh.h:277, :287)
    const RayInv ri = ray_inv(r, near);
    if (FULL || !ri.fast || far_origin(sc, r.o)) {  // the reference's tree, unculled
        const TravResult q = traverse_binary<COUNT, Stack>(sc, r, any, false, stk);
        if (COUNT) cnt.c[2] += q.nodes, cnt.c[3] += q.tris, cnt.c[15] += q.exact;
        bt = q.t, bu = q.u, bv = q.v;
        return q.best;
    }
    const TravScene tsc = trav_scene(sc);
    TravState ts = trav_begin(tsc, r);
#if BDPT_TRAV_WHILE_WHILE
    trav_while_while<COUNT>(tsc, r, ri, any, ts, stk, cnt);
#else
    if (tsc.node_slack) {  // a query-level (uniform) choice: the node step itself has no branch on it
        while (!trav_step<COUNT, true>(tsc, r, ri, any, ts, stk, cnt)) {
        }
    } else {
        while (!trav_step<COUNT, false>(tsc, r, ri, any, ts, stk, cnt)) {
        }
    }
#endif
    bt = ts.best_t, bu = ts.best_u, bv = ts.best_v;
    return ts.best;
}

// The closest hit of ONE ray (the same in every lane of the wave) walked by the
// whole wave: each round pops up to 64 pending entries (one per lane) from an
// LDS stack, tests them (a 4-wide node: node_child_keys; a leaf: wleaf_tests
// against the best so far), takes the lexicographic minimum (t, reference
// index) over the lanes and pushes the children far-first. The result is the
// serial walk's: the minimum over the candidates of every entry the walk cannot
// cull (the same conservative per-entry tests, cull_far of the best so far), ties
// to the lowest reference index, accepted only below r.max_t — the order the
// entries are visited in does not enter it. For the Russian-roulette
// continuation pass (bdpt_kernels.hip, chain kernel): a trapped subpath's walk
// takes ~9 rounds instead of ~30 dependent steps. `stack` holds `cap` entries;
// false if they did not suffice (the caller reports it). With bound < r.max_t
// only candidates below `bound` are accepted (and entries beyond it culled): a
// hit found is then the same result — the minimum over all candidates lies below
// it — and none found (best -1) means the walk must be repeated unbounded.
__device__ __forceinline__ uint64_t coop_key(float t, int idx) {
    const uint32_t b = __float_as_uint(t);
    const uint32_t o = (b & 0x80000000u) ? ~b : (b | 0x80000000u);  // float order as unsigned order
    return (static_cast<uint64_t>(o) << 32) | static_cast<uint32_t>(idx);
}
// A leaf of up to 4 triangles (the triangle tree's kTriLeafMax) for coop_closest:
// every triangle's loads issued before the first test (wleaf_tests' loop waits
// for each triangle in turn); the same acceptance rule, so the same minimum.
__device__ __forceinline__ void coop_leaf(const TravScene& sc, uint32_t link, const Ray& r, const RayInv& ri, float& bt,
                                          int& bb, float& bu, float& bv) {
    const uint32_t start = (link >> 3) & 0x0fffffffu, count = link & 7u;
    Counts cnt;  // (not a counting pass)
    if (count > 4) {
        wleaf_tests<false>(sc.wtri, sc.lbox, link, r, ri, false, bt, bb, bu, bv, cnt);
        return;
    }
    float4 q[4][3];
#pragma unroll
    for (uint32_t k = 0; k < 4; k++)
        if (k < count) {
            const float4* p = sc.wtri + 3 * static_cast<size_t>(start + k);
            q[k][0] = gld4(p), q[k][1] = gld4(p + 1), q[k][2] = gld4(p + 2);
        }
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
        if (k >= count) break;
        float t, u, v;
        if (!tri_test_edges(xyz(q[k][0]), xyz(q[k][1]), xyz(q[k][2]), r, t, u, v)) continue;
        const int idx = __float_as_int(q[k][0].w);
        if ((t < bt || (t == bt && bb >= 0 && idx < bb)) &&
            ref_leaf_passes<false>(sc.lbox, __float_as_uint(q[k][1].w), r, ri, cnt))
            bt = t, bb = idx, bu = u, bv = v;
    }
}

// The walk's LDS stack: entry e at base[e] (a wave's own array), or spread over
// the columns a wave's lanes own in a block's per-lane stack (entry e at
// base[(e / 64) * stride + e % 64], base = the wave's first lane).
typedef __attribute__((address_space(3))) u32x2 coop_lds_e;
struct CoopStack {
    uint2* base;
    int stride;  // 0: contiguous
    __device__ __forceinline__ coop_lds_e* at(int e) const {
        return (coop_lds_e*)base + (stride ? (e >> 6) * stride + (e & 63) : e);
    }
};
// A node of a cooperative walk: from the block's LDS copy when it is the root or
// one of its interior children (RootLds; rl non-null), else from HBM. The
// trapped glass chains' walks start at the root, so their first two rounds read
// LDS instead of waiting on two dependent loads (BDPT_COOP_ROOT_LDS).
struct RootLds;
__device__ __forceinline__ WNode coop_node(const TravScene& sc, uint32_t link, const RootLds* rl);
#ifndef BDPT_COOP_CP
#define BDPT_COOP_CP 1  // coop_closest walks 16 entries per round, one child box / leaf triangle per lane (coop_closest_cp)
#endif
#if BDPT_COOP_CP && !BDPT_QNODES
// coop_closest with the work of an entry spread over 4 lanes: each round pops up
// to 16 entries, and lane 4s + c takes child c of entry s (its six planes and its
// link: seven dword loads instead of the node's seven 16-byte vectors) or the
// leaf's triangles c, c + 4 — one box or triangle test per lane where the
// 64-entry round ran four box tests, a sort and up to four triangle tests in every
// busy lane. A lone walk's frontier rarely holds more than 16 entries, and a
// round of one wave alone on its SIMD costs its instructions, not its loads. The
// per-child test is node_child_keys' (slab_fast with the slack, slab_fma without;
// the same culls), the per-triangle acceptance coop_leaf's, so the result is the
// same minimum (t, index) over the same candidates; entries are pushed unsorted
// (the visiting order does not enter the result).
// A lane's share of a cooperative walk's entry `link` (coop_closest_cp): child c
// of an interior node — node_child_keys' test of that child, its entry distance
// and link in (key, lnk) when the walk must visit it — or triangles c, c + 4 of a
// leaf, with coop_leaf's acceptance rule against (lt, lb).
template <bool SLACK>
__device__ __forceinline__ void coop_entry_cp(const TravScene& sc, const Ray& r, const RayInv& ri, f3 oi, float far,
                                              uint32_t link, int c, float& lt, int& lb, float& lu, float& lv,
                                              float& key, uint32_t& lnk) {
    if (link & kLeafBit) {
        const uint32_t start = (link >> 3) & 0x0fffffffu, count = link & 7u;
        Counts cnt;  // (not a counting pass)
        for (uint32_t j = static_cast<uint32_t>(c); j < count; j += 4) {
            const float4* p = sc.wtri + 3 * static_cast<size_t>(start + j);
            const float4 q0 = gld4(p), q1 = gld4(p + 1), q2 = gld4(p + 2);
            float t, u, v;
            if (!tri_test_edges(xyz(q0), xyz(q1), xyz(q2), r, t, u, v)) continue;
            const int idx = __float_as_int(q0.w);
            if ((t < lt || (t == lt && lb >= 0 && idx < lb)) &&
                ref_leaf_passes<false>(sc.lbox, __float_as_uint(q1.w), r, ri, cnt))
                lt = t, lb = idx, lu = u, lv = v;
        }
    } else {
        // child c of the 128-byte record: lo.x hi.x lo.y hi.y lo.z hi.z links, four floats each
        const float* nd = reinterpret_cast<const float*>(sc.wnodes + kNodeStride * static_cast<size_t>(link)) + c;
        const float clx = gld1(nd), chx = gld1(nd + 4), cly = gld1(nd + 8), chy = gld1(nd + 12), clz = gld1(nd + 16),
                    chz = gld1(nd + 20);
        const uint32_t l = __float_as_uint(gld1(nd + 24));
        float tn, tf;
        int d = kSlabHit;
        if (SLACK || !BDPT_SLAB_FMA) d = slab_fast(clx, cly, clz, chx, chy, chz, r.o, ri.inv, tn, tf);
        else slab_fma(clx, cly, clz, chx, chy, chz, oi, ri.inv, tn, tf);
        const bool pass = SLACK ? d != kSlabMiss : !(tn > tf);
        if (l != kEmptyLinkDev && pass && !(tn > far) && !(tf < ri.near)) key = tn, lnk = l;
    }
}
#ifndef BDPT_COOP_CP_CALL
#define BDPT_COOP_CP_CALL 0  // 1: coop_closest_cp out of line (its registers not part of the caller's allocation)
#endif
#if BDPT_COOP_CP_CALL
#define BDPT_COOP_CP_INLINE __noinline__
#else
#define BDPT_COOP_CP_INLINE __forceinline__
#endif
template <bool SLACK>
__device__ BDPT_COOP_CP_INLINE bool coop_closest_cp(const TravScene& sc, const Ray& r, const RayInv& ri, float bound,
                                                CoopStack stk, int cap, float& best_t, int& best, float& best_u,
                                                float& best_v, uint32_t* rounds) {
    const uint32_t lane = __lane_id();
    const int slot = static_cast<int>(lane >> 2), c = static_cast<int>(lane & 3u);
    const f3 oi = SLACK || !BDPT_SLAB_FMA ? mk(0.f, 0.f, 0.f) : slab_fma_origin(r.o, ri.inv);
    best_t = bound < r.max_t ? bound : r.max_t, best = -1, best_u = best_v = 0.f;
    if (lane == 0) *stk.at(0) = u32x2{sc.wroot_link, __float_as_uint(-__builtin_inff())};
    int sp = 1;
    bool ok = true;
    while (sp > 0) {
        if (rounds) (*rounds)++;
        const int k = sp < 16 ? sp : 16;
        u32x2 e = {kEmptyLinkDev, 0u};
        if (slot < k) e = *stk.at(sp - k + slot);
        sp -= k;
        const float far = cull_far(best_t);
        const bool live = e.x != kEmptyLinkDev && !(__uint_as_float(e.y) > far);
        float lt = best_t, lu = best_u, lv = best_v;
        int lb = best;
        float key = __builtin_inff();
        uint32_t lnk = kEmptyLinkDev;
        if (live) coop_entry_cp<SLACK>(sc, r, ri, oi, far, e.x, c, lt, lb, lu, lv, key, lnk);
        // the wave's lexicographic minimum of (t, index) over the lanes that found a better hit
        uint64_t imp = __ballot(lb != best);
        if (imp) {
            uint64_t m = ~0ull;
            int w = 0;
            while (imp) {
                const int i = __ffsll(static_cast<unsigned long long>(imp)) - 1;
                imp &= imp - 1;
                const uint64_t ki = coop_key(lane_val(lt, i), lane_val(lb, i));
                if (ki < m) m = ki, w = i;
            }
            best_t = lane_val(lt, w), best = lane_val(lb, w), best_u = lane_val(lu, w), best_v = lane_val(lv, w);
        }
        const uint64_t has = __ballot(lnk != kEmptyLinkDev);
        const int n = popc64(has);
        if (sp + n > cap) {
            ok = false;
        } else {
            if (lnk != kEmptyLinkDev) *stk.at(sp + lanes_below(has)) = u32x2{lnk, __float_as_uint(key)};
            sp += n;
        }
    }
    return ok;
}
#endif

// BATCH: coop_leaf (a leaf's triangle loads issued together, 48 more live
// registers) rather than wleaf_tests.
template <bool SLACK, bool BATCH = true>
__device__ __forceinline__ bool coop_closest(const TravScene& sc, const Ray& r, const RayInv& ri, float bound,
                                             CoopStack stk, int cap, float& best_t, int& best, float& best_u,
                                             float& best_v, uint32_t* rounds = nullptr, const RootLds* rl = nullptr) {
#if BDPT_COOP_CP && !BDPT_QNODES
    (void)rl;  // (the block's LDS copy of the root: not read by the 4-lane entries)
    return coop_closest_cp<SLACK>(sc, r, ri, bound, stk, cap, best_t, best, best_u, best_v, rounds);
#endif
    const uint32_t lane = __lane_id();
    best_t = bound < r.max_t ? bound : r.max_t, best = -1, best_u = best_v = 0.f;
    if (lane == 0) *stk.at(0) = u32x2{sc.wroot_link, __float_as_uint(-__builtin_inff())};
    int sp = 1;
    bool ok = true;
    while (sp > 0) {
        if (rounds) (*rounds)++;
        const int k = sp < 64 ? sp : 64;
        u32x2 e = {kEmptyLinkDev, 0u};
        if (static_cast<int>(lane) < k) e = *stk.at(sp - k + static_cast<int>(lane));
        sp -= k;
        const float far = cull_far(best_t);
        const bool live = e.x != kEmptyLinkDev && !(__uint_as_float(e.y) > far);
        float lt = best_t, lu = best_u, lv = best_v;
        int lb = best;
        float key[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
        uint32_t lnk[4] = {kEmptyLinkDev, kEmptyLinkDev, kEmptyLinkDev, kEmptyLinkDev};
        if (live) {
            if (e.x & kLeafBit) {
                if (BATCH) {
                    coop_leaf(sc, e.x, r, ri, lt, lb, lu, lv);
                } else {
                    Counts cnt;  // (not a counting pass)
                    wleaf_tests<false>(sc.wtri, sc.lbox, e.x, r, ri, false, lt, lb, lu, lv, cnt);
                }
            }
            else node_child_keys<SLACK>(coop_node(sc, e.x, rl), r, ri, far, key, lnk);
        }
        // the wave's lexicographic minimum of (t, index) over the lanes that found
        // a better hit (usually none or one): a scalar loop over their keys
        uint64_t imp = __ballot(lb != best);
        if (imp) {
            uint64_t m = ~0ull;
            int w = 0;
            while (imp) {
                const int i = __ffsll(static_cast<unsigned long long>(imp)) - 1;
                imp &= imp - 1;
                const uint64_t ki = coop_key(lane_val(lt, i), lane_val(lb, i));
                if (ki < m) m = ki, w = i;
            }
            best_t = lane_val(lt, w), best = lane_val(lb, w), best_u = lane_val(lu, w), best_v = lane_val(lv, w);
        }
        // children far-first, so the nearest are popped first
#pragma unroll
        for (int c = 3; c >= 0; c--) {
            const uint64_t has = __ballot(lnk[c] != kEmptyLinkDev);
            const int pos = sp + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                     static_cast<uint32_t>(has >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(has), 0u)));
            const int n = popc64(has);
            if (sp + n > cap) {
                ok = false;
            } else if (lnk[c] != kEmptyLinkDev) {
                *stk.at(pos) = u32x2{lnk[c], __float_as_uint(key[c])};
            }
            if (sp + n <= cap) sp += n;
        }
    }
    return ok;
}

// coop_closest for up to four rays at once: the wave split into 64 / G groups
// of G lanes (G = 32 or 16), group g walking its own ray on its own range
// [base, base + cap) of the stack entries; inactive groups idle. Each group's
// result is coop_closest's for its ray (the same per-entry tests, the minimum
// (t, index) over the group's candidates); false for a group whose entries did
// not fit. For the Russian-roulette build's express waves holding 2-4 long walks,
// which otherwise take turns with all 64 lanes.
#ifndef BDPT_COOP_GROUPS_CP
#define BDPT_COOP_GROUPS_CP 1  // coop_closest_groups with coop_closest_cp's 4 lanes per entry (G / 4 entries per round)
#endif
#if BDPT_COOP_CP && BDPT_COOP_GROUPS_CP && !BDPT_QNODES
// coop_closest_groups in coop_closest_cp's layout: group g's lane 4s + c takes child
// c (or triangles c, c + 4) of the group's entry s, G / 4 entries per round; the
// same per-entry tests and per-group minimum, so each group's result is
// coop_closest's for its ray.
template <bool SLACK>
__device__ __forceinline__ bool coop_closest_groups_cp(const TravScene& sc, const Ray& r, const RayInv& ri,
                                                       float bound, bool active, CoopStack stk, int base, int cap,
                                                       int G, float& best_t, int& best, float& best_u, float& best_v) {
    const uint32_t lane = __lane_id();
    const int gl = static_cast<int>(lane) & (G - 1);
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (static_cast<int>(lane) - gl);
    const int slot = gl >> 2, c = gl & 3, per = G >> 2;
    const f3 oi = SLACK || !BDPT_SLAB_FMA ? mk(0.f, 0.f, 0.f) : slab_fma_origin(r.o, ri.inv);
    best_t = bound < r.max_t ? bound : r.max_t, best = -1, best_u = best_v = 0.f;
    if (active && gl == 0) *stk.at(base) = u32x2{sc.wroot_link, __float_as_uint(-__builtin_inff())};
    int sp = active ? 1 : 0;
    bool ok = true;
    while (__ballot(sp > 0)) {
        const int k = sp < per ? sp : per;
        u32x2 e = {kEmptyLinkDev, 0u};
        if (slot < k) e = *stk.at(base + sp - k + slot);
        sp -= k;
        const float far = cull_far(best_t);
        const bool live = e.x != kEmptyLinkDev && !(__uint_as_float(e.y) > far);
        float lt = best_t, lu = best_u, lv = best_v;
        int lb = best;
        float key = __builtin_inff();
        uint32_t lnk = kEmptyLinkDev;
        if (live) coop_entry_cp<SLACK>(sc, r, ri, oi, far, e.x, c, lt, lb, lu, lv, key, lnk);
        // each group's lexicographic minimum of (t, index) over its improving lanes
        uint64_t imp = __ballot(lb != best);
        if (imp) {
            uint64_t m = ~0ull;
            int w = static_cast<int>(lane);
            while (imp) {
                const int i = __ffsll(static_cast<unsigned long long>(imp)) - 1;
                imp &= imp - 1;
                const uint64_t ki = coop_key(lane_val(lt, i), lane_val(lb, i));
                if ((gmask >> i) & 1ull && ki < m) m = ki, w = i;
            }
            best_t = __shfl(lt, w), best = __shfl(lb, w), best_u = __shfl(lu, w), best_v = __shfl(lv, w);
        }
        const uint64_t has = __ballot(lnk != kEmptyLinkDev) & gmask;
        const int n = popc64(has);
        if (sp + n > cap) {
            ok = false;
        } else {
            if (lnk != kEmptyLinkDev) *stk.at(base + sp + lanes_below(has)) = u32x2{lnk, __float_as_uint(key)};
            sp += n;
        }
    }
    return ok;
}
#endif
template <bool SLACK>
__device__ __forceinline__ bool coop_closest_groups(const TravScene& sc, const Ray& r, const RayInv& ri, float bound,
                                                    bool active, CoopStack stk, int base, int cap, int G,
                                                    float& best_t, int& best, float& best_u, float& best_v,
                                                    const RootLds* rl = nullptr) {
#if BDPT_COOP_CP && BDPT_COOP_GROUPS_CP && !BDPT_QNODES
    (void)rl;
    return coop_closest_groups_cp<SLACK>(sc, r, ri, bound, active, stk, base, cap, G, best_t, best, best_u, best_v);
#endif
    const uint32_t lane = __lane_id();
    const int gl = static_cast<int>(lane) & (G - 1);
    const uint64_t gmask = (G == 64 ? ~0ull : ((1ull << G) - 1ull)) << (static_cast<int>(lane) - gl);
    best_t = bound < r.max_t ? bound : r.max_t, best = -1, best_u = best_v = 0.f;
    if (active && gl == 0) *stk.at(base) = u32x2{sc.wroot_link, __float_as_uint(-__builtin_inff())};
    int sp = active ? 1 : 0;
    bool ok = true;
    while (__ballot(sp > 0)) {
        const int k = sp < G ? sp : G;
        u32x2 e = {kEmptyLinkDev, 0u};
        if (gl < k) e = *stk.at(base + sp - k + gl);
        sp -= k;
        const float far = cull_far(best_t);
        const bool live = e.x != kEmptyLinkDev && !(__uint_as_float(e.y) > far);
        float lt = best_t, lu = best_u, lv = best_v;
        int lb = best;
        float key[4] = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
        uint32_t lnk[4] = {kEmptyLinkDev, kEmptyLinkDev, kEmptyLinkDev, kEmptyLinkDev};
        if (live) {
            if (e.x & kLeafBit) {
                Counts cnt;  // (not a counting pass)
                wleaf_tests<false>(sc.wtri, sc.lbox, e.x, r, ri, false, lt, lb, lu, lv, cnt);
            } else {
                node_child_keys<SLACK>(coop_node(sc, e.x, rl), r, ri, far, key, lnk);
            }
        }
        // each group's lexicographic minimum of (t, index) over its improving lanes
        uint64_t imp = __ballot(lb != best);
        if (imp) {
            uint64_t m = ~0ull;
            int w = static_cast<int>(lane);
            while (imp) {
                const int i = __ffsll(static_cast<unsigned long long>(imp)) - 1;
                imp &= imp - 1;
                const uint64_t ki = coop_key(lane_val(lt, i), lane_val(lb, i));
                if ((gmask >> i) & 1ull && ki < m) m = ki, w = i;
            }
            best_t = __shfl(lt, w), best = __shfl(lb, w), best_u = __shfl(lu, w), best_v = __shfl(lv, w);
        }
        // children far-first, each group on its own range
#pragma unroll
        for (int c = 3; c >= 0; c--) {
            const uint64_t has = __ballot(lnk[c] != kEmptyLinkDev) & gmask;
            const int pos = sp + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                     static_cast<uint32_t>(has >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(has), 0u)));
            const int n = popc64(has);
            if (sp + n > cap) {
                ok = false;
            } else if (lnk[c] != kEmptyLinkDev) {
                *stk.at(base + pos) = u32x2{lnk[c], __float_as_uint(key[c])};
            }
            if (sp + n <= cap) sp += n;
        }
    }
    return ok;
}

// AcceleratorBVH::intersect's shading of a closest hit (accel.h:133-166).
__device__ __forceinline__ void shade_hit(const DevScene& sc, int i, float u, float v, float t, f3 dir, Hit& h) {
    const float4* sh = sc.shade + kShadeStride * static_cast<size_t>(i);
    const f3 v0 = xyz(gld4(BDPT_SHADE_WIDE ? sh + kShadeV0 : sc.tri + 3 * static_cast<size_t>(i))),
             v1 = xyz(gld4(sh + 3)), v2 = xyz(gld4(sh + 4));
    const float4 s0 = gld4(sh), s1 = gld4(sh + 1), s2 = gld4(sh + 2);
    const float w = 1 - u - v;
    h.p = (v0 * w + v1 * u) + v2 * v;
    h.n = normalize((xyz(s0) * w + xyz(s1) * u) + xyz(s2) * v);
    f3 fs, ft;
    make_frame(h.n, fs, ft);
    h.wo = to_local(fs, ft, h.n, -dir);
    h.dist = t;
    h.mat = __float_as_int(s0.w);
    h.shape = __float_as_int(s1.w);
}

// The shadow ray of visibilityQuery (bdpt.h:498-505).
__device__ __forceinline__ Ray shadow_ray(f3 start, f3 end) {
    f3 dir = end - start;
    const float dist = sqrt_cr(dot(dir, dir));
    dir = dir / dist;
    return Ray{start, dir, kEpsilon, dist - 0.00001f};
}

// -------------------------------------------------------------------- BSDFs
__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }

#ifndef BDPT_GLOSSY_ATTR
#define BDPT_GLOSSY_ATTR __forceinline__  // the Phong-bearing eval / pdf (measured: inline +2 %)
#endif
#ifndef BDPT_EVAL_PDFS
#define BDPT_EVAL_PDFS 1  // 0: eval and the two pdfs through separate calls (round 2: 195.9 vs 190.8 for 1; round 3 without SLP: 245.2 vs 250.0)
#endif
#ifndef BDPT_GLASS_INLINE
#define BDPT_GLASS_INLINE 1  // the delta lobes' samplers inline, the Phong-bearing ones out of line (+1.1 %)
#endif
#ifndef BDPT_SAMPLE_ATTR
#define BDPT_SAMPLE_ATTR BDPT_NOINLINE  // the non-diffuse BSDF samplers out of line
#endif
// MixtureBSDF::eval == PhongBSDF::eval (mixture.h:59-75, phong.h:56-71).
// With Ks == 0 the specular term is (0 * (n + 2)) * INV_TWOPI * powf(c, n) = +0
// (powf of c in [0, 1] is finite), and val + 0 == val: skipping it is exact.
template <bool EXACT = false>
__device__ __forceinline__ f3 glossy_eval(const BsdfRecord& b, f3 wi, f3 wo) {
    f3 val = mk(0.f, 0.f, 0.f);
    if (wi.z >= 0.f && wo.z >= 0.f) {
        val = val + ld3(b.kd) * kInvPi;
        if (b.ks[0] != 0.f || b.ks[1] != 0.f || b.ks[2] != 0.f) {
            const float ex = b.exponent;
            const float c = glibc_fminf(glibc_fmaxf(dot(wi, reflect_z(wo)), 0.f), 1.f);
            val = val + ((ld3(b.ks) * (ex + 2)) * kInvTwoPi) * (EXACT ? glibc_powf(c, ex) : pow_w(c, ex));
        }
        val = val * b.scale;
        val = val * wi.z;
    }
    return val;
}

__device__ BDPT_GLOSSY_ATTR f3 glossy_eval_call(const BsdfRecord& b, f3 wi, f3 wo) { return glossy_eval(b, wi, wo); }

// BSDF::eval. The diffuse and delta lobes are a few instructions and stay
// inline; only the Phong-bearing lobes (powf) go through a call.
__device__ __forceinline__ f3 bsdf_eval(const BsdfRecord& b, f3 wi, f3 wo) {
    const int kind = b.kind;
    if (kind == BSDF_DIFFUSE) {  // diffuse.h:35-43
        if (wi.z >= 0.f && wo.z >= 0.f) return (ld3(b.kd) * kInvPi) * wi.z;
        return mk(0.f, 0.f, 0.f);
    }
    if (kind == BSDF_MIXTURE || kind == BSDF_PHONG) return glossy_eval_call(b, wi, wo);
    return mk(0.f, 0.f, 0.f);  // delta lobes (perfectmirror.h:41-47, glass.h:55-59)
}

template <bool EXACT = false>
__device__ __forceinline__ float phong_part_pdf(const BsdfRecord& b, f3 wi, f3 wo) {
    f3 rs, rt;
    const f3 rn = reflect_z(wo);
    make_frame(rn, rs, rt);
    return phong_lobe_pdf<EXACT>(to_local(rs, rt, rn, wi), b.exponent);
}

// With specw == 0, pdfPhong * 0 = +0 (pdfPhong is finite and >= 0) and
// 0 + pdfDiffuse * (1 - 0) == pdfDiffuse: skipping the Phong lobe is exact.
__device__ BDPT_GLOSSY_ATTR float glossy_pdf_call(const BsdfRecord& b, f3 wi, f3 wo) {
    if (b.kind == BSDF_MIXTURE) {  // mixture.h:78-100
        const float pd = cosine_hemisphere_pdf(wi);
        const float pp = phong_part_pdf(b, wi, wo);
        return (pp * b.specw) + (pd * (1.f - b.specw));
    }
    return phong_part_pdf(b, wi, wo);  // phong.h:73-83
}
__device__ __forceinline__ float bsdf_pdf(const BsdfRecord& b, f3 wi, f3 wo) {
    const int kind = b.kind;
    if (kind == BSDF_DIFFUSE || (kind == BSDF_MIXTURE && b.specw == 0.f))  // diffuse.h:45-50
        return cosine_hemisphere_pdf(wi);
    if (kind == BSDF_MIXTURE || kind == BSDF_PHONG) return glossy_pdf_call(b, wi, wo);
    return 0.f;
}

// eval(wi, wo), pdf(wi, wo) and pdf(wo, wi) of one BSDF — what every
// connection needs at each end (bdpt.h:374-483) — with ONE powf for the Phong
// lobe: the cosine of eval (dot(wi, reflect(wo)), clamped to [0, 1]) and the
// lobe's local z in both pdfs (Frame(reflect(wo)).toLocal(wi).z = dot(wi,
// reflect(wo)), and dot(wo, reflect(wi)) has the same products in the same
// order) are one value z. eval takes powf(clamp(z)), the pdfs powf(z) for
// z >= 0: the same call unless z > 1, where eval's powf(1, n) is exactly 1.
// Each output is bit-identical to bsdf_eval / bsdf_pdf above.
struct EvalPdfs {
    f3 f;
    float fwd, rev;  // pdf(wi, wo), pdf(wo, wi)
};
__device__ __forceinline__ EvalPdfs bsdf_eval_pdfs(const BsdfRecord& b, f3 wi, f3 wo) {
#if BDPT_EVAL_PDFS
    EvalPdfs r{mk(0.f, 0.f, 0.f), 0.f, 0.f};
    const int kind = b.kind;
    if (kind == BSDF_DIFFUSE) {
        if (wi.z >= 0.f && wo.z >= 0.f) r.f = (ld3(b.kd) * kInvPi) * wi.z;
        r.fwd = cosine_hemisphere_pdf(wi);
        r.rev = cosine_hemisphere_pdf(wo);
        return r;
    }
    if (kind != BSDF_MIXTURE && kind != BSDF_PHONG) return r;  // delta lobes
    const float ex = b.exponent;
    const float z = dot(wi, reflect_z(wo));
    const bool eval_on = wi.z >= 0.f && wo.z >= 0.f;
    const bool ks_on = b.ks[0] != 0.f || b.ks[1] != 0.f || b.ks[2] != 0.f;
    const bool lobe_pdf = kind == BSDF_PHONG || b.specw != 0.f;
    float pw = 0.f;
    if ((eval_on && ks_on) || (lobe_pdf && z >= 0.f))
        pw = pow_w(z > 1.f ? z : glibc_fminf(glibc_fmaxf(z, 0.f), 1.f), ex);
    if (eval_on) {  // glossy_eval
        f3 val = mk(0.f, 0.f, 0.f);
        val = val + ld3(b.kd) * kInvPi;
        if (ks_on) val = val + ((ld3(b.ks) * (ex + 2)) * kInvTwoPi) * (z > 1.f ? 1.f : pw);
        val = val * b.scale;
        r.f = val * wi.z;
    }
    const float pp = z >= 0.f ? (ex + 2) * kInvTwoPi * pw : 0.f;  // phong_lobe_pdf
    if (kind == BSDF_PHONG) {
        r.fwd = r.rev = pp;
    } else if (b.specw == 0.f) {
        r.fwd = cosine_hemisphere_pdf(wi);
        r.rev = cosine_hemisphere_pdf(wo);
    } else {
        r.fwd = (pp * b.specw) + (cosine_hemisphere_pdf(wi) * (1.f - b.specw));
        r.rev = (pp * b.specw) + (cosine_hemisphere_pdf(wo) * (1.f - b.specw));
    }
    return r;
#else
    return EvalPdfs{bsdf_eval(b, wi, wo), bsdf_pdf(b, wi, wo), bsdf_pdf(b, wo, wi)};
#endif
}

// glass.h:40-53
__device__ __forceinline__ float fresnel_dielectric(float eta_i, float eta_t, float cos_i, float cos_t) {
    const float eta = div_cr(eta_i, eta_t);
    const float sin2_t = eta * eta * (glibc_fmaxf(0.f, 1.f - cos_i * cos_i));
    if (sin2_t >= 1.f) return 1.f;
    const float rpar = div_cr((eta_t * cos_i) - (eta_i * cos_t), (eta_t * cos_i) + (eta_i * cos_t));
    const float rper = div_cr((eta_i * cos_i) - (eta_t * cos_t), (eta_i * cos_i) + (eta_t * cos_t));
    return (rpar * rpar + rper * rper) * 0.5f;
}

// GlassBSDF::sample (glass.h:67-108: pdf 1, no eta^2 scaling).
__device__ __forceinline__ f3 glass_sample(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
    pdf = 1.f;
    const bool entering = wo.z > 0.f;
    float eta_i = 1.f, eta_t = b.ior;
    if (!entering) {
        const float q = eta_i;
        eta_i = eta_t;
        eta_t = q;
    }
    const float eta = div_cr(eta_i, eta_t);
    const float sin2_i = glibc_fmaxf(0.f, 1.f - wo.z * wo.z);
    const float sin2_t = eta * eta * sin2_i;
    float cos_t = sqrt_cr(glibc_fmaxf(0.f, 1.f - sin2_t));
    cos_t = entering ? -cos_t : cos_t;
    const float fr = fresnel_dielectric(eta_i, eta_t, fabsf(wo.z), fabsf(cos_t));
    if (u.x < fr) {
        wi = reflect_z(wo);
        return mk(1.f, 1.f, 1.f);
    }
    wi = mk(eta * -wo.x, eta * -wo.y, cos_t);
    return ld3(b.tf);
}

// BSDF::sample: sets wi, returns f*cos, writes the solid-angle pdf.
#ifndef BDPT_SAMPLE_STRUCT
#define BDPT_SAMPLE_STRUCT 1
#endif
#if BDPT_SAMPLE_STRUCT
__device__ __forceinline__ f3 bsdf_sample_body(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
#else
__device__ BDPT_NOINLINE f3 bsdf_sample_call(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
#endif
    switch (b.kind) {
        case BSDF_MIRROR:  // perfectmirror.h:49-59
            pdf = 1.f;
            wi = reflect_z(wo);
            return mk(1.f, 1.f, 1.f);
        case BSDF_GLASS:
            return glass_sample(b, wo, u, wi, pdf);
        // The sampled value steers the walk (ContinuePathRandomWalk ends it on f == 0,
        // bdpt.h:253), so the Phong powers here stay glibc's powf in every build: the
        // fast-weight pow_w flushes results below 2^-126 to 0, which for a
        // lobe with Kd = 0 would end a path the reference continues.
        case BSDF_MIXTURE: {  // mixture.h:102-151
            f3 val;
            if (u.x < b.specw) {
                const F2 ns{div_cr(u.x, b.specw), u.y};
                f3 rs, rt;
                const f3 rn = reflect_z(wo);
                make_frame(rn, rs, rt);
                wi = to_world(rs, rt, rn, phong_lobe(ns, b.exponent));
            } else {
                const F2 ns{div_cr(u.x - b.specw, 1.f - b.specw), u.y};
                wi = cosine_hemisphere(ns);
            }
            val = glossy_eval<true>(b, wi, wo);
            if (b.specw == 0.f) pdf = cosine_hemisphere_pdf(wi);  // bsdf_pdf's exact shortcut
            else pdf = (phong_part_pdf<true>(b, wi, wo) * b.specw) + (cosine_hemisphere_pdf(wi) * (1.f - b.specw));
            return val;
        }
        case BSDF_PHONG: {  // phong.h:85-100
            f3 rs, rt;
            const f3 rn = reflect_z(wo);
            make_frame(rn, rs, rt);
            const f3 ls = phong_lobe(u, b.exponent);
            pdf = phong_lobe_pdf<true>(ls, b.exponent);
            wi = to_world(rs, rt, rn, ls);
            return glossy_eval<true>(b, wi, wo);
        }
        default:  // null BSDF (illum 5): the reference dereferences nullptr
            pdf = 0.f;
            wi = mk(0.f, 0.f, 0.f);
            return mk(0.f, 0.f, 0.f);
    }
}
#if BDPT_SAMPLE_STRUCT
// The call returns everything by value (in VGPRs): with reference outputs the
// caller's wi / pdf went through scratch around every call.
struct BsdfSample {
    f3 f, wi;
    float pdf;
};
__device__ BDPT_SAMPLE_ATTR BsdfSample bsdf_sample_call(const BsdfRecord& b, f3 wo, F2 u) {
    BsdfSample s;
    s.f = bsdf_sample_body(b, wo, u, s.wi, s.pdf);
    return s;
}
__device__ __forceinline__ f3 bsdf_sample_call(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
    const BsdfSample s = bsdf_sample_call(b, wo, u);
    wi = s.wi;
    pdf = s.pdf;
    return s.f;
}
#endif
__device__ __forceinline__ f3 bsdf_sample(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
    if (b.kind == BSDF_DIFFUSE) {  // diffuse.h:52-61
        wi = cosine_hemisphere(u);
        pdf = cosine_hemisphere_pdf(wi);
        return bsdf_eval(b, wi, wo);
    }
#if BDPT_GLASS_INLINE
    if (b.kind == BSDF_GLASS) return glass_sample(b, wo, u, wi, pdf);
    if (b.kind == BSDF_MIRROR) {  // perfectmirror.h:49-59
        pdf = 1.f;
        wi = reflect_z(wo);
        return mk(1.f, 1.f, 1.f);
    }
#endif
    return bsdf_sample_call(b, wo, u, wi, pdf);
}

__device__ __forceinline__ bool is_delta(const BsdfRecord& b) { return (b.type & kTypeDelta) != 0; }

// The direction v in the shading frame of normal n, for evaluating BSDF b:
// DiffuseBSDF's eval and pdf read only the z component, dot(v, n) (to_local),
// so a diffuse lane skips Frame(n) (a sqrt, a division and a branch); the x, y
// it leaves at 0 are never read. BDPT_DIFFUSE_Z 0 builds every frame.
#ifndef BDPT_DIFFUSE_Z
#define BDPT_DIFFUSE_Z 1
#endif
__device__ __forceinline__ f3 local_for(const BsdfRecord& b, f3 n, f3 v) {
#if BDPT_DIFFUSE_Z
    if (b.kind == BSDF_DIFFUSE) return mk(0.f, 0.f, dot(v, n));
#endif
    return local_at(n, v);
}

// ---------------------------------------------------------------- emitters
// Distribution1D::sample (math.h:107-111): upper_bound, then clamp.
__device__ __forceinline__ int cdf_sample(const float* cdf, int ncdf, float u) {
    int lo = 0, hi = ncdf;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    int i = lo - 1;
    i = i < 0 ? 0 : i;
    return i > ncdf - 2 ? ncdf - 2 : i;
}

// The same search over an LDS copy of the CDF (address space 3: ds_read).
__device__ __forceinline__ int cdf_sample_lds(const float* cdf_generic, int ncdf, float u) {
    const __attribute__((address_space(3))) float* cdf =
        (const __attribute__((address_space(3))) float*)(cdf_generic);
    int lo = 0, hi = ncdf;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    int i = lo - 1;
    i = i < 0 ? 0 : i;
    return i > ncdf - 2 ? ncdf - 2 : i;
}

// selectEmitter + sampleEmitterPosition (integrator.cpp:46-51, :73-100): 4 draws.
// Returns the emitter index.
template <class Rng>
__device__ __forceinline__ int sample_emitter(const DevScene& sc, Rng& rng, float& emitter_pdf, f3& n, f3& pos,
                                              float& pos_pdf, int* graze = nullptr) {
    const float u0 = next1(rng);
    uint32_t id = static_cast<uint32_t>(u0 * static_cast<float>(sc.nemit));
    id = id < static_cast<uint32_t>(sc.nemit - 1) ? id : static_cast<uint32_t>(sc.nemit - 1);
    emitter_pdf = sc.inv_nemit;  // 1.f / nemit
    const EmitterRecord& e = emitter_of(sc, static_cast<int>(id));
    const bool lds = sc.lds_etri_off != kNoLds;  // uniform: LDS copies of the faces and CDFs
    const float* cdf = lds ? reinterpret_cast<const float*>(g_scene_lds + sc.lds_ecdf_off) : sc.emit_cdf;
    const float u1 = next1(rng);
    const int f = lds ? cdf_sample_lds(cdf + e.cdf_offset, e.nfaces + 1, u1)
                      : cdf_sample(cdf + e.cdf_offset, e.nfaces + 1, u1);
    const F2 uv = uniform_triangle(next2(rng));
    // Typed loads on both sides (ds_read / global_load): through one generic
    // pointer the compiler emitted FLAT loads, which wait for vmcnt(0) and
    // lgkmcnt(0) together.
    float4 a, b, c, d, g;
    if (lds) {
        typedef const __attribute__((address_space(3))) v4f_t lds_v4f;
        const lds_v4f* q = (const lds_v4f*)(g_scene_lds + sc.lds_etri_off) + 5 * (e.face_offset + f);
        const v4f_t q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        a = make_float4(q0.x, q0.y, q0.z, q0.w), b = make_float4(q1.x, q1.y, q1.z, q1.w);
        c = make_float4(q2.x, q2.y, q2.z, q2.w), d = make_float4(q3.x, q3.y, q3.z, q3.w);
        g = make_float4(q4.x, q4.y, q4.z, q4.w);
    } else {
        const float4* q = sc.emit_tri + 5 * static_cast<size_t>(e.face_offset + f);
        a = gld4(q), b = gld4(q + 1), c = gld4(q + 2), d = gld4(q + 3), g = gld4(q + 4);
    }
    const f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, b.x, b.y), v2 = mk(b.z, b.w, c.x);
    const f3 n0 = mk(c.y, c.z, c.w), n1 = mk(d.x, d.y, d.z), n2 = mk(d.w, g.x, g.y);
    const float w = 1 - uv.x - uv.y;
    pos = (v0 * w + v1 * uv.x) + v2 * uv.y;
    n = normalize((n0 * w + n1 * uv.x) + n2 * uv.y);
    pos_pdf = rcp_w(e.area);
    if (graze) *graze = __float_as_int(g.z) << 24;  // the face's graze code (bdpt_capi.cpp device_emit_tri)
    return static_cast<int>(id);
}

}  // namespace dev
}  // namespace bdpt
