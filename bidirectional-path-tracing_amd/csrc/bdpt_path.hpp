// The BDPT path state machine shared by the HIP kernels: one camera sample
// (pixel, k) of BDPTIntegrator::render (reference src/integrators/bdpt.h:219-241)
// as a sequence of ray queries. A Lane holds the sample's state between
// queries; resolve() applies a query's result and advance() runs the
// integrator until the lane needs its next query (or finishes the sample).
// The megakernel (bdpt_kernels.hip) and the single-sample kernels
// (sample_state.hip) keep Lanes in registers (the cold part in LDS).
#pragma once

#include <hip/hip_runtime.h>

#include "bdpt_device.hpp"

namespace bdpt {
namespace dev {


constexpr int kLvFields = 16;  // p vcm n vc wo rr tp mat
constexpr uint32_t kFlagNoEyeAccum = 0x100u;  // single-sample API: Li is returned, not added
// Safety bound on the queries of one sample: a legal sample issues at most D
// light-walk rays, D camera splats, D eye-walk rays and, per eye vertex, one
// light sample plus D - 1 connections: < (D + 3)(D + 1) for rrDepth D. With
// Russian roulette the walks are bounded by DevFrame::depth_cap (2^25 bounces,
// each eye vertex with at most lv_max connections): 2^30 is beyond any legal sample.
__device__ __forceinline__ int max_steps_per_sample(int rr_depth) { return (rr_depth + 3) * (rr_depth + 1) + 64; }

// ---------------------------------------------------------- Russian roulette
// The reference ships with NO_RR = 1 (bdpt.h:18): every subpath stops at
// rrDepth and every stored rr is 1. Its NO_RR = 0 branch continues past rrDepth
// while sampler.next() < rrProbability (bdpt.h:68, :188), with rrProbability =
// (depth + 1) < rrDepth ? 1 : (getLuminance(throughput) < 0.01 ? 0.5 : 1)
// (bdpt.h:129, :201) stored in the vertex and multiplying every pdf of it
// (bdpt.h:250, :272, :342, :410, :417, :461-472). BDPT_RR 0: the NO_RR = 1
// builds (rr is the constant 1, nothing of it is compiled); 1: the RR build of
// the megakernel (bdpt_kernels_rr.hip); 2: chosen per launch (DevFrame::rr_mode,
// the single-sample build).
#ifndef BDPT_RR
#define BDPT_RR 0
#endif
__device__ __forceinline__ bool rr_on(const DevFrame& fr) {
#if BDPT_RR == 1
    return true;
#elif BDPT_RR == 2
    return fr.rr_mode != 0;
#else
    (void)fr;
    return false;
#endif
}
__device__ __forceinline__ float rr_probability(const DevFrame& fr, int depth, f3 tp) {
    if (!rr_on(fr) || (depth + 1) < fr.rr_depth) return 1.f;
    return dot(tp, mk(0.212671f, 0.715160f, 0.072169f)) < 0.01f ? 0.5f : 1.f;  // getLuminance (math.h:56-58)
}

// Light-vertex scratch, one contiguous record per lane: vertex v of slot s is
// the four float4 at lv[(s * maxv + v) * 4 + q] — (p, vcm) (n, vc) (wo, rr)
// (tp, mat). A lane reads or writes a whole 64-byte vertex from one cache
// line; the divergent shading code touches no line it does not use.
struct LightStore {
    float4* __restrict__ base;
    uint32_t maxv, slot;
    bool tid_rel = false;  // slot is the block's first; the lane adds threadIdx.x at each access (opaque_tid)
    __device__ __forceinline__ float4* at(int v) const {
        const uint32_t s = tid_rel ? slot + opaque_tid() : slot;
        return base + (static_cast<size_t>(s) * maxv + static_cast<uint32_t>(v)) * 4;
    }
    // vertex v of the lane threadIdx.x == tid (tid_rel stores only)
    __device__ __forceinline__ float4* at_tid(int v, uint32_t tid) const {
        return base + (static_cast<size_t>(slot + tid) * maxv + static_cast<uint32_t>(v)) * 4;
    }
};
__device__ __forceinline__ LightStore light_store(float* lv, int lv_max, uint32_t slot) {
    return LightStore{reinterpret_cast<float4*>(lv), static_cast<uint32_t>(lv_max > 1 ? lv_max : 1), slot};
}

struct Vertex {  // PathVertex (bdpt.h:24-35); its Frame is rebuilt from n where used
    f3 p, n, wo, tp;
    float vcm, vc, rr;
    int mat;
};

#ifndef BDPT_LV_NT
#define BDPT_LV_NT 0  // 1: light-vertex records use non-temporal loads / stores (keep L2 for the scene)
#endif
__device__ __forceinline__ void lv_st(float4* p, float4 x) {
#if BDPT_LV_NT
    __builtin_nontemporal_store(v4f_t{x.x, x.y, x.z, x.w}, (__attribute__((address_space(1))) v4f_t*)(p));
#else
    gst4(p, x);
#endif
}
__device__ __forceinline__ float4 lv_ld(const float4* p) {
#if BDPT_LV_NT
    const v4f_t v = __builtin_nontemporal_load((const __attribute__((address_space(1))) v4f_t*)(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return gld4(p);
#endif
}
#ifndef BDPT_PROBE_NO_LV_STORE
#define BDPT_PROBE_NO_LV_STORE 0  // accounting probe only (a wrong image): light-vertex records not written
#endif
__device__ __forceinline__ void store_vertex(const LightStore& ls, int v, const Hit& h, f3 tp, float vcm, float vc,
                                             float rr) {
    if (BDPT_PROBE_NO_LV_STORE) return;
    float4* q = ls.at(v);
    lv_st(q, make_float4(h.p.x, h.p.y, h.p.z, vcm));
    lv_st(q + 1, make_float4(h.n.x, h.n.y, h.n.z, vc));
    lv_st(q + 2, make_float4(h.wo.x, h.wo.y, h.wo.z, rr));
    lv_st(q + 3, make_float4(tp.x, tp.y, tp.z, __int_as_float(h.mat)));
}

__device__ __forceinline__ Vertex load_vertex_at(const float4* q) {
    const float4 a = lv_ld(q), b = lv_ld(q + 1), c = lv_ld(q + 2), d = lv_ld(q + 3);
    Vertex x;
    x.p = xyz(a), x.vcm = a.w;
    x.n = xyz(b), x.vc = b.w;
    x.wo = xyz(c), x.rr = c.w;
    x.tp = xyz(d), x.mat = __float_as_int(d.w);
    return x;
}
__device__ __forceinline__ Vertex load_vertex(const LightStore& ls, int v) {
    const float4* q = ls.at(v);
    const float4 a = lv_ld(q), b = lv_ld(q + 1), c = lv_ld(q + 2), d = lv_ld(q + 3);
    Vertex x;
    x.p = xyz(a), x.vcm = a.w;
    x.n = xyz(b), x.vc = b.w;
    x.wo = xyz(c), x.rr = c.w;  // rr: always 1 under NO_RR (bdpt.h:18), where x * rr == x is not formed
    x.tp = xyz(d), x.mat = __float_as_int(d.w);
    return x;
}

#ifndef BDPT_CONN_EARLY_COS
#define BDPT_CONN_EARLY_COS 3  // 1: connectVertices rejects on the cosines before building frames; 2: also connectToLight (+1.3 %); 3: also connectToCamera (+0.6 %)
#endif

// ContinuePathRandomWalk (bdpt.h:243-291): BSDF sample (2 draws), throughput,
// vc / vcm recursion (Georgiev VCM Eqs. 52-54) and the next ray.
__device__ __forceinline__ bool continue_walk(const BsdfRecord& b, const Hit& h, LazyMT& rng, f3& tp, int& depth,
                                              float& vc, float& vcm, Ray& ray, float rrp) {
    const bool delta = is_delta(b);
    float pdf;
    f3 wi;
    const f3 f = bsdf_sample(b, h.wo, next2(rng), wi, pdf);
    pdf *= rrp;
    const float absCosOut = fabsf(wi.z);
    if (is_zero(f)) return false;
    tp = tp * (f * rcp_w(pdf));
    depth++;
    const float prevRev = delta ? pdf : bsdf_pdf(b, h.wo, wi) * rrp;  // pdf of the swapped (wo, wi)
    if (delta) {
        vc = div_w(absCosOut, pdf) * (prevRev * vc);
        vcm = 0.f;
    } else {
        vc = div_w(absCosOut, pdf) * (vcm + prevRev * vc);
        vcm = rcp_w(pdf);
    }
    ray = Ray{h.p, world_at(h.n, wi), kEpsilon, 3.402823466e+38f};  // FLT_MAX (core.h:120)
    return true;
}

// splatToImagePlane (bdpt.h:485-496): worldToCamera, cameraToClip, /w, NDCToScreen.
__device__ __forceinline__ void splat_pixel(const CameraConstants& c, f3 p, int& x, int& y) {
    const float* m = c.w2c;
    float a0 = (m[0] * p.x + m[4] * p.y) + (m[8] * p.z + m[12] * 1.f);
    float a1 = (m[1] * p.x + m[5] * p.y) + (m[9] * p.z + m[13] * 1.f);
    float a2 = (m[2] * p.x + m[6] * p.y) + (m[10] * p.z + m[14] * 1.f);
    float a3 = (m[3] * p.x + m[7] * p.y) + (m[11] * p.z + m[15] * 1.f);
    m = c.c2clip;
    float b0 = (m[0] * a0 + m[4] * a1) + (m[8] * a2 + m[12] * a3);
    float b1 = (m[1] * a0 + m[5] * a1) + (m[9] * a2 + m[13] * a3);
    float b2 = (m[2] * a0 + m[6] * a1) + (m[10] * a2 + m[14] * a3);
    float b3 = (m[3] * a0 + m[7] * a1) + (m[11] * a2 + m[15] * a3);
    const float w = b3;
    b0 = div_cr(b0, w), b1 = div_cr(b1, w), b2 = div_cr(b2, w), b3 = div_cr(b3, w);
    m = c.ndc2screen;
    const float d0 = (m[0] * b0 + m[4] * b1) + (m[8] * b2 + m[12] * b3);
    const float d1 = (m[1] * b0 + m[5] * b1) + (m[9] * b2 + m[13] * b3);
    x = x86_trunc_i32(d0);
    y = x86_trunc_i32(d1);
}

// Camera ray of Renderer::render (renderer.cpp:162-192); 2 jitter draws if spp > 1.
__device__ __forceinline__ f3 camera_dir(const DevFrame& fr, int pixel, LazyMT& rng) {
    const CameraConstants& c = fr.cam;
    const int j = pixel % fr.W, i = pixel / fr.W;
    const float y = (1.f - (static_cast<float>(i) + 0.5f) * c.invH) * 2.f - 1.f;
    const float x = ((static_cast<float>(j) + 0.5f) * c.invW) * 2.f - 1.f;
    float px, py;
    if (fr.spp == 1) {
        px = x * c.angle * c.aspect;
        py = y * c.angle;
    } else {
        F2 rs = next2(rng);
        rs.x -= 0.5f;
        rs.y -= 0.5f;
        rs.x = rs.x * c.invW;
        rs.y = rs.y * c.invH;
        px = (x + rs.x) * c.angle * c.aspect;
        py = (y + rs.y) * c.angle;
    }
    const float* m = c.c2w;  // cameraToWorld * (px, py, -near, 0)
    f3 d;
    d.x = (m[0] * px + m[4] * py) + (m[8] * -1.f + m[12] * 0.f);
    d.y = (m[1] * px + m[5] * py) + (m[9] * -1.f + m[13] * 0.f);
    d.z = (m[2] * px + m[6] * py) + (m[10] * -1.f + m[14] * 0.f);
    return normalize(d);
}

// --------------------------------------------------------- lane state machine
enum : uint32_t {  // the query a lane waits on
    ST_IDLE = 0,
    ST_PRIMARY,  // render(): primary closest hit (bdpt.h:225)
    ST_LIGHT,    // lightSubpathWalk closest hit (bdpt.h:190)
    ST_SPLAT,    // connectToCamera visibility (bdpt.h:318)
    ST_EYE,      // eyeSubpathWalk closest hit (bdpt.h:70)
    ST_NEE,      // connectToLight visibility (bdpt.h:405)
    ST_CONN,     // connectVertices visibility (bdpt.h:451)
    ST_DEFER,    // no query: the lane resumes at A_START_EYE in the next shading step
    ST_PARKED,   // Russian-roulette build: the sample's deep walk continues in the chain kernel
};
enum : uint32_t {  // actions that need no query
    A_ISSUED = 0,
    A_START_LIGHT,
    A_NEE,  // connectToLight after the emitter sample
    A_LIGHT_NEXT,
    A_LIGHT_VERTEX,
    A_LIGHT_CONTINUE,
    A_START_EYE,
    A_EYE_NEXT,
    A_EYE_VERTEX,
    A_CONN,
    A_EYE_CONTINUE,
    A_FINISH,
    A_DONE,
};

// Per-lane state between queries. The hot part lives in registers; the part
// only some actions touch (LaneCold) lives in LDS, one 92-byte record per
// lane — an odd number of dwords (23), so a wave's accesses are bank-conflict free —
// which keeps the megakernel's register allocation (and its scratch spills)
// down without slowing the actions that use it.
struct LaneCold {
    f3 tp;        // subpath throughput
    float vc, vcm;
    f3 cam_d;     // the camera ray direction (the eye walk re-traces it, bdpt.h:59,70)
    f3 Li;        // eye estimate of the sample; during the light walk: the primary hit's (t, u, v)
    f3 pend;      // contribution applied if the pending shadow ray is unoccluded
    int pend_px;  // splat pixel of a pending camera connection
    int pixel;
    int prim_tri;  // primary hit triangle (its t, u, v sit in Li until the eye walk starts)
    int steps;    // queries issued for the current sample
    int nl;       // stored light vertices
    int ci;       // next light vertex to connect
    int depth;
    uint32_t pure;  // isPathPureSpecular
    float rr;       // rrProbability of the current vertex (Russian-roulette builds; keeps the record odd-dword)
};
static_assert(sizeof(LaneCold) == 92, "odd dword stride keeps LDS accesses conflict free");

struct Lane {
    LazyMT rng;
    uint32_t state;
    Ray ray;  // the pending query
    Hit h;    // current subpath vertex
    LaneCold& c;
    __device__ explicit Lane(LaneCold& cold) : c(cold) {}
};

// rgb[pixel] += radiance * misWeight under the pixel's lock (bdpt.h:363-370).
// The single-sample build returns the splats of its one sample as a list
// instead (fb = header {count, capacity, 0, 0} then (pixel, r, g, b) records),
// so the caller adds them to its own framebuffer in the reference's order.
#ifndef BDPT_PROBE_NO_SPLAT
#define BDPT_PROBE_NO_SPLAT 0
#endif
__device__ __forceinline__ void splat_add(float* __restrict__ fb, int pixel, f3 v) {
#if BDPT_SAMPLER_STATE
    uint32_t* const hdr = reinterpret_cast<uint32_t*>(fb);
    const uint32_t k = hdr[0];
    hdr[0] = k + 1;
    if (k < hdr[1]) {
        float* e = fb + 4 + 4 * static_cast<size_t>(k);
        e[0] = __int_as_float(pixel), e[1] = v.x, e[2] = v.y, e[3] = v.z;
    }
#elif BDPT_PROBE_NO_SPLAT
    (void)fb, (void)pixel, (void)v;  // accounting probe only (a wrong image): no camera-splat atomics
#else
    float* px = fb + 3 * static_cast<size_t>(pixel);
    gadd(px + 0, v.x);
    gadd(px + 1, v.y);
    gadd(px + 2, v.z);
#endif
}

// Eye-estimate sums per wave (frame kernels). With spp a multiple of 64 the
// megakernel's 64-sample refill chunks each cover ONE pixel, and the samples a
// wave runs at a time come from its few most recent chunks. Each wave keeps a
// sum (x, y, z, pixel bits in w) for each of its last BDPT_EYE_SLOTS chunks in
// LDS: a finishing sample whose pixel has a slot adds to it (ds_add_f32) and
// the slot goes to the framebuffer once, when its chunk's place is reused or
// the kernel ends; any other sample adds to the framebuffer directly. The sums
// are the same products in another order (float reassociation, as the device
// atomics already are); each framebuffer add is a memory-side request of its
// own, so ~3 of the ~9 per sample become ~3 per 64 samples.
#ifndef BDPT_EYE_SLOTS
#define BDPT_EYE_SLOTS 4
#endif
#if BDPT_EYE_SLOTS && !BDPT_SAMPLER_STATE
constexpr int kEyeSlotWaves = 4;  // waves per 256-lane frame-kernel block
__shared__ float4 eye_slots[kEyeSlotWaves][BDPT_EYE_SLOTS];
__device__ __forceinline__ float4* wave_eye_slots() { return eye_slots[(threadIdx.x >> 6) & (kEyeSlotWaves - 1)]; }
// Lane 0 of the wave: slot k to the framebuffer, then reset to `pixel` (-1: unused).
__device__ __forceinline__ void eye_slot_reset(float* __restrict__ fb, int k, int pixel) {
    float4* const s = wave_eye_slots();
    const float4 e = s[k];
    const int p = __float_as_int(e.w);
    if (p >= 0 && (e.x != 0.f || e.y != 0.f || e.z != 0.f)) {
        float* px = fb + 3 * static_cast<size_t>(p);
        gadd(px + 0, e.x);
        gadd(px + 1, e.y);
        gadd(px + 2, e.z);
    }
    s[k] = make_float4(0.f, 0.f, 0.f, __int_as_float(pixel));
}
#endif

// Shadow-ray tasks (BDPT_HELP, the frame kernels without Russian roulette; round 6,
// VERDICT r5 item 1). The wave's owners hold ~99 connection tasks per shading step,
// and serialising them through each owner's one query per step kept both the
// shading steps (one per connection) and the walk loop's lane occupancy (waiting
// lanes idle) low. Here an owner computes every connection of a vertex at once —
// connectToCamera's splat (bdpt.h:295-371), connectToLight (bdpt.h:374-430) and
// connectVertices with all light vertices (bdpt.h:434-483), everything but the
// visibility test, in the reference's order and arithmetic — and pushes each
// shadow ray with its contribution (already scaled by 1 / spp for the eye
// estimate) and target pixel into its wave's ring, then continues its walk in the
// same shading step. Lanes of the wave that wait in the walk loop (their own
// result ready, or no sample) claim tasks and walk them; an unoccluded one adds its
// contribution to the pixel (the wave's eye slot, else the framebuffer). The
// visibility tests and contributions are the reference's; only the order of the
// float additions into a pixel changes (as with the device atomics). A full ring
// makes the owner trace that shadow ray itself, as the serial build does.
#ifndef BDPT_HELP
#define BDPT_HELP 0
#endif
#if BDPT_HELP && !BDPT_SAMPLER_STATE
constexpr uint32_t kTaskSplat = 0x40000000u;   // meta bit: a camera splat (framebuffer add, bdpt.h:363-370)
constexpr uint32_t kTaskPixel = 0x3fffffffu;
constexpr int kResShaded = -2;  // an own closest-hit result already applied to the lane (walk loop, help_compact)
// The wave's ring positions live in LDS, in the Russian-roulette field of its
// first two lanes' cold records (unused by these builds; the LDS of 4 resident
// blocks is full): head (tasks claimed) in lane 0's, tail (pushed) in lane 1's.
struct TaskCtl {
    lds_u32* head;
    lds_u32* tail;
};
__device__ __forceinline__ TaskCtl task_ctl(const LaneCold& mine) {
    lds_u32* const w = (lds_u32*)(&mine - (opaque_tid() & 63));
    constexpr uint32_t kRrWord = offsetof(LaneCold, rr) / 4, kStride = sizeof(LaneCold) / 4;
    return TaskCtl{w + kRrWord, w + kStride + kRrWord};
}
__device__ __forceinline__ float4* task_ring(const DevFrame& fr) {
    const uint32_t wave = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x * 4 + (threadIdx.x >> 6))));
    return fr.tasks + static_cast<size_t>(wave) * fr.task_cap * 3;
}
// Called by the lanes that push (their exec mask is the set): true if this lane's
// task went into the ring (false: the ring is full; the caller traces it itself).
#ifndef BDPT_HELP_SOA
#define BDPT_HELP_SOA 1  // the ring as three planes of 16-byte vectors (consecutive slots' pushes and claims coalesce)
#endif
// float4 k (0..2) of ring slot `slot`
__device__ __forceinline__ float4* task_vec(float4* ring, uint32_t cap, uint32_t slot, int k) {
    return BDPT_HELP_SOA ? ring + static_cast<size_t>(k) * cap + slot : ring + 3 * static_cast<size_t>(slot) + k;
}
__device__ __forceinline__ bool task_push(const LaneCold& mine, const DevFrame& fr, const Ray& r, bool nocull, f3 c,
                                          int pixel, bool splat, Counts& cnt) {
    const TaskCtl ctl = task_ctl(mine);
    const uint64_t m = __ballot(true);
    const uint32_t head = *ctl.head, tail = *ctl.tail;
    const uint32_t n = static_cast<uint32_t>(popc64(m)), rank = static_cast<uint32_t>(lanes_below(m));
    const uint32_t space = fr.task_cap - (tail - head);
    const uint32_t k = n < space ? n : space;
    *ctl.tail = tail + k;  // (every pushing lane writes the same value)
    cnt.q[rank < k ? 0 : 1]++;  // (counting pass: pushed / refused)
    if (rank >= k) return false;
    float4* const ring = task_ring(fr);
    const uint32_t slot = (tail + rank) & (fr.task_cap - 1);
    // (o, max_t) (d, near cull) (contribution, pixel | splat bit)
    gst4(task_vec(ring, fr.task_cap, slot, 0), make_float4(r.o.x, r.o.y, r.o.z, r.max_t));
    gst4(task_vec(ring, fr.task_cap, slot, 1), make_float4(r.d.x, r.d.y, r.d.z, nocull ? kNoCullNear : kCullNear));
    gst4(task_vec(ring, fr.task_cap, slot, 2),
         make_float4(c.x, c.y, c.z, __uint_as_float(static_cast<uint32_t>(pixel) | (splat ? kTaskSplat : 0u))));
    return true;
}
#else
constexpr int kResShaded = -2;
__device__ __forceinline__ bool task_push(const LaneCold&, const DevFrame&, const Ray&, bool, f3, int, bool, Counts&) {
    return false;
}
#endif
constexpr bool kTasks = BDPT_HELP && !BDPT_SAMPLER_STATE;

// An eye-estimate addition for the pixel: the wave's slot when it holds the pixel, else the framebuffer.
__device__ __forceinline__ void eye_add(float* __restrict__ fb, int pixel, f3 add) {
#if BDPT_EYE_SLOTS && !BDPT_SAMPLER_STATE
    float4* const s = wave_eye_slots();
    int k = -1;
#pragma unroll
    for (int j = 0; j < BDPT_EYE_SLOTS; j++)
        if (__float_as_int(s[j].w) == pixel) k = j;
    if (k >= 0) {
        atomicAdd(&s[k].x, add.x);
        atomicAdd(&s[k].y, add.y);
        atomicAdd(&s[k].z, add.z);
        return;
    }
#endif
    float* px = fb + 3 * static_cast<size_t>(pixel);
    gadd(px + 0, add.x);
    gadd(px + 1, add.y);
    gadd(px + 2, add.z);
}

template <bool COUNT>
__device__ __forceinline__ void finish(Lane& L, const DevFrame& fr, float* __restrict__ fb, Counts& cnt) {
    if (COUNT) {
        cnt.c[7] += L.rng.n;
        cnt.m[1] = max(cnt.m[1], static_cast<uint32_t>(L.c.depth));
        cnt.m[2] = max(cnt.m[2], static_cast<uint32_t>(L.c.steps));
        if (fr.row_cost)  // the sample's queries to its local row (bdpt_get_row_costs)
            gadd(fr.row_cost + (L.c.pixel / fr.W - fr.row_offset) / fr.row_stride,
                 static_cast<unsigned long long>(L.c.steps));
    }
    // rgb[p] += acc * (1 / spp) (renderer.cpp:202), one sample at a time.
    if (!(fr.flags & kFlagNoEyeAccum) && (L.c.Li.x != 0.f || L.c.Li.y != 0.f || L.c.Li.z != 0.f)) {
        const float inv_spp = fr.inv_spp;  // 1.f / spp
        eye_add(fb, L.c.pixel, L.c.Li * inv_spp);
    }
    L.state = ST_IDLE;
}

// Advances a lane from action `act` until it issues its next query or ends its
// sample. The actions form a DAG between queries, so one forward sweep in
// topological order runs every lane's whole chain: each action body executes at
// most once per call, for all lanes that reach it wherever they entered the
// chain (a loop over a switch would re-run a body for every lane that reached it
// one step later). Work two actions share runs in one body: the emitter sample
// of lightSubpathWalk and connectToLight, and ContinuePathRandomWalk of both
// subpaths. The only edges against this order — a light subpath that ends at its
// BSDF sample or its depth cap and starts the eye subpath — are deferred to the
// next shading step (ST_DEFER) instead of being run by a second sweep.
// Counting pass: lanes and wave executions per body ([10], [11]) and wave
// clocks per body (counters [21 + k]).
#define BDPT_ACTION(ID, COND)                 \
    if (COUNT) tally_action(cnt, (COND));     \
    if (COND) do {                            \
        const ActionClock<COUNT> clk_(cnt, ID);
#define BDPT_END \
    }            \
    while (0)
template <bool ON>
struct ActionClock {
    __device__ ActionClock(Counts&, int) {}
};
template <>
struct ActionClock<true> {
    Counts& c;
    int id;
    uint64_t t0;
    __device__ ActionClock(Counts& cnt, int i) : c(cnt), id(i), t0(__builtin_amdgcn_s_memtime()) {}
    __device__ ~ActionClock() {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (first_active_lane()) c.c[id] += static_cast<uint32_t>(t1 - t0);
    }
};
__device__ __forceinline__ void tally_action(Counts& cnt, bool on) {
    if (on) {
        cnt.c[10]++;
        if (first_active_lane()) cnt.c[11]++;  // one wave-level execution of this body
    }
}

// The subpath loop test of bdpt.h:68 / :188. With Russian roulette a subpath
// that reaches DevFrame::depth_cap (the light-vertex store's bound) ends there
// and the sample is counted in *capped (the frame is then not the reference's).
__device__ __forceinline__ bool walk_continues(Lane& L, const DevFrame& fr) {
    if (L.c.depth < fr.rr_depth) return true;
    const float u = next1(L.rng);
    if (!rr_on(fr) || !(u < L.c.rr)) return false;
    if (L.c.depth >= fr.depth_cap) {
        gadd(fr.capped, 1u);
        return false;
    }
    return true;
}

// cull_near_for's rule for a shadow ray in direction d leaving the lane's current
// vertex (NEE, connectVertices): true = no near cull.
__device__ __forceinline__ bool vertex_nocull(const Lane& L, f3 d);

// BDPT_GRAZE_IN_DIST 1: a vertex's near-cull threshold (graze_threshold) is
// decoded once, in its vertex body, into Hit::dist (dead after that body), and
// the queries leaving the vertex compare against it (cull_near_for).
#ifndef BDPT_GRAZE_IN_DIST
#define BDPT_GRAZE_IN_DIST 0
#endif
#if BDPT_GRAZE_IN_DIST
#define BDPT_DIST_TO_GRAZE L.h.dist = graze_threshold(L.h.shape);
#else
#define BDPT_DIST_TO_GRAZE
#endif
#ifndef BDPT_SPLIT_CONTINUE
#define BDPT_SPLIT_CONTINUE 0  // 1: the light subpath's continuation runs before the eye subpath's start, so a light walk that ends starts its eye walk in the same sweep (no ST_DEFER step); the eye continuation is its own body
#endif
/* Bodies placed at two points of the sweep (BDPT_SPLIT_CONTINUE). */
#define BDPT_BODY_LIGHT_VERTEX \
    BDPT_ACTION(26, act == A_LIGHT_VERTEX) {  /* bdpt.h:193-209 */ \
        const float dist2 = L.h.dist * L.h.dist; \
        BDPT_DIST_TO_GRAZE \
        const float absCosIn = fabsf(L.h.wo.z); \
        L.c.vcm *= div_w(dist2, absCosIn); \
        L.c.vc *= rcp_w(absCosIn); \
        act = A_LIGHT_CONTINUE; \
        if (rr_on(fr)) L.c.rr = rr_probability(fr, L.c.depth, L.c.tp);  /* bdpt.h:201-204 */ \
        const BsdfRecord& b = bsdf_of(sc, L.h.mat); \
        if (is_delta(b)) break; \
        if (COUNT) cnt.t_step++;  /* a camera-connection task (Counts::q) */ \
        /* connectToCamera (bdpt.h:295-371): everything but the visibility test. */ \
        f3 e2l = L.h.p - cam_o; \
        const float invD2 = rcp_w(dot(e2l, e2l)); \
        e2l = e2l * sqrt_w(invD2); \
        int xp, yp; \
        splat_pixel(fr.cam, L.h.p, xp, yp); \
        if (xp < 0 || yp < 0 || xp >= fr.W || yp >= fr.H) break; \
        const float cosCamera = dot(fwd, e2l); \
        if (cosCamera <= 0.f) break; \
        const bool early_cos_ = BDPT_CONN_EARLY_COS >= 3; /* reject on wi.z = dot(-e2l, n) (the frame z component, to_local) first */ \
        if (early_cos_ && dot(-e2l, L.h.n) <= 0.f) break; \
        const f3 wi = early_cos_ ? local_for(b, L.h.n, -e2l) : local_at(L.h.n, -e2l); \
        const EvalPdfs ep = bsdf_eval_pdfs(b, wi, L.h.wo); \
        const f3 f = ep.f; \
        if (is_zero(f) || (!early_cos_ && wi.z <= 0.f)) break; \
        const float d = div_w(fr.cam.vnear, cosCamera); \
        const float img2solid = div_w(d * d, cosCamera); \
        const float img2surf = img2solid * (wi.z * invD2); \
        const float surf2img = rcp_w(img2surf); \
        const float nlight = static_cast<float>(fr.W * fr.H); \
        f3 rad = L.c.tp * (f * rcp_w(wi.z)); \
        rad = rad * rcp_w(surf2img); \
        rad = rad * fr.inv_pixels;  /* rcp(nlight) */ \
        rad = rad * fr.inv_spp;  /* rcp(spp) */ \
        const float reversePdf_a = 1.f * img2surf; \
        const float prevRev = ep.rev * (rr_on(fr) ? L.c.rr : 1.f);  /* swapped (wi, wo) * lightVertex.rr (bdpt.h:342) */ \
        const float lightWeight = div_w(reversePdf_a, nlight) * (L.c.vcm + prevRev * L.c.vc); \
        const float mis = rcp_w(lightWeight + 1.f + 0.f); \
        const f3 pend_ = (fr.strategy == 0) ? rad * mis : rad; \
        const int px_ = yp * fr.W + xp; \
        const Ray sr_ = shadow_ray(cam_o, L.h.p); \
        if (kTasks && task_push(L.c, fr, sr_, false, pend_, px_, true, cnt)) break;  /* a helper walks it (act: A_LIGHT_CONTINUE) */ \
        L.c.pend = pend_; \
        L.c.pend_px = px_; \
        L.ray = sr_; \
        L.state = ST_SPLAT; \
        act = A_ISSUED; \
    } BDPT_END;
#define BDPT_BODY_CONTINUE(ACT_, COND_) \
    /* ContinuePathRandomWalk of either subpath (light: bdpt.h:211-215, eye: bdpt.h:152). */ \
    BDPT_ACTION(28, COND_) { \
        const bool light = act == A_LIGHT_CONTINUE; \
        const BsdfRecord& b = bsdf_of(sc, L.h.mat); \
        const bool delta = is_delta(b); \
        const float rrp = rr_on(fr) ? L.c.rr : 1.f; \
        /* the store is full: the vertex would be pushed only if the walk continues (bdpt.h:211-215) */ \
        const bool full = rr_on(fr) && light && !delta && L.c.nl >= fr.lv_max; \
        if (light && !delta && !full) store_vertex(ls, L.c.nl, L.h, L.c.tp, L.c.vcm, L.c.vc, rrp);  /* the pre-walk state */ \
        const bool more = continue_walk(b, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, rrp); \
        if (full && more) {  /* it would be stored: flag the sample, end the light walk */ \
            gadd(fr.capped, 1u); \
            L.state = ST_DEFER; \
            act = A_ISSUED; \
            break; \
        } \
        if (!light) { \
            act = more ? A_EYE_NEXT : A_FINISH; \
        } else if (more) { \
            if (!delta) { \
                L.c.nl++; \
                if (COUNT) cnt.c[4]++; \
            } \
            act = A_LIGHT_NEXT; \
        } else if (BDPT_SPLIT_CONTINUE) {  /* the light subpath ends; the eye subpath starts in this sweep */ \
            act = A_START_EYE; \
        } else {  /* the light subpath ends; the eye subpath starts next step */ \
            L.state = ST_DEFER; \
            act = A_ISSUED; \
        } \
    } BDPT_END;
#define BDPT_BODY_LIGHT_NEXT \
    /* Loop conditions `depth < m_rrDepth || (sampler.next() < rrProbability && !NO_RR)` */ \
    /* (bdpt.h:188, :68): past rrDepth one draw, then (RR only) a continuation. */ \
    BDPT_ACTION(29, act == A_LIGHT_NEXT) { \
        if (walk_continues(L, fr)) { \
            L.state = ST_LIGHT; \
            act = A_ISSUED; \
        } else if (BDPT_SPLIT_CONTINUE) { \
            act = A_START_EYE;  /* the eye subpath starts in this sweep */ \
        } else { \
            L.state = ST_DEFER;  /* the eye subpath starts next step */ \
            act = A_ISSUED; \
        } \
    } BDPT_END;

// PART 0: the whole sweep; 1: the bodies before connectVertices, returning the
// action reached; 2: connectVertices and the bodies after it (the BDPT_HELP_BATCH
// schedule runs the wave's connections between the two, conn_batch).
template <bool COUNT, int PART = 0>
__device__ uint32_t advance(Lane& L, uint32_t act, const DevScene& sc, const DevFrame& fr, float* __restrict__ fb,
                            const LightStore& ls, Counts& cnt) {
    const f3 cam_o = mk(fr.cam_o[0], fr.cam_o[1], fr.cam_o[2]);
    const f3 fwd = mk(fr.cam.fwd[0], fr.cam.fwd[1], fr.cam.fwd[2]);
    if (COUNT && PART != 2 && act == A_CONN && fr.strategy == 0) cnt.t_step += static_cast<uint32_t>(L.c.nl - L.c.ci);  // (Counts::q)
    if (PART != 2) {
#if BDPT_SPLIT_CONTINUE
    BDPT_BODY_LIGHT_VERTEX
    BDPT_BODY_CONTINUE(A_LIGHT_CONTINUE, act == A_LIGHT_CONTINUE)
    BDPT_BODY_LIGHT_NEXT
#endif
    BDPT_ACTION(21, act == A_START_EYE) {  // eyeSubpathWalk prologue (bdpt.h:47-65)
        if (COUNT && fr.strategy != 2) cnt.m[0] = max(cnt.m[0], static_cast<uint32_t>(L.c.depth));  // the light walk's
        const f3 prim = L.c.Li;  // the primary hit's (t, u, v), kept since resolve(ST_PRIMARY)
        if (fr.strategy == 1) {  // LIGHT_TRACING: Li = Le at the primary hit (bdpt.h:231)
            const int mat = __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(L.c.prim_tri)).w);
            L.c.Li = ld3(bsdf_of(sc, mat).emission);
            act = A_FINISH;
            break;
        }
        const float cosCamera = dot(fwd, L.c.cam_d);
        const float d = div_w(fr.cam.vnear, cosCamera);
        const float t1Pdf = 1.f * div_w(d * d, cosCamera);
        L.c.tp = mk(1.f, 1.f, 1.f);
        L.c.vc = 0.f;
        L.c.vcm = static_cast<float>(fr.W * fr.H) * rcp_w(t1Pdf);
        L.c.depth = 1;
        L.c.pure = 1u;
        if (rr_on(fr)) L.c.rr = 1.f;  // rrProbability before the first vertex (bdpt.h:65)
        L.c.Li = mk(0.f, 0.f, 0.f);
        L.ray = Ray{cam_o, L.c.cam_d, 1.f, 1000.f};
        act = A_EYE_NEXT;
        if (1 < fr.rr_depth) {
            // The eye walk's first intersect (bdpt.h:70) re-traces render()'s
            // primary ray (bdpt.h:225): same ray, same scene, so the same
            // (accepted) hit. It is reused instead of traced again.
            shade_hit(sc, L.c.prim_tri, prim.y, prim.z, prim.x, L.ray.d, L.h);
            L.c.steps++;
            act = A_EYE_VERTEX;
        }
    } BDPT_END;
    BDPT_ACTION(22, act == A_EYE_VERTEX) {  // bdpt.h:73-136
        const float dist2 = L.h.dist * L.h.dist;
        BDPT_DIST_TO_GRAZE
        const float absCosIn = fabsf(L.h.wo.z);
        L.c.vcm *= div_w(dist2, absCosIn);
        L.c.vc *= rcp_w(absCosIn);
        const BsdfRecord& b = bsdf_of(sc, L.h.mat);
        const f3 emission = ld3(b.emission);  // getEmission = materials[matID].emission
        if (!is_zero(emission)) {
            const int eid = shape_emitter_of(sc, shape_id(L.h.shape));
            if (eid >= 0) {  // (the reference asserts otherwise, integrator.cpp:56)
                const EmitterRecord& e = emitter_of(sc, eid);
                const float emitterPdf = sc.inv_nemit;  // 1.f / nemit
                if (L.c.depth > 1) {
                    f3 contrib = ld3(e.radiance) * L.c.tp;
                    const float pA = rcp_w(e.area * emitterPdf);
                    const float camW = pA * L.c.vcm + (pA * kInvTwoPi) * L.c.vc;
                    const float mis = rcp_w(1.f + camW);
                    if (fr.strategy == 2) {  // PATH_TRACING (bdpt.h:110-113)
                        if (L.c.pure) L.c.Li = L.c.Li + contrib;
                    } else {
                        if (!L.c.pure) contrib = contrib * mis;
                        L.c.Li = L.c.Li + contrib;
                    }
                } else if (L.c.depth == 1) {
                    L.c.Li = L.c.Li + emission;
                }
            }
            act = A_FINISH;
            break;
        }
        if (rr_on(fr)) L.c.rr = rr_probability(fr, L.c.depth, L.c.tp);  // bdpt.h:129-134
        if (is_delta(b)) {
            act = A_EYE_CONTINUE;
            break;
        }
        L.c.pure = 0u;
        L.c.ci = 0;
        act = A_NEE;
    } BDPT_END;
    // The emitter sample (4 draws) of lightSubpathWalk (bdpt.h:162-163) and of
    // connectToLight (bdpt.h:376-381): selectEmitter + sampleEmitterPosition.
    int e_id = 0, e_graze = 0;
    float e_pdf = 0.f, e_pos_pdf = 0.f;
    f3 e_n = mk(0.f, 0.f, 0.f), e_p = e_n;
    BDPT_ACTION(23, act == A_START_LIGHT || act == A_NEE) {
        e_id = sample_emitter(sc, L.rng, e_pdf, e_n, e_p, e_pos_pdf, &e_graze);
    } BDPT_END;
    BDPT_ACTION(24, act == A_START_LIGHT) {  // lightSubpathWalk prologue (bdpt.h:158-182): 6 draws
        const EmitterRecord& e = emitter_of(sc, e_id);
        float areaPdf = e_pos_pdf;
        const f3 edir = uniform_hemisphere(next2(L.rng));
        float emissionPdf = kInvTwoPi * areaPdf;
        areaPdf *= e_pdf;
        emissionPdf *= e_pdf;
        f3 fs, ft;
        make_frame(e_n, fs, ft);
        L.ray = Ray{e_p, to_world(fs, ft, e_n, edir), kEpsilon, 3.402823466e+38f};
        L.h.n = e_n;  // the surface the first light ray leaves (cull_near_for); the walk's resolve overwrites L.h
#ifndef BDPT_EMIT_GRAZE
#define BDPT_EMIT_GRAZE 1  // 0: the emitter face's graze code is not used (A/B only)
#endif
        if (BDPT_EMIT_GRAZE) L.h.shape = e_graze;  // its graze code (the shape id is not read before the walk's resolve)
        if (BDPT_GRAZE_IN_DIST) L.h.dist = graze_threshold(e_graze);
        L.c.tp = (ld3(e.radiance) * edir.z) * rcp_w(emissionPdf);
        L.c.vc = edir.z * rcp_w(emissionPdf);
        L.c.vcm = div_w(areaPdf, emissionPdf);
        L.c.nl = 0;
        L.c.depth = 1;
        if (rr_on(fr)) L.c.rr = 1.f;  // bdpt.h:187
        if (edir.z <= 0.f) {  // bdpt.h:179-182 (the eye subpath follows)
            L.state = ST_DEFER;
            act = A_ISSUED;
        } else if (BDPT_SPLIT_CONTINUE) {  // the loop test of bdpt.h:188 here: its body runs earlier in the sweep
            L.state = walk_continues(L, fr) ? ST_LIGHT : ST_DEFER;
            act = A_ISSUED;
        } else {
            act = A_LIGHT_NEXT;
        }
    } BDPT_END;
    BDPT_ACTION(25, act == A_NEE) {  // connectToLight (bdpt.h:374-430): everything but the visibility test
        act = A_CONN;
        if (COUNT) cnt.t_step += 1u + (fr.strategy == 0 ? static_cast<uint32_t>(L.c.nl) : 0u);  // (Counts::q)
        const BsdfRecord& b = bsdf_of(sc, L.h.mat);
        const EmitterRecord& e = emitter_of(sc, e_id);
        f3 dir = L.h.p - e_p;
        const float d2 = dot(dir, dir);
        dir = dir * rsqrt_w(d2);
#if BDPT_CONN_EARLY_COS >= 2
        const float cosAtLight = dot(e_n, dir);
        const float cosAtEye = dot(-dir, L.h.n);  // = the frame's z component (to_local)
        if (cosAtLight <= 0.f || cosAtEye <= 0.f) break;
        const f3 wi = local_for(b, L.h.n, -dir);
#else
        const f3 wi = local_at(L.h.n, -dir);
        const float cosAtLight = dot(e_n, dir);
        const float cosAtEye = wi.z;
        if (cosAtLight <= 0.f || cosAtEye <= 0.f) break;
#endif
        const float pdf_w = div_w((e_pdf * e_pos_pdf) * d2, cosAtLight);
        const EvalPdfs ep = bsdf_eval_pdfs(b, wi, L.h.wo);
        const f3 Li = ((ep.f * rcp_w(pdf_w)) * L.c.tp) * ld3(e.radiance);
        if (is_zero(Li)) break;
        const float rrE = rr_on(fr) ? L.c.rr : 1.f;  // eyeVertex.rr (bdpt.h:410, :417)
        const float lightWeight = div_w(ep.fwd * rrE, pdf_w);
        const float eyePrevRev = ep.rev * rrE;
        const float eyeCurRev_a = cosAtEye * rcp_w(d2) * kInvTwoPi;
        const float eyeWeight = eyeCurRev_a * (L.c.vcm + eyePrevRev * L.c.vc);
        const float mis = rcp_w(lightWeight + 1.f + eyeWeight);
        const f3 pend = (fr.strategy == 0) ? Li * mis : Li;
        const Ray sr = shadow_ray(L.h.p, e_p);
        if (kTasks && task_push(L.c, fr, sr, vertex_nocull(L, sr.d), pend * fr.inv_spp, L.c.pixel, false, cnt))
            break;  // a helper walks it (act: A_CONN)
        L.c.pend = pend;
        L.ray = sr;
        L.state = ST_NEE;
        act = A_ISSUED;
    } BDPT_END;
#if !BDPT_SPLIT_CONTINUE
    BDPT_BODY_LIGHT_VERTEX
#endif
    }  // PART != 2
    if (PART == 1) return act;
    BDPT_ACTION(27, act == A_CONN) {  // connectVertices (bdpt.h:434-483) with light vertex ci
        act = A_EYE_CONTINUE;
        if (fr.strategy != 0) break;  // LIGHT/PATH_TRACING builds skip connections (bdpt.h:145)
        const BsdfRecord& be = bsdf_of(sc, L.h.mat);
        while (L.c.ci < L.c.nl) {
            const Vertex V = load_vertex(ls, L.c.ci);
            if (COUNT) cnt.c[5]++;
            f3 dir = L.h.p - V.p;
            const float invD2 = rcp_w(dot(dir, dir));
            dir = dir * sqrt_w(invD2);
#if BDPT_CONN_EARLY_COS >= 1
            // the frames' z components are dot(v, n) (to_local), so the
            // rejection test runs before the frames are built
            const float cosL = dot(dir, V.n), cosE = dot(-dir, L.h.n);
            if (cosL <= 0.f || cosE <= 0.f) {
                L.c.ci++;
                continue;
            }
            const BsdfRecord& bl = bsdf_of(sc, V.mat);
            const f3 wiL = local_for(bl, V.n, dir);  // Frame(n) is a pure function of n
            const f3 wiE = local_for(be, L.h.n, -dir);
#else
            const f3 wiL = local_at(V.n, dir);  // Frame(n) is a pure function of n
            const f3 wiE = local_at(L.h.n, -dir);
            const float cosL = wiL.z, cosE = wiE.z;
            if (cosL <= 0.f || cosE <= 0.f) {
                L.c.ci++;
                continue;
            }
            const BsdfRecord& bl = bsdf_of(sc, V.mat);
#endif
            const EvalPdfs eL = bsdf_eval_pdfs(bl, wiL, V.wo), eE = bsdf_eval_pdfs(be, wiE, L.h.wo);
            f3 Li = eL.f * eE.f;
            Li = Li * ((V.tp * L.c.tp) * invD2);
            const float rrL = rr_on(fr) ? V.rr : 1.f, rrE = rr_on(fr) ? L.c.rr : 1.f;  // bdpt.h:461-472
            const float eyePathRev_w = eL.fwd * rrL;
            const float lightPrevRev = eL.rev * rrL;
            const float lightPathRev_w = eE.fwd * rrE;
            const float eyePrevRev = eE.rev * rrE;
            const float lightPathRev_a = lightPathRev_w * cosL * invD2;
            const float eyePathRev_a = eyePathRev_w * cosE * invD2;
            const float lightWeight = lightPathRev_a * (V.vcm + lightPrevRev * V.vc);
            const float eyeWeight = eyePathRev_a * (L.c.vcm + eyePrevRev * L.c.vc);
            const float mis = rcp_w(lightWeight + 1.f + eyeWeight);
            const Ray sr = shadow_ray(L.h.p, V.p);
            if (kTasks && task_push(L.c, fr, sr, vertex_nocull(L, sr.d), (Li * mis) * fr.inv_spp, L.c.pixel, false, cnt)) {
                L.c.ci++;  // a helper walks it; the next light vertex now
                continue;
            }
            L.c.pend = Li * mis;
            L.ray = sr;
            L.state = ST_CONN;
            act = A_ISSUED;
            break;
        }
    } BDPT_END;
#if BDPT_SPLIT_CONTINUE
    BDPT_BODY_CONTINUE(A_EYE_CONTINUE, act == A_EYE_CONTINUE)
#else
    BDPT_BODY_CONTINUE(A_LIGHT_CONTINUE, act == A_LIGHT_CONTINUE || act == A_EYE_CONTINUE)
    BDPT_BODY_LIGHT_NEXT
#endif
    BDPT_ACTION(30, act == A_EYE_NEXT) {
        if (walk_continues(L, fr)) {
            L.state = ST_EYE;
            act = A_ISSUED;
        } else {
            act = A_FINISH;
        }
    } BDPT_END;
    BDPT_ACTION(31, act == A_FINISH) {
        finish<COUNT>(L, fr, fb, cnt);
        act = A_DONE;
    } BDPT_END;
    return act;
}
#undef BDPT_ACTION
#undef BDPT_END
#undef BDPT_BODY_LIGHT_VERTEX
#undef BDPT_BODY_CONTINUE
#undef BDPT_BODY_LIGHT_NEXT

#ifndef BDPT_SCAN_BITS
#define BDPT_SCAN_BITS 1  // conn_batch's prefix sum by ballots per bit of the counts (0: six __shfl_up steps)
#endif
#if BDPT_HELP && !BDPT_SAMPLER_STATE
// connectVertices of every owner lane that reached A_CONN in this shading step
// (bdpt.h:434-483, all its remaining light vertices), flattened over the wave:
// task i of the prefix sum over the owners' counts runs on lane i mod 64, with the
// owner's eye vertex from its registers (ds_bpermute), its cold state from LDS and
// its light vertex from its slot; each connection's shadow ray is pushed to the
// wave's ring like the serial body's (the same arithmetic in the same order). Called
// by all 64 lanes between advance<.., 1> and advance<.., 2>; owners leave with
// ci = nl. When the ring cannot take every connection, nothing is batched and the
// owners connect one by one in advance<.., 2> (which falls back to tracing them).
template <bool COUNT>
__device__ __forceinline__ void conn_batch(Lane& L, bool owner, const DevScene& sc, const DevFrame& fr,
                                           const LightStore& ls, Counts& cnt) {
    const int k = owner ? L.c.nl - L.c.ci : 0;
    const uint64_t om = __ballot(k > 0);
    if (!om) return;
    const int me = static_cast<int>(opaque_tid() & 63);
#if BDPT_SCAN_BITS
    // exclusive prefix sum of k over the wave, one bit of k at a time: lanes below
    // with the bit set (mbcnt of a ballot) times its weight — no LDS round trips
    int excl = 0, total = 0;
    for (int b = 0, rest = k; __ballot(rest != 0); b++, rest >>= 1) {  // (wave-uniform)
        const uint64_t m = __ballot(rest & 1);
        excl += lanes_below(m) << b;
        total += popc64(m) << b;
    }
#else
    int incl = k;  // inclusive prefix sum of k over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int t = __shfl_up(incl, off);
        if (me >= off) incl += t;
    }
    const int total = lane_val(incl, 63), excl = incl - k;
#endif
    {
        const TaskCtl ctl = task_ctl(L.c);
        if (static_cast<uint32_t>(total) > fr.task_cap - (*ctl.tail - *ctl.head)) return;
    }
    LaneCold* const wave_cold = &L.c - me;
    for (int r0 = 0; r0 < total; r0 += 64) {  // (wave-uniform)
        const int i = r0 + me;
        int o = -1, j = 0;
        for (uint64_t m = om; m; m &= m - 1) {  // the owner of task i (scalar loop over the owners)
            const int b = __ffsll(static_cast<unsigned long long>(m)) - 1;
            const int eb = __builtin_amdgcn_readlane(excl, b), kb = __builtin_amdgcn_readlane(k, b);
            if (i >= eb && i < eb + kb) o = b, j = i - eb;
        }
        const int src = o >= 0 ? o : me;
        const f3 hp = mk(__shfl(L.h.p.x, src), __shfl(L.h.p.y, src), __shfl(L.h.p.z, src));
        const f3 hn = mk(__shfl(L.h.n.x, src), __shfl(L.h.n.y, src), __shfl(L.h.n.z, src));
        const f3 hwo = mk(__shfl(L.h.wo.x, src), __shfl(L.h.wo.y, src), __shfl(L.h.wo.z, src));
        const int hmat = __shfl(L.h.mat, src), hshape = __shfl(L.h.shape, src);
        if (o < 0) continue;
        const LaneCold& oc = wave_cold[o];
        const Vertex V = load_vertex_at(ls.at_tid(oc.ci + j, (opaque_tid() & ~63u) + static_cast<uint32_t>(o)));
        if (COUNT) cnt.c[5]++;
        f3 dir = hp - V.p;
        const float invD2 = rcp_w(dot(dir, dir));
        dir = dir * sqrt_w(invD2);
        const float cosL = dot(dir, V.n), cosE = dot(-dir, hn);
        if (cosL <= 0.f || cosE <= 0.f) continue;
        const BsdfRecord& be = bsdf_of(sc, hmat);
        const BsdfRecord& bl = bsdf_of(sc, V.mat);
        const f3 wiL = local_for(bl, V.n, dir);
        const f3 wiE = local_for(be, hn, -dir);
        const EvalPdfs eL = bsdf_eval_pdfs(bl, wiL, V.wo), eE = bsdf_eval_pdfs(be, wiE, hwo);
        f3 Li = eL.f * eE.f;
        Li = Li * ((V.tp * oc.tp) * invD2);
        const float eyePathRev_w = eL.fwd;  // (rr = 1: these builds are NO_RR = 1, bdpt.h:461-472)
        const float lightPrevRev = eL.rev;
        const float lightPathRev_w = eE.fwd;
        const float eyePrevRev = eE.rev;
        const float lightPathRev_a = lightPathRev_w * cosL * invD2;
        const float eyePathRev_a = eyePathRev_w * cosE * invD2;
        const float lightWeight = lightPathRev_a * (V.vcm + lightPrevRev * V.vc);
        const float eyeWeight = eyePathRev_a * (oc.vcm + eyePrevRev * oc.vc);
        const float mis = rcp_w(lightWeight + 1.f + eyeWeight);
        const Ray sr = shadow_ray(hp, V.p);
#if BDPT_GRAZE_IN_DIST
#error "conn_batch: BDPT_GRAZE_IN_DIST keeps the threshold in Hit::dist"
#endif
        task_push(L.c, fr, sr, graze_exempt(sr.d, hn, hshape), (Li * mis) * fr.inv_spp, oc.pixel, false, cnt);
    }
    if (k > 0) L.c.ci = L.c.nl;
}
#endif

// Pixel and Sampler seed of sample `s` of the shard: seed_base + p * spp + k
// (the per-(pixel, sample) convention of SURVEY §8c on renderer.cpp:155).
__device__ __forceinline__ uint32_t sample_seed(uint64_t s, const DevFrame& fr, int& pixel) {
    const uint64_t per_row = static_cast<uint64_t>(fr.W) * fr.spp;
    uint64_t lr = s / per_row;
    const uint64_t q = s % per_row;
    if (fr.row_order) lr = static_cast<uint64_t>(((const gbl_i32*)fr.row_order)[lr]);  // bdpt_set_row_order
    const int j = static_cast<int>(q / fr.spp), k = static_cast<int>(q % fr.spp);
    const int row = fr.row_offset + static_cast<int>(lr) * fr.row_stride;
    pixel = row * fr.W + j;
    return fr.seed_base + static_cast<uint32_t>(pixel) * static_cast<uint32_t>(fr.spp) + static_cast<uint32_t>(k);
}

// Starts sample `s` of the shard on this lane: seed, camera ray, primary query.
// x397 = mt_x397(seed) when the caller precomputed it (HAVE_X397).
template <bool HAVE_X397 = false>
__device__ __forceinline__ void start_sample(Lane& L, uint64_t s, const DevFrame& fr, uint32_t x397 = 0) {
    int pixel;
    const uint32_t seed = sample_seed(s, fr, pixel);
    L.c.pixel = pixel;
    if (HAVE_X397) mt_seed_with(L.rng, seed, x397);
    else mt_seed(L.rng, seed);
    L.c.cam_d = camera_dir(fr, L.c.pixel, L.rng);
    L.ray = Ray{mk(fr.cam_o[0], fr.cam_o[1], fr.cam_o[2]), L.c.cam_d, 1.f, 1000.f};
    L.c.Li = mk(0.f, 0.f, 0.f);
    L.c.steps = 0;
    L.state = ST_PRIMARY;
}

__device__ __forceinline__ bool is_shadow_state(uint32_t st) { return st == ST_SPLAT || st == ST_NEE || st == ST_CONN; }

// The near-cull threshold of the lane's pending query (kGrazeCos, graze_exempt,
// bdpt_device.hpp): none for a query that leaves the current vertex (or, for the
// first light-subpath ray, the emitter: A_START_LIGHT puts its normal and face
// code in L.h) nearly parallel to its triangle's plane; camera queries keep it.
__device__ __forceinline__ bool vertex_nocull(const Lane& L, f3 d) {
#if BDPT_GRAZE_IN_DIST
    return fabsf(dot(d, L.h.n)) < L.h.dist;
#else
    return graze_exempt(d, L.h.n, L.h.shape);
#endif
}
__device__ __forceinline__ float cull_near_for(const Lane& L) {
    const uint32_t st = L.state;
    if (st == ST_PRIMARY || st == ST_SPLAT) return kCullNear;
#if BDPT_GRAZE_IN_DIST
    return fabsf(dot(L.ray.d, L.h.n)) < L.h.dist ? kNoCullNear : kCullNear;
#else
    return graze_exempt(L.ray.d, L.h.n, L.h.shape) ? kNoCullNear : kCullNear;
#endif
}

// Applies the result of the lane's pending query (closest hit: leaf-order
// triangle index res >= 0 with t, u, v; shadow ray: res >= 0 = occluded) and
// returns the action the state machine continues with.
template <bool COUNT>
__device__ __forceinline__ uint32_t resolve(Lane& L, int res, float t, float u, float v, const DevScene& sc,
                                            const DevFrame& fr, float* __restrict__ fb, Counts& cnt) {
    const bool any = is_shadow_state(L.state);
    const bool shaded = kTasks && res == kResShaded;  // applied in the walk loop already (help_compact)
    bool hit = res >= 0 || shaded;
    if (hit && !any && !shaded) hit = (t <= L.ray.max_t && t >= L.ray.min_t);  // accel.h:133
    // The primary hit is shaded later, by the eye walk's first vertex (A_START_EYE
    // keeps its (t, u, v)); the light walk overwrites L.h before reading it.
    if (hit && !any && !shaded && L.state != ST_PRIMARY) shade_hit(sc, res, u, v, t, L.ray.d, L.h);
    uint32_t act;
    switch (L.state) {
        case ST_PRIMARY:
            if (!hit) act = A_FINISH;
            else {
                if (!shaded) {
                    L.c.prim_tri = res;
                    L.c.Li = mk(t, u, v);
                }
                act = (fr.strategy == 2) ? A_START_EYE : A_START_LIGHT;
            }
            break;
        case ST_LIGHT: act = hit ? A_LIGHT_VERTEX : A_START_EYE; break;
        case ST_SPLAT:
            if (!hit) {
                if (COUNT) cnt.c[6]++;
                splat_add(fb, L.c.pend_px, L.c.pend);
            }
            act = A_LIGHT_CONTINUE;
            break;
        case ST_EYE: act = hit ? A_EYE_VERTEX : A_FINISH; break;
        case ST_NEE:
            if (!hit) L.c.Li = L.c.Li + L.c.pend;
            act = A_CONN;
            break;
        case ST_CONN:
            if (!hit) L.c.Li = L.c.Li + L.c.pend;
            L.c.ci++;
            act = A_CONN;
            break;
        case ST_DEFER: act = A_START_EYE; break;
        default: act = A_DONE;
    }
    // A state-machine bug must not hang the GPU: bound the queries per sample.
    if (++L.c.steps > (rr_on(fr) ? (1 << 30) : max_steps_per_sample(fr.rr_depth)) && act != A_FINISH) act = A_FINISH;
    return act;
}

// BDPT_HELP: an own closest-hit result applied where resolve() would apply it
// (accel.h:133's range test, the primary hit's (t, u, v) into the cold state, or
// the hit shaded into L.h), so the lane's ray registers are free for a helper walk;
// res becomes kResShaded (a hit) or -1 (a miss).
__device__ __forceinline__ void help_compact(Lane& L, int& res, float t, float u, float v, const DevScene& sc) {
    const uint32_t st = L.state;
    if (res < 0 || !(st == ST_PRIMARY || st == ST_LIGHT || st == ST_EYE)) return;
    if (!(t <= L.ray.max_t && t >= L.ray.min_t)) {
        res = -1;
        return;
    }
    if (st == ST_PRIMARY) {
        L.c.prim_tri = res;
        L.c.Li = mk(t, u, v);
    } else {
        shade_hit(sc, res, u, v, t, L.ray.d, L.h);
    }
    res = kResShaded;
}

// Schedules without an overlapped walk run a deferred action at once.
template <bool COUNT>
__device__ __forceinline__ void run_deferred(Lane& L, const DevScene& sc, const DevFrame& fr, float* __restrict__ fb,
                                             const LightStore& ls, Counts& cnt) {
    while (L.state == ST_DEFER)
        advance<COUNT>(L, resolve<COUNT>(L, -1, 0.f, 0.f, 0.f, sc, fr, fb, cnt), sc, fr, fb, ls, cnt);
}

// out: kCounters sums, then the 3 maxima of Counts::m.
__device__ __forceinline__ void flush_counts(const Counts& cnt, unsigned long long* out) {
    for (int i = 0; i < kCounters; i++) {
        unsigned long long v = cnt.c[i];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0 && v) gadd(out + i, v);
    }
    for (int i = 0; i < 3; i++) {
        uint32_t v = cnt.m[i];
        for (int off = 32; off > 0; off >>= 1) v = max(v, static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), off)));
        if ((threadIdx.x & 63) == 0 && v) gmax(out + kCounters + i, static_cast<unsigned long long>(v));
    }
    for (int i = 0; i < 4; i++) {
        unsigned long long v = cnt.q[i];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0 && v) gadd(out + kCounters + 3 + i, v);
    }
}

}  // namespace dev
}  // namespace bdpt
