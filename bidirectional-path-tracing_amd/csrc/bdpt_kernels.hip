// HIP kernels for the MI355X (gfx950) BDPT hot path.
//
// bdpt_frame_kernel — persistent megakernel with a per-lane state machine.
// One lane owns one camera sample (pixel, k) at a time and runs
// BDPTIntegrator::render (reference src/integrators/bdpt.h:219-241) as a
// sequence of ray queries: every loop iteration performs exactly ONE BVH query
// per lane (a closest hit for the light / eye subpath walks, or a shadow ray for
// a camera splat, a next-event estimation or a vertex connection), then
// advances the lane's state until it needs its next query. Keeping the
// traversal in a single place keeps register pressure bounded and lets lanes
// that are at different points of their paths share the traversal loop. Lanes
// that finish a sample immediately pull a new one (one atomic per wave per
// refill), so no lane idles while its wave still has work.
//
// Light vertices live in an HBM scratch buffer in lane-contiguous layout; the
// traversal stack of every lane lives in LDS.
//
// bdpt_sample_kernel — a single (ray, sampler) call for the drop-in
// Integrator::render(const Ray&, Sampler&) entry point (same state machine,
// one lane).
#include <hip/hip_runtime.h>

#ifndef BDPT_BSDF_TABLE
#if BDPT_SAMPLER_STATE
#define BDPT_BSDF_TABLE 2  // one wave: the table's place is chosen per launch
#else
#define BDPT_BSDF_TABLE 0  // frame kernels: LDS (bdpt_kernels_hbm.hip is the HBM build)
#endif
#endif

// The frame kernels without Russian roulette weight paths with the hardware
// reciprocal / square root (device_math.hpp rcp_w): the paths stay the
// reference's bit for bit, contributions move by a few ulp. The Russian-roulette
// build (its throughput steers the roulette) and the single-sample build keep the
// IEEE operations.
#ifndef BDPT_FAST_WEIGHTS
#if !(defined(BDPT_SAMPLER_STATE) && BDPT_SAMPLER_STATE) && !(defined(BDPT_RR) && BDPT_RR)
#define BDPT_FAST_WEIGHTS 1
#endif
#endif

// Shadow-ray tasks walked by waiting lanes (bdpt_path.hpp task_push): only the
// overlapped frame kernels without Russian roulette build them (round 6: Caustic
// 512^2 x 256 288.5 -> 323.4 Msamples/s, synth1m 1024^2 x 64 203.2 -> 218.9,
// HardLight 512^2 x 256 1478.5 -> 1485.1).
#ifndef BDPT_HELP
#define BDPT_HELP 1
#endif
#if (defined(BDPT_RR) && BDPT_RR) || (defined(BDPT_SAMPLER_STATE) && BDPT_SAMPLER_STATE) || \
    (defined(BDPT_OVERLAP) && !BDPT_OVERLAP)
#undef BDPT_HELP
#define BDPT_HELP 0
#endif

// The eye-estimate slots (bdpt_path.hpp) are claimed with the 64-sample chunks.
#if defined(BDPT_SEED_CHUNK) && !BDPT_SEED_CHUNK && !defined(BDPT_EYE_SLOTS)
#define BDPT_EYE_SLOTS 0
#endif
#include "bdpt_path.hpp"

namespace bdpt {
namespace dev {

#ifndef BDPT_WAVES_PER_EU
#define BDPT_WAVES_PER_EU 4  // waves per SIMD the register allocator must leave room for
#endif
constexpr int kBlock = 256;
#ifndef BDPT_OVERLAP
#define BDPT_OVERLAP 1  // overlapped walk / shade schedule in the megakernel (0: one query then shade, in lockstep)
#endif
#ifndef BDPT_TRAV_SPLIT
#define BDPT_TRAV_SPLIT 8  // > 0: leaf and interior-node steps in separate iterations (leaf step if 4 * leaf lanes >= SPLIT * node lanes; round 5: 6 over 8, then 8 over 6 / 10 / 12 once node steps also follow leaf iterations)
#endif
#ifndef BDPT_SEED_CHUNK
#define BDPT_SEED_CHUNK 1  // refill from per-wave chunks of 64 samples seeded together (0: per-refill seeding)
#endif
#ifndef BDPT_WALK_UNROLL
#define BDPT_WALK_UNROLL 1  // extra interior-node steps per walk iteration (measured: 0: 201.7, 1: 203.6)
#endif
#ifndef BDPT_SHADE_READY
#define BDPT_SHADE_READY 44  // lanes with a finished query that trigger the wave's shading step (round 5 re-sweep: 44 over 48)
#endif
#ifndef BDPT_TAIL_SHADE
#define BDPT_TAIL_SHADE 2  // once a wave has no samples left to claim: 1 shade at 1 ready lane, 2 at BDPT_TAIL_FRAC / 8 of its busy lanes
#endif
#ifndef BDPT_TAIL_FRAC
#define BDPT_TAIL_FRAC 6  // (measured, 512x512x256 1/8 shard: end tail 2.19 -> 1.93 ms, steady state unchanged)
#endif
#ifndef BDPT_EXPRESS_DEPTH
#define BDPT_EXPRESS_DEPTH 512  // Russian-roulette build: a subpath this deep puts its wave in express mode (below; DevFrame::express_depth, set per render)
#endif
#ifndef BDPT_ROOT_LDS
#define BDPT_ROOT_LDS 1  // 1: the traversal root and its interior children in LDS, tested when a walk begins (RootLds; measured +1.6 %)
#endif

#ifndef BDPT_COOP_ALONE
#define BDPT_COOP_ALONE (BDPT_RR == 1 && !BDPT_SAMPLER_STATE)  // a lone trapped walk walked by its whole wave (below)
#endif
#ifndef BDPT_COOP_MAX
#define BDPT_COOP_MAX 4  // express waves with up to this many busy lanes walk their closest hits in turn with the whole wave
#endif
#ifndef BDPT_RR_DIAG
#define BDPT_RR_DIAG 1
#endif
#ifndef BDPT_COOP_BATCH
#define BDPT_COOP_BATCH 0  // the megakernel's wave walk tests leaves with wleaf_tests (coop_leaf's batched loads cost spills)
#endif
#ifndef BDPT_EXPRESS_WALK
#define BDPT_EXPRESS_WALK 0  // 1: a lone trapped lane's delta chain out of line (express_walk; 1.5 % faster on the trapped chain, +49 VGPR spills in the RR build)
#endif
#if BDPT_RR == 1 && !BDPT_SAMPLER_STATE && BDPT_EXPRESS_WALK
// Russian roulette: a subpath trapped by total internal reflection bounces
// between delta surfaces for up to millions of steps, each a
// closest-hit walk plus the sweep's work for a delta vertex. Once its wave holds
// nothing else (express mode with one busy lane) those bounces run here, back to
// back: the walk, then exactly what the sweep does at a delta, non-emitting
// vertex — the vertex update (bdpt.h:73-136 / :193-209, no connection: delta),
// ContinuePathRandomWalk (bdpt.h:243-291), the loop test (bdpt.h:68 / :188) —
// until the chain ends. Out of line: the loop keeps only its own state in
// registers, where the megakernel's sweep spills (a lone lane waits out every
// scratch access). Returns true with the result (res, t, u, v) of a query the
// sweep resolves (a miss, a non-delta or emitting hit); false when the walk
// ended here (light: ST_DEFER, the eye subpath next; eye: the sample finished).
__device__ __noinline__ bool express_walk(Lane& Lcaller, const DevScene& sc, const DevFrame& fr, float* __restrict__ fb,
                                          const Stack stk, int& res, float& rt, float& ru, float& rv) {
    Counts cnt;  // (not a counting pass)
    // the lane's register state as locals (the caller's copy is written back on return)
    Lane L(Lcaller.c);
    L.rng = Lcaller.rng, L.state = Lcaller.state, L.ray = Lcaller.ray, L.h = Lcaller.h;
    struct WriteBack {
        Lane& to;
        const Lane& from;
        __device__ ~WriteBack() { to.rng = from.rng, to.state = from.state, to.ray = from.ray, to.h = from.h; }
    } wb{Lcaller, L};
    for (;;) {
        const bool light = L.state == ST_LIGHT;
        float t = 0.f, u = 0.f, v = 0.f;
        const int r = traverse<false, false>(sc, L.ray, false, stk, t, u, v, cnt, cull_near_for(L));
        const bool hit = r >= 0 && t <= L.ray.max_t && t >= L.ray.min_t;  // accel.h:133
        const BsdfRecord* b = nullptr;
        if (hit) b = &bsdf_of(sc, __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(r)).w));
        if (!hit || !is_delta(*b) || !is_zero(ld3(b->emission)) || L.c.steps + 1 > (1 << 30)) {
            res = r, rt = t, ru = u, rv = v;  // the sweep resolves it
            return true;
        }
        ++L.c.steps;  // resolve(): one more query, the hit shaded
        shade_hit(sc, r, u, v, t, L.ray.d, L.h);
        const float dist2 = L.h.dist * L.h.dist;
        BDPT_DIST_TO_GRAZE
        const float absCosIn = fabsf(L.h.wo.z);
#if BDPT_RING_AHEAD
        if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && fr.diag) gadd(fr.diag + kDiagErrors, 1ull);
#endif
        L.c.vcm *= div_cr(dist2, absCosIn);
        L.c.vc *= rcp_cr(absCosIn);
        L.c.rr = rr_probability(fr, L.c.depth, L.c.tp);  // bdpt.h:129-134 / :201-204
        const bool more = continue_walk(*b, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, L.c.rr);
        if (!more || !walk_continues(L, fr)) {
            if (light) L.state = ST_DEFER;  // the eye subpath starts next step
            else finish<false>(L, fr, fb, cnt);  // L.state = ST_IDLE
            return false;
        }
    }
}
#endif

#ifndef BDPT_PARK
#define BDPT_PARK (BDPT_RR == 1 && !BDPT_SAMPLER_STATE)  // the Russian-roulette continuation pass (below; opt-in per render)
#endif
#if BDPT_PARK
// Russian-roulette continuation pass. A subpath trapped in glass by total
// internal reflection is a serial chain of up to millions of delta bounces
// (DESIGN.md §8); in the megakernel each of them is one lane's walk at ~30
// dependent steps. A lane whose light or eye walk passes fr.park_depth bounces
// saves its sample (registers and cold state; its light vertices and MT19937
// ring stay in its slot) and stops taking samples; after the frame, the chain
// kernel continues every saved sample with one wave per sample — the closest
// hit walked by all 64 lanes (coop_closest), the delta bounce itself on lane 0
// — until the chain reaches a vertex the megakernel must shade (a miss, a
// non-delta or emitting hit) or the subpath ends; a resume launch of the
// megakernel on the same grid then continues each sample in its own slot. The
// same functions in the same order (express_walk's bounce), so the same bits.
constexpr uint32_t kParkWords = kParkSlotWords;
enum : uint32_t {
    kParkStatus = 0,        // 0 none, 1 parked, 2 returned by the chain kernel
    kParkResumeDepth = 1,   // the subpath depth at the last resume (a resumed walk parks again D bounces later)
    kParkRng = 2,           // LazyMT (4)
    kParkState = 6,
    kParkRay = 7,           // o, d, min_t, max_t (8)
    kParkHit = 15,          // p, wo, n, dist, mat, shape (12)
    kParkCold = 27,         // LaneCold (23)
};
static_assert(kParkCold + sizeof(LaneCold) / 4 <= kParkWords, "park record");
__device__ __forceinline__ uint32_t* park_record(const DevFrame& fr, uint32_t slot) {
    return fr.park + static_cast<size_t>(slot) * kParkWords;
}
__device__ __forceinline__ uint32_t* park_list(const DevFrame& fr, uint32_t nslots) {
    return fr.park + static_cast<size_t>(nslots) * kParkWords;
}
__device__ __forceinline__ void park_save(uint32_t* rec, const Lane& L) {
    const uint32_t w[kParkCold - kParkRng] = {
        L.rng.a0, L.rng.a1, L.rng.b, L.rng.n, L.state,
        __float_as_uint(L.ray.o.x), __float_as_uint(L.ray.o.y), __float_as_uint(L.ray.o.z),
        __float_as_uint(L.ray.d.x), __float_as_uint(L.ray.d.y), __float_as_uint(L.ray.d.z),
        __float_as_uint(L.ray.min_t), __float_as_uint(L.ray.max_t),
        __float_as_uint(L.h.p.x), __float_as_uint(L.h.p.y), __float_as_uint(L.h.p.z),
        __float_as_uint(L.h.wo.x), __float_as_uint(L.h.wo.y), __float_as_uint(L.h.wo.z),
        __float_as_uint(L.h.n.x), __float_as_uint(L.h.n.y), __float_as_uint(L.h.n.z),
        __float_as_uint(L.h.dist), static_cast<uint32_t>(L.h.mat), static_cast<uint32_t>(L.h.shape)};
    gbl_u32* const g = (gbl_u32*)rec;
#pragma unroll
    for (uint32_t k = 0; k < kParkCold - kParkRng; k++) g[kParkRng + k] = w[k];
    const uint32_t* c = reinterpret_cast<const uint32_t*>(&L.c);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(LaneCold) / 4; k++) g[kParkCold + k] = c[k];
}
__device__ __forceinline__ void park_restore(const uint32_t* rec, Lane& L) {
    const gbl_u32* const g = (const gbl_u32*)rec;
    L.rng = LazyMT{g[kParkRng], g[kParkRng + 1], g[kParkRng + 2], g[kParkRng + 3]};
    L.state = g[kParkState];
    const float* r = reinterpret_cast<const float*>(rec + kParkRay);
    L.ray = Ray{mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], r[7]};
    const float* h = reinterpret_cast<const float*>(rec + kParkHit);
    L.h.p = mk(h[0], h[1], h[2]), L.h.wo = mk(h[3], h[4], h[5]), L.h.n = mk(h[6], h[7], h[8]);
    L.h.dist = h[9], L.h.mat = static_cast<int>(g[kParkHit + 10]), L.h.shape = static_cast<int>(g[kParkHit + 11]);
    uint32_t* c = reinterpret_cast<uint32_t*>(&L.c);
#pragma unroll
    for (uint32_t k = 0; k < sizeof(LaneCold) / 4; k++) c[k] = g[kParkCold + k];
}
// The lane's sample leaves the megakernel here (the query it was about to walk
// is the chain kernel's first).
__device__ __forceinline__ bool park_lane(const DevFrame& fr, uint32_t nslots, uint32_t slot, const Lane& L) {
    uint32_t* const rec = park_record(fr, slot);
    if ((fr.park_flags & kParkResume) && !(L.c.depth > static_cast<int>(((const gbl_u32*)rec)[kParkResumeDepth]) + fr.park_depth))
        return false;  // resumed: D more bounces first
    park_save(rec, L);
    ((gbl_u32*)rec)[kParkStatus] = 1u;
    uint32_t* const list = park_list(fr, nslots);
    const uint32_t k = gadd(list, 1u);
    ((gbl_u32*)list)[1 + k] = slot;
    if (fr.diag) gadd(fr.diag + kDiagParked, 1ull);
    return true;
}
#define BDPT_BUSY(st) ((st) != ST_IDLE && (st) != ST_PARKED)
#else
#define BDPT_BUSY(st) ((st) != ST_IDLE)
#endif

#if BDPT_RR == 1 && !BDPT_SAMPLER_STATE && BDPT_EXPRESS_CHAIN == 2
// The lone long walk's chain of delta bounces (express mode, one busy lane b): each
// closest hit walked by the whole wave (coop_closest), the bounce itself on lane b,
// back to back until the chain reaches a vertex the sweep must shade. Out of line,
// called by all 64 lanes, so the megakernel's register allocation is not sized for
// it. Returns -1 with the last walk's result in (t, r, u, v, ok) for the sweep; 0 when
// the chain ended here (lane b: ST_DEFER or finished); 2 when lane b's next query
// must begin at the loop top (the reference's tree, or a culled root).
template <bool SLACK>
__device__ __noinline__ int express_chain(Lane& Lcaller, int b, RayInv& ri_caller, const DevScene& sc,
                                          const DevFrame& fr, float* __restrict__ fb, const TravScene& tsc,
                                          uint2* stack_base, const RootLds* coop_rl, float& t, int& r, float& u,
                                          float& v, bool& ok) {
    Counts cnt;  // (not a counting pass)
    Lane L(Lcaller.c);
    L.rng = Lcaller.rng, L.state = Lcaller.state, L.ray = Lcaller.ray, L.h = Lcaller.h;
    RayInv ri = ri_caller;
    const int me = static_cast<int>(__lane_id());
    const CoopStack cs{stack_base, kBlock};
    int bounced = -1;
    for (;;) {
        Ray q;
        q.o = mk(lane_val(L.ray.o.x, b), lane_val(L.ray.o.y, b), lane_val(L.ray.o.z, b));
        q.d = mk(lane_val(L.ray.d.x, b), lane_val(L.ray.d.y, b), lane_val(L.ray.d.z, b));
        q.min_t = lane_val(L.ray.min_t, b), q.max_t = lane_val(L.ray.max_t, b);
        RayInv qi;
        qi.inv = mk(lane_val(ri.inv.x, b), lane_val(ri.inv.y, b), lane_val(ri.inv.z, b));
        qi.near = lane_val(ri.near, b);
        qi.fast = true;
        const float guess = BDPT_GRAZE_IN_DIST ? -1.f : lane_val(L.h.dist, b);
        r = -1;
        ok = true;
        for (int pass = guess > 0.f ? 0 : 1; pass < 2 && r < 0 && ok; pass++) {
            const float bound = pass == 0 ? 2.f * guess : q.max_t;
            ok = coop_closest<SLACK, BDPT_COOP_BATCH>(tsc, q, qi, bound, cs, 64 * kLdsStack, t, r, u, v, nullptr, coop_rl);
        }
        if (!ok) break;
        int more = -1;
        if (me == b && r >= 0 && t <= L.ray.max_t && t >= L.ray.min_t) {  // accel.h:133
            const BsdfRecord& bb = bsdf_of(sc, __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(r)).w));
            if (is_delta(bb) && is_zero(ld3(bb.emission)) && L.c.steps + 1 <= (1 << 30)) {
                ++L.c.steps;  // resolve(): one more query, the hit shaded
                shade_hit(sc, r, u, v, t, L.ray.d, L.h);
                const float dist2 = L.h.dist * L.h.dist;
                BDPT_DIST_TO_GRAZE
                const float absCosIn = fabsf(L.h.wo.z);
#if BDPT_RING_AHEAD
                if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && fr.diag) gadd(fr.diag + kDiagErrors, 1ull);
#endif
                L.c.vcm *= div_w(dist2, absCosIn);  // bdpt.h:193-209 / :73-136 (no connection at a delta vertex)
                L.c.vc *= rcp_w(absCosIn);
                L.c.rr = rr_probability(fr, L.c.depth, L.c.tp);
                const bool light = L.state == ST_LIGHT;
                const bool cont = continue_walk(bb, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, L.c.rr);
                if (cont && walk_continues(L, fr)) {  // bdpt.h:188 / :68
                    ri = ray_inv(L.ray, cull_near_for(L));
                    more = ri.fast && !far_origin(sc, L.ray.o) && !(L.ray.min_t > L.ray.max_t) ? 1 : 2;
                } else {
                    if (light) L.state = ST_DEFER;  // the eye subpath starts next step
                    else finish<false>(L, fr, fb, cnt);  // L.state = ST_IDLE
                    more = 0;
                }
            }
        }
        more = lane_val(more, b);
        if (more == 1) continue;
        bounced = more;
        break;
    }
    Lcaller.rng = L.rng, Lcaller.state = L.state, Lcaller.ray = L.ray, Lcaller.h = L.h;
    ri_caller = ri;
    return bounced;
}
#endif

// One query for the lane's pending state, then the state advance.
template <bool FULL, bool COUNT>
__device__ __forceinline__ void step(Lane& L, const DevScene& sc, const DevFrame& fr, float* __restrict__ fb,
                                     const LightStore& ls, const Stack& stk, Counts& cnt) {
    const bool any = is_shadow_state(L.state), query = L.state != ST_DEFER;
    if (COUNT && query) cnt.c[any ? 1 : 0]++;
    float t = 0.f, u = 0.f, v = 0.f;
    const uint64_t c0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    const int res = query ? traverse<FULL, COUNT>(sc, L.ray, any, stk, t, u, v, cnt, cull_near_for(L)) : -1;
    const uint64_t c1 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
#if BDPT_DEEP_RNG && BDPT_RING_AHEAD
    if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && fr.diag) gadd(fr.diag + kDiagErrors, 1ull);
#endif
    const uint32_t act = resolve<COUNT>(L, res, t, u, v, sc, fr, fb, cnt);
    advance<COUNT>(L, act, sc, fr, fb, ls, cnt);
    if (COUNT && first_active_lane()) {  // wave clocks in traversal / in the state advance
        const uint64_t c2 = __builtin_amdgcn_s_memtime();
        cnt.c[12] += static_cast<uint32_t>(c1 - c0);
        cnt.c[13] += static_cast<uint32_t>(c2 - c1);
    }
}

#if !BDPT_SAMPLER_STATE
// Kernel parameters live in a small device buffer; the loop re-derives its
// pointer to them every iteration (through an empty asm) so the compiler loads
// the rarely used camera / frame constants at their point of use instead of
// pinning ~100 of them in SGPRs for the whole persistent loop (which spilled).
struct KParams {
    DevScene sc;
    DevFrame fr;
    float* fb;
    float* lv;
    uint2* gstack;  // traversal-stack overflow, (depth - kLdsStack) entries per slot
    uint32_t nslots;
    unsigned long long* work;
    unsigned long long* counters;
};

// SLACK: interior boxes with slab_fast's ambiguity slack (DevScene::node_slack,
// decided per render on the host); a template parameter so the node step of
// the walk loop carries no branch on it.
#ifndef BDPT_UNROLL_ANY
#define BDPT_UNROLL_ANY 1  // the extra node step also after a leaf iteration, for lanes that popped to an interior node (with split 8: Caustic +1.0 %, HardLight +1.8 %, synth1m +1.0 %)
#endif
#ifndef BDPT_COOP_GROUPS
#define BDPT_COOP_GROUPS 1  // express waves with 2-4 long walks walk them at once in groups of 32 / 16 lanes (coop_closest_groups; RR Caustic frames 42.7-45.2 s vs 43.8-54.0)
#endif
#ifndef BDPT_HELP_BATCH
#define BDPT_HELP_BATCH 1  // BDPT_HELP: the shading step's connections flattened over the wave (conn_batch; serial: 283.0 vs 322.8)
#endif
#if !BDPT_HELP
#undef BDPT_HELP_BATCH
#define BDPT_HELP_BATCH 0
#endif
#ifndef BDPT_HELP_CLOCKS
#define BDPT_HELP_CLOCKS 0  // measurement only: the counting pass's stack-depth words carry the claim / completion / batch clocks
#endif
#ifndef BDPT_EXPRESS_CHAIN
#define BDPT_EXPRESS_CHAIN 0  // RR build: a lone long walk's delta bounces back to back inside the express block
#endif
#ifndef BDPT_CHAIN_RING_WAVE
#define BDPT_CHAIN_RING_WAVE 1  // the inline chain's generator ring refilled by the whole wave (mt_ring_ahead_wave)
#endif
#if !(BDPT_EXPRESS_CHAIN == 1 && BDPT_DEEP_RNG && BDPT_RING_AHEAD)
#undef BDPT_CHAIN_RING_WAVE
#define BDPT_CHAIN_RING_WAVE 0
#endif
#ifndef BDPT_EXPRESS_PROBE
#define BDPT_EXPRESS_PROBE 0  // measurement only (RR build): express waves with one busy lane, clocks per iteration and in the coop walk
#endif
#if BDPT_RR != 1
#undef BDPT_EXPRESS_PROBE
#define BDPT_EXPRESS_PROBE 0
#endif
#ifndef BDPT_HELP_SREG
#define BDPT_HELP_SREG 1  // BDPT_HELP: the ring positions held in SGPRs during the walk loop (no LDS reads per iteration; 324.6 vs 322.7)
#endif
#ifndef BDPT_HELP_HOIST
#define BDPT_HELP_HOIST 0  // BDPT_HELP: a claim's record loads issued before the lane's own hit is shaded
#endif
#ifndef BDPT_HELP_DEFER
#define BDPT_HELP_DEFER 0  // BDPT_HELP: a claimed task's walk begins one walk iteration after its record loads (305.8 vs 323.5: not kept)
#endif
#ifndef BDPT_HELP_MIN
#define BDPT_HELP_MIN 16  // BDPT_HELP: fewest waiting lanes that start a claim round (unless the ring holds fewer tasks; 1 / 8 / 12 / 16 / 20 / 24: 264.9 / 322.7 / 323.3 / 323.4 / 319.8 / 266.4)
#endif
#ifndef BDPT_TAIL_PROBE
#define BDPT_TAIL_PROBE 0  // measurement only (non-RR builds): the drain phase in the RR diag words (tools/tail_probe.py)
#endif
#ifndef BDPT_READY_HOIST
#define BDPT_READY_HOIST 1  // the shade threshold read before the walk loop instead of in it (Caustic +0.85 %, synth1m +1.2 %)
#endif
#ifndef BDPT_TID_REMAT
#define BDPT_TID_REMAT 1  // the lane's traversal-stack and light-vertex addresses re-derived from threadIdx.x at each use
#endif
// "this is lane 0" from an opaque threadIdx.x (lanes_below: bdpt_device.hpp).
__device__ __forceinline__ bool lane0() { return (opaque_tid() & 63) == 0; }
#ifndef BDPT_TAIL_CHUNK
#define BDPT_TAIL_CHUNK 4  // 0: 64-sample chunks throughout; else finer claims near the end (below)
#endif
// Where the finer claims begin, in quarters of the grid's lanes from the frame's end:
// 16-sample claims from BDPT_TAIL_Z16 / 4 x lanes, 4-sample ones from BDPT_TAIL_Z4 / 4 x
// lanes. Round 6 re-measured them on the task build (each claim seeds a whole wave's
// generators, so finer claims cost throughput): 16 / 8 / 4 quarters with the 4-sample
// claims from 2: Caustic 325.2 / 325.6 / 327.8 Msamples/s, the 1/8 row shard's kernel
// efficiency 0.951 / 0.958-0.965 / 0.961-0.969 and, two frames in flight, 0.957 / 0.975
// / 0.981 (profiles/round6_r6s_tail.log)
#ifndef BDPT_TAIL_Z16
#define BDPT_TAIL_Z16 4
#endif
#ifndef BDPT_TAIL_Z4
#define BDPT_TAIL_Z4 2
#endif
#ifndef BDPT_CLAIM_SCALAR
#define BDPT_CLAIM_SCALAR 1  // the claimed chunk base broadcast by readfirstlane (scalar) instead of a shuffle
#endif
// Samples the wave claims next, from the last chunk it claimed (wave-uniform).
__device__ __forceinline__ uint64_t tail_chunk(uint64_t last_base, uint64_t total) {
    if (!BDPT_TAIL_CHUNK) return 64;
    const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * kBlock;
    return last_base + BDPT_TAIL_Z16 * lanes / 4 < total ? 64 : last_base + BDPT_TAIL_Z4 * lanes / 4 < total ? 16 : 4;
}

template <bool FULL, bool COUNT, bool SLACK>
__global__ __launch_bounds__(kBlock, BDPT_WAVES_PER_EU) void bdpt_frame_kernel(const KParams* __restrict__ kpp) {
    const KParams& kp = *kpp;
    __shared__ uint2 stack_mem[kLdsStack * kBlock];
#if BDPT_ROOT_LDS && BDPT_OVERLAP
    __shared__ RootLds root_lds;
    const bool root_in_lds = !FULL && root_lds_usable(kp.sc);
    if (!FULL) root_lds_fill(root_lds, kp.sc);
#endif
    scene_tables_to_lds(kp.sc);
#if BDPT_TID_REMAT
    const Stack stk{stack_mem, kBlock, kLdsStack, kp.gstack, kp.nslots, blockIdx.x * kBlock, true};
#else
    const Stack stk{stack_mem + threadIdx.x, kBlock, kLdsStack, kp.gstack, kp.nslots, blockIdx.x * kBlock + threadIdx.x};
#endif
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    cnt.m[0] = cnt.m[1] = cnt.m[2] = 0;
    cnt.q[0] = cnt.q[1] = cnt.q[2] = cnt.q[3] = 0;
    cnt.t_step = 0;
#if BDPT_TID_REMAT
    LightStore ls = light_store(kp.lv, kp.fr.lv_max, blockIdx.x * kBlock);
    ls.tid_rel = true;
#else
    const LightStore ls = light_store(kp.lv, kp.fr.lv_max, blockIdx.x * kBlock + threadIdx.x);
#endif
    unsigned long long* const work = kp.work;
    const uint64_t total = kp.fr.total_samples;
    __shared__ LaneCold cold_mem[kBlock];
    Lane L(cold_mem[threadIdx.x]);
    L.state = ST_IDLE;
    bool exhausted = false;  // wave-uniform
#if BDPT_PARK
    if (kp.fr.park_flags & kParkResume) {  // a resume launch: the chain kernel's samples, no claims
        exhausted = true;
        gbl_u32* const rec = (gbl_u32*)park_record(kp.fr, blockIdx.x * kBlock + threadIdx.x);
        if (rec[kParkStatus] == 2u) {
            park_restore((const uint32_t*)rec, L);
            rec[kParkStatus] = 0u;
            rec[kParkResumeDepth] = static_cast<uint32_t>(L.c.depth);
        }
    }
#endif
#if BDPT_SEED_CHUNK
    uint64_t chunk_base = 0;  // wave-uniform: the wave's current chunk of samples
    int chunk_pos = 0, chunk_n = 0;
    bool global_done = false;
    uint32_t chunk_x397 = 0;  // lane i: mt_x397 of sample chunk_base + i
#if BDPT_EYE_SLOTS
    static_assert(kBlock == 64 * kEyeSlotWaves, "one eye-slot row per wave");
    uint32_t chunk_seq = 0;  // wave-uniform: chunks claimed so far (their eye slot: seq mod BDPT_EYE_SLOTS)
    if (lane0())
        for (int k = 0; k < BDPT_EYE_SLOTS; k++) wave_eye_slots()[k] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
#endif
#endif
#if BDPT_OVERLAP
    const TravScene tsc = trav_scene(kp.sc);
    bool tracing = false, has_res = false, q_any = false;
    TravState ts{};
    RayInv ri{};
    int res = -1;
    float rt = 0.f, ru = 0.f, rv = 0.f;
#endif
    // Russian roulette: a subpath trapped in glass by total internal reflection
    // runs for millions of bounces, one bounce per shading step of
    // its wave. A wave holding a subpath past BDPT_EXPRESS_DEPTH stops refilling
    // and shades as soon as any lane has a result, so once its other samples end
    // the trapped lane advances one bounce per walk instead of one per shared
    // shading step (the frame cannot end before it does).
    bool long_walk = false;
#if BDPT_EXPRESS_PROBE
    uint64_t xp_iters = 0, xp_coop = 0, xp_total = 0, xp_t = 0, xp_walk = 0;  // (wave-uniform)
    bool xp_prev = false;
#endif
#if BDPT_HELP
    // helping: the lane walks a task's shadow ray (tracing is set too) or, with BDPT_HELP_DEFER,
    // waits one iteration for its claimed record (hwait)
    bool helping = false;
#if BDPT_HELP_DEFER
    bool hwait = false;
#endif
    {
        const TaskCtl ctl = task_ctl(L.c);
        if (lane0()) *ctl.head = *ctl.tail = 0u;
    }
#else
    constexpr bool helping = false;
#endif
#if BDPT_COOP_ALONE
    bool coop_wait = false;  // a closest-hit walk begun, waiting for its turn to be walked by the whole wave
#endif
    const uint64_t clock0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
#if BDPT_TAIL_PROBE && BDPT_RR != 1
    uint64_t t_drain = 0, t_few = 0;  // wave-uniform (BDPT_TAIL_PROBE)
#endif
#ifndef BDPT_DIAG
#define BDPT_DIAG 1  // 0: no timeline stamps (A/B only)
#endif
    // the kernel's timeline (DevFrame::diag), read through the parameter block
    // where it is stamped (a pointer held across the loop costs SGPR spills)
    if (BDPT_DIAG && kp.fr.diag && lane0()) gmin(kp.fr.diag + kDiagStart, __builtin_amdgcn_s_memrealtime());
    for (;;) {
        // Re-derived every iteration (opaque to the optimiser) so constants are
        // read where they are used instead of being pinned in registers; typed
        // as constant-address-space memory so those reads are scalar loads.
        typedef const __attribute__((address_space(4))) KParams* ConstKParams;
        uint64_t pa = (uint64_t)(ConstKParams)kpp;
        asm volatile("" : "+s"(pa));
        const KParams* P = (const KParams*)(ConstKParams)pa;
        const uint64_t longs = BDPT_RR == 1 && BDPT_EXPRESS_DEPTH > 0 ? __ballot(long_walk) : 0ull;
        const bool express = longs != 0;  // wave-uniform
#if BDPT_EXPRESS_PROBE
        // express waves with one busy lane: iterations, their clocks, and the coop block's share
        const bool xp_lone = express && popc64(__ballot(BDPT_BUSY(L.state))) == 1;
        {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            if (xp_prev) xp_total += now - xp_t;
            xp_t = now;
            xp_prev = xp_lone;
            if (xp_lone) xp_iters++;
        }
#endif
#if BDPT_RR == 1
        if (BDPT_DIAG && BDPT_RR_DIAG && express && lane0() && P->fr.diag) {  // how many trapped walks share a wave (bdpt_stats)
            const int k = popc64(longs);
            gmax(P->fr.diag + kDiagLongMax, static_cast<unsigned long long>(k));
            gadd(P->fr.diag + (k == 1 ? kDiagExpress1 : k <= BDPT_COOP_MAX ? kDiagExpressCoop : kDiagExpressMore), 1ull);
        }
#endif
#if BDPT_SEED_CHUNK
        // Refill idle lanes from the wave's chunk of 64 consecutive samples. A
        // chunk is claimed with one atomic and the seeding recurrence of all its
        // samples (mt_x397) runs once with every lane busy, instead of once per
        // refill with only the refilled lanes doing useful work.
        while (!exhausted && !express) {
            const bool refill = L.state == ST_IDLE && !(BDPT_HELP && helping);  // (a helper's L.ray is its task's)
            const uint64_t idle = __ballot(refill);
            if (!idle) break;
            if (chunk_pos >= chunk_n) {
                if (global_done) {
                    exhausted = true;
                    break;
                }
                // Near the frame's end a wave's unstarted chunk samples wait for
                // its busy lanes (up to a whole sample's latency) while other
                // waves run dry: once the claims seen by this wave come within
                // BDPT_TAIL_Z16 / 4 x the grid's lanes of the end, claim 16, then
                // 4 samples at a time (any sizes partition [0, total)).
                const uint64_t want = tail_chunk(chunk_base, total);
                unsigned long long base = 0;
                if (lane0()) base = gadd(work, static_cast<unsigned long long>(want));
#if BDPT_CLAIM_SCALAR
                // wave-uniform in scalar registers (a shuffle's result is a VGPR pair)
                base = static_cast<unsigned long long>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base))) |
                       static_cast<unsigned long long>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(base >> 32)))
                           << 32;
#else
                base = __shfl(base, 0);
#endif
                if (base >= total) {
                    exhausted = true;
                    break;
                }
                chunk_base = base;
                chunk_n = static_cast<int>(total - base < want ? total - base : want);
                chunk_pos = 0;
                global_done = base + want >= total;
                if (BDPT_DIAG && global_done && lane0() && P->fr.diag)  // the frame's last chunk (one wave claims it)
                    P->fr.diag[kDiagLastClaim] = __builtin_amdgcn_s_memrealtime();
                int px;
                chunk_x397 = mt_x397(sample_seed(base + (opaque_tid() & 63), P->fr, px));
#if BDPT_EYE_SLOTS
                // the chunk's pixel when all 64 samples share one (spp a multiple of 64)
                const int cpx = lane_val(px, 0);
                if (lane0())
                    eye_slot_reset(P->fb, static_cast<int>(chunk_seq % BDPT_EYE_SLOTS), P->fr.spp % 64 == 0 ? cpx : -1);
                chunk_seq++;
#endif
            }
            const int m = min(popc64(idle), chunk_n - chunk_pos);
            const int rank = lanes_below(idle);
            const uint32_t x397 = __shfl(chunk_x397, (chunk_pos + rank) & 63);
            if (refill && rank < m) start_sample<true>(L, chunk_base + chunk_pos + rank, P->fr, x397);
            chunk_pos += m;
        }
#else
        if (!exhausted) {  // refill idle lanes: one atomic per wave
            const uint64_t idle = __ballot(L.state == ST_IDLE);
            if (idle) {
                const int n = popc64(idle);
                const int leader = __ffsll(static_cast<unsigned long long>(idle)) - 1;
                unsigned long long base = 0;
                if ((opaque_tid() & 63) == static_cast<uint32_t>(leader)) base = gadd(work, static_cast<unsigned long long>(n));
                base = __shfl(base, leader);
                if (L.state == ST_IDLE) {
                    const uint64_t s = base + lanes_below(idle);
                    if (s < total) start_sample(L, s, P->fr);
                }
                if (base + n >= total) exhausted = true;
            }
        }
#endif
#if BDPT_HELP
        // the wave ends only with its task ring drained and no helper walking
        if (__ballot(BDPT_BUSY(L.state) || helping) == 0 && *task_ctl(L.c).head == *task_ctl(L.c).tail) {
#else
        if (__ballot(BDPT_BUSY(L.state)) == 0) {
#endif
            if (exhausted) break;
            continue;
        }
#if BDPT_TAIL_PROBE && BDPT_RR != 1
        if (exhausted) {  // the wave's drain: when it began, when at most 4 lanes were left busy
            if (!t_drain) t_drain = __builtin_amdgcn_s_memrealtime();
            if (!t_few && popc64(__ballot(BDPT_BUSY(L.state))) <= 4) t_few = __builtin_amdgcn_s_memrealtime();
        }
#endif
#if BDPT_OVERLAP
        // Overlapped schedule: lanes keep walking their query across loop
        // iterations; a lane whose query finished waits (result kept) until
        // enough lanes of the wave are ready, then those lanes shade together
        // while the slow walkers resume afterwards from where they stopped.
#if BDPT_RR == 1 && BDPT_EXPRESS_WALK
        if (!COUNT && express) {  // a trapped subpath alone in its wave: its delta chain out of line
            const bool alone = popc64(__ballot(BDPT_BUSY(L.state))) == 1;
            if (alone && !tracing && !has_res && (L.state == ST_LIGHT || L.state == ST_EYE)) {
                if (express_walk(L, P->sc, P->fr, P->fb, stk, res, rt, ru, rv)) has_res = true;
                if (!has_res) {
                    long_walk = false;  // the chain ended: the lane's next step comes from the sweep
                    continue;
                }
            }
        }
#endif
#if BDPT_PARK
        if (!COUNT && (P->fr.park_flags & kParkOn) && !tracing && !has_res && (L.state == ST_LIGHT || L.state == ST_EYE) &&
            L.c.depth > P->fr.park_depth && park_lane(P->fr, P->nslots, blockIdx.x * kBlock + opaque_tid(), L)) {
            L.state = ST_PARKED;
            long_walk = false;
#if BDPT_COOP_ALONE
            coop_wait = false;
#endif
        }
#endif
#if BDPT_COOP_ALONE
        bool began = false;  // this lane began a culled closest-hit walk in this iteration
#endif
#if BDPT_COOP_ALONE
        if (BDPT_BUSY(L.state) && !tracing && !has_res && !coop_wait) {  // a new query: begin its walk
#else
        if (BDPT_BUSY(L.state) && !tracing && !has_res) {  // a new query: begin its walk
#endif
            q_any = is_shadow_state(L.state);
            if (COUNT && L.state != ST_DEFER) cnt.c[q_any ? 1 : 0]++;
            ri = ray_inv(L.ray, cull_near_for(L));
            if (L.state == ST_DEFER) {  // no query: the deferred action runs in this shading step
                res = -1;
                has_res = true;
            } else if (L.ray.min_t > L.ray.max_t) {  // the reference culls the root (bvh.h:277, :287)
                res = -1, rt = L.ray.max_t, ru = rv = 0.f;
                has_res = true;
            } else if (FULL || !ri.fast || far_origin(P->sc, L.ray.o)) {  // the reference's tree, unculled
                const TravResult q = traverse_binary<COUNT, Stack>(P->sc, L.ray, q_any, false, stk);
                if (COUNT) cnt.c[2] += q.nodes, cnt.c[3] += q.tris, cnt.c[15] += q.exact;
                res = q.best, rt = q.t, ru = q.u, rv = q.v;
                has_res = true;
            } else {
                ts = trav_begin(tsc, L.ray);
                tracing = true;
#if BDPT_COOP_ALONE
                began = !q_any;
#endif
#if BDPT_ROOT_LDS
                if (root_in_lds && !walk_begin_lds<COUNT, SLACK>(root_lds, L.ray, ri, q_any, ts, stk, cnt)) {
                    res = -1, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;  // no child hit: a miss
                    tracing = false;
                    has_res = true;
#if BDPT_COOP_ALONE
                    began = false;  // (complete: nothing for the wave to walk)
#endif
                }
#endif
            }
        }
#if BDPT_COOP_ALONE
        // Subpaths trapped in glass (express mode: the wave no longer refills). When
        // the wave holds at most BDPT_COOP_MAX busy lanes and each of them has a
        // closest-hit walk begun (in this iteration, or waiting from an earlier one),
        // the wave walks one of them with all 64 lanes (coop_closest: ~10 rounds
        // instead of ~30 dependent steps) on the LDS stack columns of its lanes — no
        // lane holds a walk in progress then, so the columns are free — and the
        // others wait for their turn (waiting lanes first, so every walk gets one).
        // The walk is bounded by twice the lane's last hit distance first (a chain in
        // glass repeats its chord lengths). A lane whose walk did not fit the columns
        // walks alone from the root; waiting lanes walk alone once the wave holds more
        // than BDPT_COOP_MAX busy lanes or leaves express mode (their walk restarts),
        // in their turn: a walk begun while another lane still walks alone waits too.
#if BDPT_EXPRESS_PROBE
        const uint64_t xc0 = __builtin_amdgcn_s_memtime();
#endif
        if (!COUNT && express) {
#if BDPT_ROOT_LDS
            const RootLds* const coop_rl = root_in_lds ? &root_lds : nullptr;
#else
            const RootLds* const coop_rl = nullptr;
#endif
            const uint64_t busy = __ballot(BDPT_BUSY(L.state)), wt = __ballot(coop_wait), bg = __ballot(began);
#if BDPT_COOP_GROUPS
            if (!(P->fr.sched_flags & kSchedNoCoopGroups) && popc64(busy) >= 2 && popc64(busy) <= BDPT_COOP_MAX &&
                (bg | wt) == busy) {
                // 2-4 long walks: each walked by its own group of 32 or 16 lanes, all at once
                const int kb = popc64(busy), G = kb == 2 ? 32 : 16;
                const int me = static_cast<int>(opaque_tid() & 63), gi = me / G;
                int src = -1;  // the lane whose walk this lane's group takes: the gi-th busy lane
                {
                    uint64_t m = busy;
                    for (int g = 0; g < 4 && m; g++) {
                        const int bit = __ffsll(static_cast<unsigned long long>(m)) - 1;
                        if (gi == g) src = bit;
                        m &= m - 1;
                    }
                }
                const bool act = src >= 0;
                const int sl = act ? src : me;
                Ray q;
                q.o = mk(__shfl(L.ray.o.x, sl), __shfl(L.ray.o.y, sl), __shfl(L.ray.o.z, sl));
                q.d = mk(__shfl(L.ray.d.x, sl), __shfl(L.ray.d.y, sl), __shfl(L.ray.d.z, sl));
                q.min_t = __shfl(L.ray.min_t, sl), q.max_t = __shfl(L.ray.max_t, sl);
                RayInv qi;
                qi.inv = mk(__shfl(ri.inv.x, sl), __shfl(ri.inv.y, sl), __shfl(ri.inv.z, sl));
                qi.near = __shfl(ri.near, sl);
                qi.fast = true;
                const float guess = BDPT_GRAZE_IN_DIST ? -1.f : __shfl(L.h.dist, sl);
                const CoopStack cs{stack_mem + (threadIdx.x & ~63u), kBlock};
                const int cap = kLdsStack * G, gbase = gi * cap;
                const bool bounded = act && guess > 0.f;
                float t = 0.f, u = 0.f, v = 0.f;
                int r = -1;
                bool ok = coop_closest_groups<SLACK>(tsc, q, qi, bounded ? 2.f * guess : q.max_t, act, cs, gbase, cap, G,
                                                     t, r, u, v, coop_rl);
                const bool again = bounded && ok && r < 0;  // nothing below the bound: the walk unbounded
                if (__ballot(again)) {
                    float t2 = 0.f, u2 = 0.f, v2 = 0.f;
                    int r2 = -1;
                    const bool ok2 = coop_closest_groups<SLACK>(tsc, q, qi, q.max_t, again, cs, gbase, cap, G, t2, r2, u2, v2,
                                                                coop_rl);
                    if (again) t = t2, u = u2, v = v2, r = r2, ok = ok2;
                }
                // each walk's owner takes its group's result (group = the owner's rank among the busy lanes)
                const int rl = (BDPT_BUSY(L.state) ? lanes_below(busy) : 0) * G;
                t = __shfl(t, rl), u = __shfl(u, rl), v = __shfl(v, rl), r = __shfl(r, rl);
                ok = __shfl(ok ? 1 : 0, rl) != 0;
                if (BDPT_BUSY(L.state)) {
                    coop_wait = false;
                    if (ok) {
                        res = r, rt = t, ru = u, rv = v;
                        tracing = false;
                        has_res = true;
                    } else {
                        ts = trav_begin(tsc, L.ray);  // its stack columns were the wave's
                    }
                }
            } else
#endif
            if (popc64(busy) <= BDPT_COOP_MAX && (bg | wt) == busy) {
                const int b = __ffsll(static_cast<unsigned long long>(wt ? wt : bg)) - 1;
                const int me = static_cast<int>(opaque_tid() & 63);
                const CoopStack cs{stack_mem + (threadIdx.x & ~63u), kBlock};
                float t = 0.f, u = 0.f, v = 0.f;
                int r = -1;
                bool ok = true;
                // A lone long walk (BDPT_EXPRESS_CHAIN): its delta bounces run here, back to
                // back, each walked by the whole wave, until the chain reaches a vertex the
                // sweep must shade — the loop top, the walk loop and the sweep's empty bodies
                // took ~40 % of each bounce's clocks (round 6 probe, BDPT_EXPRESS_PROBE).
                const bool chain = BDPT_EXPRESS_CHAIN && popc64(busy) == 1;
                int bounced = -1;  // -1: the result goes to the sweep; 0: the chain ended here; 2: its next query begins at the loop top
#if BDPT_CHAIN_RING_WAVE
                uint32_t chain_g = 0;  // lane b's ring outputs generated, as the wave last left it (0: unknown)
#endif
#if BDPT_EXPRESS_CHAIN == 2
                if (chain) {
                    bounced = express_chain<SLACK>(L, b, ri, P->sc, P->fr, P->fb, tsc, stack_mem + (threadIdx.x & ~63u),
                                                   coop_rl, t, r, u, v, ok);
                } else
#endif
                for (;;) {
                    Ray q;
                    q.o = mk(lane_val(L.ray.o.x, b), lane_val(L.ray.o.y, b), lane_val(L.ray.o.z, b));
                    q.d = mk(lane_val(L.ray.d.x, b), lane_val(L.ray.d.y, b), lane_val(L.ray.d.z, b));
                    q.min_t = lane_val(L.ray.min_t, b), q.max_t = lane_val(L.ray.max_t, b);
                    RayInv qi;
                    qi.inv = mk(lane_val(ri.inv.x, b), lane_val(ri.inv.y, b), lane_val(ri.inv.z, b));
                    qi.near = lane_val(ri.near, b);
                    qi.fast = true;
                    // the lane's last hit distance (Hit::dist, shade_hit), the bound's guess
                    const float guess = BDPT_GRAZE_IN_DIST ? -1.f : lane_val(L.h.dist, b);
                    r = -1;
                    ok = true;
#if BDPT_EXPRESS_PROBE
                    const uint64_t xw0 = __builtin_amdgcn_s_memtime();
#endif
                    for (int pass = guess > 0.f ? 0 : 1; pass < 2 && r < 0 && ok; pass++) {
                        const float bound = pass == 0 ? 2.f * guess : q.max_t;
                        ok = SLACK ? coop_closest<true, BDPT_COOP_BATCH>(tsc, q, qi, bound, cs, 64 * kLdsStack, t, r, u, v,
                                                                         nullptr, coop_rl)
                                   : coop_closest<false, BDPT_COOP_BATCH>(tsc, q, qi, bound, cs, 64 * kLdsStack, t, r, u, v,
                                                                          nullptr, coop_rl);
                    }
#if BDPT_EXPRESS_PROBE
                    if (xp_lone) xp_walk += __builtin_amdgcn_s_memtime() - xw0;
#endif
                    if (BDPT_EXPRESS_CHAIN != 1 || !chain || !ok) break;
#if BDPT_CHAIN_RING_WAVE
                    if (chain) {  // lane b's generator ring, refilled by the wave when its next bounce could reach the end
                        const uint32_t bn = static_cast<uint32_t>(lane_val(static_cast<int>(L.rng.n), b));
                        if (bn + BDPT_RING_AHEAD >= chain_g)
                            chain_g = mt_ring_ahead_wave(b, bn, static_cast<uint32_t>(lane_val(static_cast<int>(L.rng.a0), b)));
                    }
#endif
                    int more = -1;  // (lane b) -1: not a delta bounce; 0: the chain ended; 1: next bounce here; 2: at the loop top
                    if (me == b && r >= 0 && t <= L.ray.max_t && t >= L.ray.min_t) {  // accel.h:133
                        const BsdfRecord& bb =
                            bsdf_of(P->sc, __float_as_int(gld4(P->sc.shade + kShadeStride * static_cast<size_t>(r)).w));
                        if (is_delta(bb) && is_zero(ld3(bb.emission)) && L.c.steps + 1 <= (1 << 30)) {
                            // the sweep's work at a delta, non-emitting vertex: resolve() (one more
                            // query, the hit shaded), the vertex update (bdpt.h:193-209 / :73-136, no
                            // connection at a delta vertex), ContinuePathRandomWalk (bdpt.h:243-291)
                            // and the loop test (bdpt.h:188 / :68)
                            ++L.c.steps;
                            shade_hit(P->sc, r, u, v, t, L.ray.d, L.h);
                            const float dist2 = L.h.dist * L.h.dist;
                            BDPT_DIST_TO_GRAZE
                            const float absCosIn = fabsf(L.h.wo.z);
#if BDPT_DEEP_RNG && BDPT_RING_AHEAD
#if BDPT_CHAIN_RING_WAVE
                            const bool ring_ok = chain_g >= L.rng.n + BDPT_RING_AHEAD;  // the wave generated far enough
#else
                            constexpr bool ring_ok = false;
#endif
                            if (L.rng.n + BDPT_RING_AHEAD >= 227 && !ring_ok && !mt_ring_ahead(L.rng) && P->fr.diag)
                                gadd(P->fr.diag + kDiagErrors, 1ull);
#endif
                            L.c.vcm *= div_w(dist2, absCosIn);
                            L.c.vc *= rcp_w(absCosIn);
                            L.c.rr = rr_probability(P->fr, L.c.depth, L.c.tp);
                            const bool light = L.state == ST_LIGHT;
                            const bool cont = continue_walk(bb, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, L.c.rr);
                            if (cont && walk_continues(L, P->fr)) {
                                ri = ray_inv(L.ray, cull_near_for(L));
                                more = ri.fast && !far_origin(P->sc, L.ray.o) && !(L.ray.min_t > L.ray.max_t) ? 1 : 2;
                            } else {
                                if (light) L.state = ST_DEFER;  // the eye subpath starts next step
                                else finish<false>(L, P->fr, P->fb, cnt);  // L.state = ST_IDLE
                                more = 0;
                            }
                        }
                    }
                    more = lane_val(more, b);
                    if (more == 1) continue;  // the next bounce's walk, by the whole wave
                    bounced = more;
                    break;
                }
                if (bounced >= 0) {  // lane b's bounces ran here: no result pending
                    if (me == b) {
                        coop_wait = false;
                        tracing = false;
                        has_res = false;
                        long_walk = L.state != ST_IDLE && L.c.depth > P->fr.express_depth;
                    }
                } else if (me == b) {
                    coop_wait = false;
                    if (ok) {
                        res = r, rt = t, ru = u, rv = v;
                        tracing = false;
                        has_res = true;
                    } else {
                        ts = trav_begin(tsc, L.ray);  // its stack columns were the wave's
                    }
                } else if (began) {
                    coop_wait = true;  // its turn comes in a later iteration
                    tracing = false;
                }
            } else if (popc64(busy) <= BDPT_COOP_MAX) {
                // some lane still walks alone (a shadow ray, or a walk that did not fit
                // the columns): walks begun now wait for it, so they are walked by the wave
                if (began) {
                    coop_wait = true;
                    tracing = false;
                }
            } else {
                coop_wait = false;  // too many busy lanes: waiting walks restart alone next iteration
            }
        } else {
            coop_wait = false;
        }
#if BDPT_EXPRESS_PROBE
        if (xp_lone) xp_coop += __builtin_amdgcn_s_memtime() - xc0;
#endif
#endif
        const uint64_t c0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
#if BDPT_READY_HOIST
        // read once per shading step: in the walk loop its scalar load waited (lgkmcnt)
        // on the lane's LDS stack traffic every iteration
        const int steady_ready = P->fr.shade_ready > 0 ? P->fr.shade_ready : BDPT_SHADE_READY;
#endif
#if BDPT_HELP && BDPT_HELP_SREG
        // the ring's positions in scalar registers while the wave walks (pushes happen
        // only in the shading step; claims below write the head back)
        uint32_t qhead = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(*task_ctl(L.c).head)));
        const uint32_t qtail = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(*task_ctl(L.c).tail)));
#endif
        for (;;) {  // walk until enough lanes have a result to shade
#if BDPT_HELP
            uint64_t tr = __ballot(tracing);
            const uint64_t ready = __ballot(has_res && !helping);  // helpers shade after their walk
            if (popc64(ready) >= (BDPT_TAIL_SHADE == 1 && exhausted ? 1
                                  : BDPT_TAIL_SHADE == 2 && exhausted ? max(1, (popc64(tr | ready) * BDPT_TAIL_FRAC) >> 3)
                                                                      : steady_ready))
                break;
            // Lanes that wait (a result kept, or no sample) claim the ring's oldest
            // tasks, one each, and walk their shadow rays with the walk code below.
            bool hfin = false;  // a helper walk that ended in this iteration (result in ts.best)
            // a claimed task's walk begins: the root's LDS tests, or at once a result
            auto help_begin = [&](float near) {
                q_any = true;
                if (COUNT) cnt.c[1]++;
                ri = ray_inv(L.ray, near);
                ts.best = -1;
                if (L.ray.min_t > L.ray.max_t) {  // the reference culls the root: unoccluded
                    hfin = true;
                } else if (!ri.fast || far_origin(P->sc, L.ray.o)) {  // the reference's tree, unculled
                    const TravResult qr = traverse_binary<COUNT, Stack>(P->sc, L.ray, true, false, stk);
                    if (COUNT) cnt.c[2] += qr.nodes, cnt.c[3] += qr.tris, cnt.c[15] += qr.exact;
                    ts.best = qr.best;
                    hfin = true;
                } else {
                    ts = trav_begin(tsc, L.ray);
                    tracing = true;
#if BDPT_ROOT_LDS
                    if (root_in_lds && !walk_begin_lds<COUNT, SLACK>(root_lds, L.ray, ri, true, ts, stk, cnt)) {
                        tracing = false;  // no child hit: unoccluded
                        hfin = true;
                    }
#endif
                }
            };
#if BDPT_HELP_DEFER
            if (hwait) {  // claimed in the previous iteration: its record has arrived meanwhile
                hwait = false;
                L.c.pend = mk(ts.best_t, ts.best_u, ts.best_v);
                L.c.pend_px = static_cast<int>(ts.link);
                help_begin(ri.near);
            }
#endif
            const uint64_t hk0 = COUNT && BDPT_HELP_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
            {
                const TaskCtl ctl = task_ctl(L.c);
#if BDPT_HELP_SREG
                const uint32_t head = qhead, tail = qtail;
#else
                const uint32_t head = *ctl.head, tail = *ctl.tail;
#endif
                // (a lane waiting on its own shadow ray, pushed by itself when the ring was
                // full, keeps its pending contribution in L.c.pend: it does not help)
                const bool cand = !helping && !tracing && (has_res ? !is_shadow_state(L.state) : L.state == ST_IDLE);
                uint64_t cm = head != tail ? __ballot(cand) : 0ull;
                // claim rounds only with enough takers (each round exposes one record load):
                // BDPT_HELP_MIN lanes, or any once the wave's own walks have ended
                if (popc64(cm) < BDPT_HELP_MIN && popc64(cm) < static_cast<int>(tail - head) && __ballot(tracing)) cm = 0;
                if (cm) {
                    if (COUNT && lane0()) cnt.q[2]++;  // (counting pass: claim rounds)
                    const uint32_t n = min(static_cast<uint32_t>(popc64(cm)), tail - head);
                    const uint32_t rank = static_cast<uint32_t>(lanes_below(cm));
                    *ctl.head = head + n;
#if BDPT_HELP_SREG
                    qhead = head + n;
#endif
                    if (cand && rank < n) {
#if !BDPT_HELP_HOIST
                        if (has_res) help_compact(L, res, rt, ru, rv, P->sc);  // frees L.ray
#endif
                        const uint32_t slot = (head + rank) & (P->fr.task_cap - 1);
                        float4* const ring = task_ring(P->fr);
                        const uint32_t cap = P->fr.task_cap;
                        const float4 a = gld4(task_vec(ring, cap, slot, 0)), b = gld4(task_vec(ring, cap, slot, 1)),
                                     c = gld4(task_vec(ring, cap, slot, 2));
#if BDPT_HELP_HOIST
                        // the record's loads are in flight while the lane's own hit is shaded
                        // (one exposed latency per claim round instead of two)
                        if (has_res) help_compact(L, res, rt, ru, rv, P->sc);  // frees L.ray
#endif
                        if (COUNT) cnt.q[3]++;  // (counting pass: claims)
                        L.ray = Ray{xyz(a), xyz(b), kEpsilon, a.w};
                        helping = true;
#if BDPT_HELP_DEFER
                        // the walk begins next iteration (the loads land meanwhile): the near
                        // cull, contribution and pixel wait in the lane's idle walk registers
                        ri.near = b.w;
                        ts.best_t = c.x, ts.best_u = c.y, ts.best_v = c.z;
                        ts.link = __float_as_uint(c.w);
                        hwait = true;
#else
                        // the contribution and pixel into the lane's (free) pending-connection
                        // fields: the slot may be pushed over once claimed
                        L.c.pend = xyz(c);
                        L.c.pend_px = __float_as_int(c.w);
                        help_begin(b.w);
#endif
                    }
                }
            }
            if (COUNT && BDPT_HELP_CLOCKS && first_active_lane())  // (probe build: claim block clocks in stack_gt8)
                cnt.c[16] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - hk0);
            tr = __ballot(tracing);
#if BDPT_HELP_DEFER
            if (!tr && !__ballot(hfin) && !__ballot(hwait)) break;
#else
            if (!tr && !__ballot(hfin)) break;
#endif
#else
            const uint64_t tr = __ballot(tracing);
            if (!tr) break;
            const uint64_t ready = __ballot(has_res);
            if (popc64(ready) >= (express ? 1
                                    : BDPT_TAIL_SHADE == 1 && exhausted ? 1
                                    : BDPT_TAIL_SHADE == 2 && exhausted ? max(1, (popc64(tr | ready) * BDPT_TAIL_FRAC) >> 3)
#if BDPT_READY_HOIST
                                                                        : steady_ready))
#else
                                                                        : (P->fr.shade_ready > 0 ? P->fr.shade_ready : BDPT_SHADE_READY)))
#endif
                break;
#endif
#if BDPT_TRAV_SPLIT
            // Lanes at a leaf and lanes at an interior node step in alternate
            // iterations (whichever group is larger in the sense of the ratio
            // below) instead of both code paths running in every iteration.
            const bool at_leaf = (ts.link & kLeafBit) != 0;
            const uint64_t lv = __ballot(tracing && at_leaf);
            const bool do_leaf = popc64(lv) * 4 >= popc64(tr & ~lv) * BDPT_TRAV_SPLIT;
            bool fin = tracing && at_leaf == do_leaf && trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
            // BDPT_WALK_UNROLL more interior-node steps before the wave's ballots
#pragma unroll
            for (int k = 0; k < BDPT_WALK_UNROLL; k++)
                if ((BDPT_UNROLL_ANY || !do_leaf) && tracing && !fin && !(ts.link & kLeafBit))
                    fin = trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
            if (fin) {
#else
            if (tracing && trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt)) {
#endif
#if BDPT_HELP
                tracing = false;
                if (helping) {
                    hfin = true;
                } else {
                    res = ts.best, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                    has_res = true;
                }
#else
                res = ts.best, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                tracing = false;
                has_res = true;
#endif
            }
#if BDPT_HELP
            const uint64_t hk1 = COUNT && BDPT_HELP_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
            if (hfin) {  // the task's shadow ray: unoccluded -> its contribution to the pixel
                helping = false;
                if (ts.best < 0) {
                    const uint32_t meta = static_cast<uint32_t>(L.c.pend_px);
                    const int px = static_cast<int>(meta & kTaskPixel);
                    if (meta & kTaskSplat) {
                        if (COUNT) cnt.c[6]++;
                        splat_add(P->fb, px, L.c.pend);
                    } else {
                        eye_add(P->fb, px, L.c.pend);
                    }
                }
            }
            if (COUNT && BDPT_HELP_CLOCKS && first_active_lane())  // (probe build: completion clocks in stack_gt12)
                cnt.c[17] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - hk1);
#endif
        }
        const uint64_t c1 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        const bool shade_now = has_res && !(BDPT_HELP && helping);  // (a helper mid-walk shades next time)
#if BDPT_HELP_BATCH
        uint32_t act2 = A_DONE;
#endif
        const bool shading = COUNT && __ballot(shade_now) != 0;
        if (shade_now) {
            has_res = false;
#if BDPT_DEEP_RNG && BDPT_RING_AHEAD
            // the draws of this step past 227 are read from the ring: generate them first
            if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && P->fr.diag)
                gadd(P->fr.diag + kDiagErrors, 1ull);
#endif
            const uint64_t r0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t act = resolve<COUNT>(L, res, rt, ru, rv, P->sc, P->fr, P->fb, cnt);
            if (COUNT && first_active_lane()) cnt.c[20] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - r0);
#if BDPT_HELP_BATCH
            act2 = advance<COUNT, 1>(L, act, P->sc, P->fr, P->fb, ls, cnt);
#else
            advance<COUNT>(L, act, P->sc, P->fr, P->fb, ls, cnt);
#endif
            if (BDPT_RR == 1) long_walk = L.state != ST_IDLE && L.c.depth > P->fr.express_depth;
        }
#if BDPT_HELP_BATCH
        // the connections of the eye vertices reached in this step, over the whole wave
        if (__ballot(shade_now)) {
            const uint64_t hk2 = COUNT && BDPT_HELP_CLOCKS ? __builtin_amdgcn_s_memtime() : 0;
            conn_batch<COUNT>(L, shade_now && act2 == A_CONN && P->fr.strategy == 0, P->sc, P->fr, ls, cnt);
            if (COUNT && BDPT_HELP_CLOCKS && first_active_lane())  // (probe build: batch clocks in stack_gt16)
                cnt.c[18] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - hk2);
            if (shade_now) advance<COUNT, 2>(L, act2, P->sc, P->fr, P->fb, ls, cnt);
        }
#endif
        if (COUNT && first_active_lane()) {
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
            cnt.c[12] += static_cast<uint32_t>(c1 - c0);
            cnt.c[13] += static_cast<uint32_t>(c2 - c1);
        }
        if (COUNT && shading && !BDPT_HELP) {  // the connection tasks the wave held in this shading step (Counts::q)
            uint32_t tw = cnt.t_step;
            for (int off = 32; off > 0; off >>= 1) tw += static_cast<uint32_t>(__shfl_xor(static_cast<int>(tw), off));
            cnt.t_step = 0;
            if (lane0()) cnt.q[0] += tw, cnt.q[1]++, cnt.q[2] += tw >= 32u, cnt.q[3] += tw >= 64u;
        }
#else
        if (L.state != ST_IDLE) step<FULL, COUNT>(L, P->sc, P->fr, P->fb, ls, stk, cnt);
#endif
    }
#if BDPT_SEED_CHUNK && BDPT_EYE_SLOTS
    if (lane0())  // every sample of the wave has finished: the slots' sums to the framebuffer
        for (int k = 0; k < BDPT_EYE_SLOTS; k++) eye_slot_reset(kp.fb, k, -1);
#endif
    if (BDPT_DIAG && lane0() && kpp->fr.diag) gmax(kpp->fr.diag + kDiagEnd, __builtin_amdgcn_s_memrealtime());
#if BDPT_EXPRESS_PROBE
    if (lane0() && xp_iters) {  // into bdpt_stats.sched (a timed run writes nothing else there)
        gadd(kpp->counters + kCounters + 3, static_cast<unsigned long long>(xp_iters));
        gadd(kpp->counters + kCounters + 3 + 1, static_cast<unsigned long long>(xp_coop));
        gadd(kpp->counters + kCounters + 3 + 2, static_cast<unsigned long long>(xp_total));
        gadd(kpp->counters + kCounters + 3 + 3, static_cast<unsigned long long>(xp_walk));  // of xp_coop: in the walks
    }
#endif
#if BDPT_TAIL_PROBE && BDPT_RR != 1
    // longest drain with <= 4 busy lanes, longest drain, their sum over waves, waves that had one
    if (lane0() && kpp->fr.diag) {
        const uint64_t end = __builtin_amdgcn_s_memrealtime();
        unsigned long long* const d = kpp->fr.diag;
        if (t_few) gmax(d + kDiagLongMax, static_cast<unsigned long long>(end - t_few));
        if (t_drain) gmax(d + kDiagExpress1, static_cast<unsigned long long>(end - t_drain));
        if (t_few) gadd(d + kDiagExpressCoop, static_cast<unsigned long long>(end - t_few));
        if (t_few) gadd(d + kDiagExpressMore, 1ull);
    }
#endif
    if (COUNT) {
        if (lane0()) cnt.c[14] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - clock0);
        flush_counts(cnt, kp.counters);
    }
}


#if BDPT_PARK
// The continuation pass's chain kernel: one wave per parked sample (see park_lane).
#ifndef BDPT_CHAIN_PROBE
#define BDPT_CHAIN_PROBE 0
#endif
#ifndef BDPT_CHAIN_LDS_RING
#define BDPT_CHAIN_LDS_RING 1  // the chain's MT19937 ring in LDS (each draw an LDS read instead of an HBM round trip)
#endif
constexpr int kChainStack = 2048;  // LDS entries of the wave's shared walk stack
__global__ __launch_bounds__(64) void bdpt_chain_kernel(const KParams* __restrict__ kpp) {
    const KParams& kp = *kpp;
    __shared__ uint2 cstack[kChainStack];
    __shared__ LaneCold cold;
#if BDPT_CHAIN_LDS_RING
    __shared__ uint32_t lring[kMtRingSlotWords];
#endif
    scene_tables_to_lds(kp.sc);
    const uint32_t lane = threadIdx.x;
#if BDPT_EYE_SLOTS
    if (lane == 0)  // no eye-estimate slots here: a sample that ends adds to the framebuffer itself
        for (int k = 0; k < BDPT_EYE_SLOTS; k++) wave_eye_slots()[k] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
#endif
    const DevScene& sc = kp.sc;
    const DevFrame& fr = kp.fr;
    const TravScene tsc = trav_scene(sc);
    const gbl_u32* const list = (const gbl_u32*)park_list(fr, kp.nslots);
    const uint32_t n = list[0];
    Counts cnt;  // (not a counting pass)
    // BDPT_CHAIN_PROBE: bounces, walk rounds, and the longest walk's bounces and clocks into bdpt_stats.sched
    uint64_t pc[4] = {0u, 0u, 0u, 0u};
    uint32_t rounds32 = 0;
    uint32_t* const probe_rounds = BDPT_CHAIN_PROBE ? &rounds32 : nullptr;
    const uint64_t k0 = BDPT_CHAIN_PROBE ? __builtin_amdgcn_s_memtime() : 0;
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t slot = list[1 + i];
        uint32_t* const rec = park_record(fr, slot);
        Lane L(cold);
        float guess = -1.f;  // the last hit distance of this chain (wave-uniform)
        const uint64_t w0 = BDPT_CHAIN_PROBE ? __builtin_amdgcn_s_memtime() : 0, wb = pc[0];
#if BDPT_CHAIN_LDS_RING
        // the slot's MT19937 ring (and generator cursor) in LDS while the chain draws from it
        gbl_u32* const hring = (gbl_u32*)(sc.mt_ring + static_cast<size_t>(slot) * kMtRingSlotWords);
        for (uint32_t k = lane; k < kMtRingSlotWords; k += 64) lring[k] = hring[k];
        if (lane == 0) {
            const uint64_t a = reinterpret_cast<uint64_t>(static_cast<uint32_t*>(lring));
            g_scene_lds[0] = static_cast<uint32_t>(a), g_scene_lds[1] = static_cast<uint32_t>(a >> 32);
            g_scene_lds[3] = 0u;  // mt_ring_slot: lring for lane 0
            park_restore(rec, L);
        }
        __syncthreads();
#else
        if (lane == 0) {
            park_restore(rec, L);
            g_scene_lds[3] = slot;  // the sample's MT19937 ring (mt_ring_slot, lane 0)
        }
#endif
        for (;;) {
            const uint64_t c0 = BDPT_CHAIN_PROBE ? __builtin_amdgcn_s_memtime() : 0;
            // lane 0's query, walked by the wave
            Ray q;
            q.o = mk(lane_val(L.ray.o.x, 0), lane_val(L.ray.o.y, 0), lane_val(L.ray.o.z, 0));
            q.d = mk(lane_val(L.ray.d.x, 0), lane_val(L.ray.d.y, 0), lane_val(L.ray.d.z, 0));
            q.min_t = lane_val(L.ray.min_t, 0), q.max_t = lane_val(L.ray.max_t, 0);
            const float near = lane_val(lane == 0 ? cull_near_for(L) : 0.f, 0);
            if (q.min_t > q.max_t) break;  // the megakernel resolves it (a miss)
            const RayInv ri = ray_inv(q, near);
            if (!ri.fast || far_origin(sc, q.o)) break;  // the reference's tree: the megakernel walks it
            // A chain in glass repeats its chord lengths: the walk first accepts only hits
            // below twice the last one (culling the boxes beyond), then, if none, unbounded.
            float t, u, v;
            int r = -1;
            bool ok = true;
            for (int pass = guess > 0.f ? 0 : 1; pass < 2 && r < 0 && ok; pass++) {
                const float bound = pass == 0 ? 2.f * guess : q.max_t;
                const CoopStack cs{cstack, 0};
                ok = tsc.node_slack ? coop_closest<true>(tsc, q, ri, bound, cs, kChainStack, t, r, u, v, probe_rounds)
                                    : coop_closest<false>(tsc, q, ri, bound, cs, kChainStack, t, r, u, v, probe_rounds);
            }
            if (BDPT_CHAIN_PROBE) pc[0]++, pc[2] += __builtin_amdgcn_s_memtime() - c0;
            guess = r >= 0 ? t : -1.f;
            if (!ok) {
                if (lane == 0 && fr.diag) gadd(fr.diag + kDiagErrors, 1ull);
                break;
            }
            const bool hit = r >= 0 && t <= q.max_t && t >= q.min_t;  // accel.h:133
            if (!hit) break;
            const BsdfRecord& b = bsdf_of(sc, __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(r)).w));
            if (!is_delta(b) || !is_zero(ld3(b.emission))) break;  // a vertex the megakernel shades
            int more = 0;
            if (lane == 0 && L.c.steps + 1 <= (1 << 30)) {
                // the sweep's work at a delta, non-emitting vertex (express_walk's bounce): resolve(),
                // the vertex update (bdpt.h:193-209 / :73-136), ContinuePathRandomWalk, the loop test
                ++L.c.steps;
                shade_hit(sc, r, u, v, t, L.ray.d, L.h);
                const float dist2 = L.h.dist * L.h.dist;
                BDPT_DIST_TO_GRAZE
                const float absCosIn = fabsf(L.h.wo.z);
#if BDPT_RING_AHEAD
                if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && fr.diag)
                    gadd(fr.diag + kDiagErrors, 1ull);
#endif
                L.c.vcm *= div_cr(dist2, absCosIn);
                L.c.vc *= rcp_cr(absCosIn);
                L.c.rr = rr_probability(fr, L.c.depth, L.c.tp);
                const bool light = L.state == ST_LIGHT;
                const bool cont = continue_walk(b, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, L.c.rr);
                if (cont && walk_continues(L, fr)) {
                    more = 1;
                } else if (light) {
                    L.state = ST_DEFER;  // the eye subpath starts in the megakernel's next step
                } else {
                    finish<false>(L, fr, kp.fb, cnt);  // L.state = ST_IDLE
                }
            }
            if (!lane_val(more, 0)) break;
        }
        if (lane == 0) {
            park_save(rec, L);
            ((gbl_u32*)rec)[kParkStatus] = 2u;
            if (BDPT_CHAIN_PROBE) {  // the longest walk: its bounces and clocks
                gmax(kp.counters + kCounters + 3 + 2, static_cast<unsigned long long>(pc[0] - wb));
                gmax(kp.counters + kCounters + 3 + 3, static_cast<unsigned long long>(__builtin_amdgcn_s_memtime() - w0));
            }
        }
#if BDPT_CHAIN_LDS_RING
        __syncthreads();
        for (uint32_t k = lane; k < kMtRingSlotWords; k += 64) hring[k] = lring[k];
#endif
    }
    if (BDPT_CHAIN_PROBE && lane == 0 && n > blockIdx.x) {
        gadd(kp.counters + kCounters + 3, static_cast<unsigned long long>(pc[0]));
        gadd(kp.counters + kCounters + 3 + 1, static_cast<unsigned long long>(rounds32));
    }
    (void)k0;
}
#endif
#endif  // !BDPT_SAMPLER_STATE

#if BDPT_SAMPLER_STATE
// One Integrator::render(ray, sampler) call on one lane (single-sample build,
// sample_state.hip): the sampler is the caller's std::mt19937 state, whose
// address sc.mt_ring carries into the LDS header (mt_state_u32); splats go to
// the list `fb` (splat_add). out = Li.xyz, draws taken.
__global__ __launch_bounds__(64) void bdpt_sample_kernel(DevScene sc, DevFrame fr, float* __restrict__ fb,
                                                         float* __restrict__ lvbuf, uint2* __restrict__ gstack,
                                                         Ray ray, float* __restrict__ out) {
    __shared__ uint2 stack_mem[kLdsStack * 64];
    scene_tables_to_lds(sc);
    if (threadIdx.x != 0) return;
    Counts cnt;
    const LightStore ls = light_store(lvbuf, fr.lv_max, 0);
    __shared__ LaneCold cold_mem[1];
    Lane L(cold_mem[0]);
    L.rng = LazyMT{0u, 0u, 0u, 0u};  // unused: next1 draws from the caller's state
    L.c.pixel = 0;
    L.c.cam_d = ray.d;
    L.ray = ray;
    L.c.Li = mk(0.f, 0.f, 0.f);
    L.c.steps = 0;
    L.state = ST_PRIMARY;
    DevFrame f1 = fr;
    f1.flags |= kFlagNoEyeAccum;  // Integrator::render returns Li; the caller accumulates it
    const Stack stk{stack_mem, 64, kLdsStack, gstack, 1, 0};
    while (L.state != ST_IDLE) step<false, false>(L, sc, f1, fb, ls, stk, cnt);
    out[0] = L.c.Li.x, out[1] = L.c.Li.y, out[2] = L.c.Li.z;
    out[3] = __uint_as_float(L.rng.n);
}

#endif  // BDPT_SAMPLER_STATE

}  // namespace dev

// ------------------------------------------------------------ host launchers
#if !BDPT_SAMPLER_STATE
size_t frame_params_bytes() { return sizeof(dev::KParams); }

// `dparams` is a device buffer of frame_params_bytes() owned by the caller; it
// is filled on `stream` before the launch (stream order protects reuse).
hipError_t launch_frame(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                        uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                        hipStream_t stream, void* dparams) {
    const bool full = (fr.flags & 2u) != 0, count = (fr.flags & 1u) != 0, slack = sc.node_slack != 0;
    const dev::KParams host{sc, fr, fb, lvbuf, gstack, nslots, work, counters};
    hipError_t e = hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    const dev::KParams* kp = static_cast<const dev::KParams*>(dparams);
    const dim3 g(grid), b(dev::kBlock);
    const size_t lds = 4 * static_cast<size_t>(sc.lds_words);
    // FULL walks the reference's binary tree: SLACK does not apply
    if (full && count) hipLaunchKernelGGL((dev::bdpt_frame_kernel<true, true, true>), g, b, lds, stream, kp);
    else if (full) hipLaunchKernelGGL((dev::bdpt_frame_kernel<true, false, true>), g, b, lds, stream, kp);
    else if (count && slack) hipLaunchKernelGGL((dev::bdpt_frame_kernel<false, true, true>), g, b, lds, stream, kp);
    else if (count) hipLaunchKernelGGL((dev::bdpt_frame_kernel<false, true, false>), g, b, lds, stream, kp);
    else if (slack) hipLaunchKernelGGL((dev::bdpt_frame_kernel<false, false, true>), g, b, lds, stream, kp);
    else hipLaunchKernelGGL((dev::bdpt_frame_kernel<false, false, false>), g, b, lds, stream, kp);
    return hipGetLastError();
}


#if BDPT_PARK
// The Russian-roulette continuation pass's chain kernel (one wave per parked
// sample, grid-stride over the list); same parameter block as launch_frame.
hipError_t launch_chain(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                        uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                        hipStream_t stream, void* dparams) {
    const dev::KParams host{sc, fr, fb, lvbuf, gstack, nslots, work, counters};
    hipError_t e = hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(dev::bdpt_chain_kernel, dim3(grid), dim3(64), 4 * static_cast<size_t>(sc.lds_words), stream,
                       static_cast<const dev::KParams*>(dparams));
    return hipGetLastError();
}
#endif
#endif  // !BDPT_SAMPLER_STATE

#if BDPT_SAMPLER_STATE
// sc.mt_ring = the device copy of the caller's std::mt19937 state (625 words);
// splats = the splat list (header + records, see splat_add).
hipError_t launch_sample(const dev::DevScene& sc, const dev::DevFrame& fr, float* splats, float* lvbuf, uint2* gstack,
                         const dev::Ray& ray, float* out, hipStream_t stream) {
    hipLaunchKernelGGL(dev::bdpt_sample_kernel, dim3(1), dim3(64), 4 * static_cast<size_t>(sc.lds_words), stream, sc,
                       fr, splats, lvbuf, gstack, ray, out);
    return hipGetLastError();
}
#else

// Resident 256-lane blocks per CU for the frame kernel (VGPR and LDS limited).
int frame_kernel_blocks_per_cu(size_t dyn_lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::bdpt_frame_kernel<false, false, false>, dev::kBlock,
                                                     dyn_lds) !=
            hipSuccess ||
        n <= 0)
        n = BDPT_WAVES_PER_EU;
    return n;
}

int frame_kernel_lds_stack() { return dev::kLdsStack; }
int frame_kernel_block() { return dev::kBlock; }
int light_vertex_fields() { return dev::kLvFields; }

#endif  // BDPT_SAMPLER_STATE

}  // namespace bdpt
