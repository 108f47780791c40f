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
#define BDPT_TRAV_SPLIT 8  // > 0: leaf and interior-node steps in separate iterations (leaf step if 4 * leaf lanes >= SPLIT * node lanes)
#endif
#ifndef BDPT_SEED_CHUNK
#define BDPT_SEED_CHUNK 1  // refill from per-wave chunks of 64 samples seeded together (0: per-refill seeding)
#endif
#ifndef BDPT_WALK_UNROLL
#define BDPT_WALK_UNROLL 1  // extra interior-node steps per walk iteration (measured: 0: 201.7, 1: 203.6)
#endif
#ifndef BDPT_SHADE_READY
#define BDPT_SHADE_READY 48  // lanes with a finished query that trigger the wave's shading step
#endif
#ifndef BDPT_TAIL_SHADE
#define BDPT_TAIL_SHADE 2  // once a wave has no samples left to claim: 1 shade at 1 ready lane, 2 at BDPT_TAIL_FRAC / 8 of its busy lanes
#endif
#ifndef BDPT_TAIL_FRAC
#define BDPT_TAIL_FRAC 6  // (measured, 512x512x256 1/8 shard: end tail 2.19 -> 1.93 ms, steady state unchanged)
#endif
#ifndef BDPT_EXPRESS_DEPTH
#define BDPT_EXPRESS_DEPTH 512  // Russian-roulette build: a subpath this deep puts its wave in express mode (below)
#endif
#ifndef BDPT_ROOT_LDS
#define BDPT_ROOT_LDS 1  // 1: the traversal root and its interior children in LDS, tested when a walk begins (RootLds; measured +1.6 %)
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
#ifndef BDPT_TID_REMAT
#define BDPT_TID_REMAT 1  // the lane's traversal-stack and light-vertex addresses re-derived from threadIdx.x at each use
#endif
// The lane's rank among the set lanes of m below it (mbcnt: no per-lane mask
// held across the loop), and "this is lane 0" from an opaque threadIdx.x.
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return static_cast<int>(__builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u)));
}
__device__ __forceinline__ bool lane0() { return (opaque_tid() & 63) == 0; }
#ifndef BDPT_TAIL_CHUNK
#define BDPT_TAIL_CHUNK 4  // x the grid's lanes from the end: finer claims (0: 64-sample chunks throughout)
#endif
#ifndef BDPT_CLAIM_SCALAR
#define BDPT_CLAIM_SCALAR 1  // the claimed chunk base broadcast by readfirstlane (scalar) instead of a shuffle
#endif
// Samples the wave claims next, from the last chunk it claimed (wave-uniform).
__device__ __forceinline__ uint64_t tail_chunk(uint64_t last_base, uint64_t total) {
    if (!BDPT_TAIL_CHUNK) return 64;
    const uint64_t lanes = static_cast<uint64_t>(gridDim.x) * kBlock;
    return last_base + BDPT_TAIL_CHUNK * lanes < total ? 64 : last_base + lanes / 2 < total ? 16 : 4;
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
    const uint64_t clock0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
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
        const bool express = BDPT_RR == 1 && BDPT_EXPRESS_DEPTH > 0 && __ballot(long_walk) != 0;  // wave-uniform
#if BDPT_SEED_CHUNK
        // Refill idle lanes from the wave's chunk of 64 consecutive samples. A
        // chunk is claimed with one atomic and the seeding recurrence of all its
        // samples (mt_x397) runs once with every lane busy, instead of once per
        // refill with only the refilled lanes doing useful work.
        while (!exhausted && !express) {
            const uint64_t idle = __ballot(L.state == ST_IDLE);
            if (!idle) break;
            if (chunk_pos >= chunk_n) {
                if (global_done) {
                    exhausted = true;
                    break;
                }
                // Near the frame's end a wave's unstarted chunk samples wait for
                // its busy lanes (up to a whole sample's latency) while other
                // waves run dry: once the claims seen by this wave come within
                // BDPT_TAIL_CHUNK x the grid's lanes of the end, claim 16, then
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
                const int cpx = __shfl(px, 0);
                if (lane0())
                    eye_slot_reset(P->fb, static_cast<int>(chunk_seq % BDPT_EYE_SLOTS), P->fr.spp % 64 == 0 ? cpx : -1);
                chunk_seq++;
#endif
            }
            const int m = min(__popcll(idle), chunk_n - chunk_pos);
            const int rank = lanes_below(idle);
            const uint32_t x397 = __shfl(chunk_x397, (chunk_pos + rank) & 63);
            if (L.state == ST_IDLE && rank < m) start_sample<true>(L, chunk_base + chunk_pos + rank, P->fr, x397);
            chunk_pos += m;
        }
#else
        if (!exhausted) {  // refill idle lanes: one atomic per wave
            const uint64_t idle = __ballot(L.state == ST_IDLE);
            if (idle) {
                const int n = __popcll(idle);
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
        if (__ballot(L.state != ST_IDLE) == 0) {
            if (exhausted) break;
            continue;
        }
#if BDPT_OVERLAP
        // Overlapped schedule: lanes keep walking their query across loop
        // iterations; a lane whose query finished waits (result kept) until
        // enough lanes of the wave are ready, then those lanes shade together
        // while the slow walkers resume afterwards from where they stopped.
#if BDPT_RR == 1 && BDPT_EXPRESS_WALK
        if (!COUNT && express) {  // a trapped subpath alone in its wave: its delta chain out of line
            const bool alone = __popcll(__ballot(L.state != ST_IDLE)) == 1;
            if (alone && !tracing && !has_res && (L.state == ST_LIGHT || L.state == ST_EYE)) {
                if (express_walk(L, P->sc, P->fr, P->fb, stk, res, rt, ru, rv)) has_res = true;
                if (!has_res) {
                    long_walk = false;  // the chain ended: the lane's next step comes from the sweep
                    continue;
                }
            }
        }
#endif
        if (L.state != ST_IDLE && !tracing && !has_res) {  // a new query: begin its walk
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
#if BDPT_ROOT_LDS
                if (root_in_lds && !walk_begin_lds<COUNT, SLACK>(root_lds, L.ray, ri, q_any, ts, stk, cnt)) {
                    res = -1, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;  // no child hit: a miss
                    tracing = false;
                    has_res = true;
                }
#endif
            }
        }
        const uint64_t c0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        for (;;) {  // walk until enough lanes have a result to shade
            const uint64_t tr = __ballot(tracing);
            if (!tr) break;
            const uint64_t ready = __ballot(has_res);
            if (__popcll(ready) >= (express ? 1
                                    : BDPT_TAIL_SHADE == 1 && exhausted ? 1
                                    : BDPT_TAIL_SHADE == 2 && exhausted ? max(1, (__popcll(tr | ready) * BDPT_TAIL_FRAC) >> 3)
                                                                        : BDPT_SHADE_READY))
                break;
#if BDPT_TRAV_SPLIT
            // Lanes at a leaf and lanes at an interior node step in alternate
            // iterations (whichever group is larger in the sense of the ratio
            // below) instead of both code paths running in every iteration.
            const bool at_leaf = (ts.link & kLeafBit) != 0;
            const uint64_t lv = __ballot(tracing && at_leaf);
            const bool do_leaf = __popcll(lv) * 4 >= __popcll(tr & ~lv) * BDPT_TRAV_SPLIT;
            bool fin = tracing && at_leaf == do_leaf && trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
            // BDPT_WALK_UNROLL more interior-node steps before the wave's ballots
#pragma unroll
            for (int k = 0; k < BDPT_WALK_UNROLL; k++)
                if (!do_leaf && tracing && !fin && !(ts.link & kLeafBit))
                    fin = trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
            if (fin) {
#else
            if (tracing && trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt)) {
#endif
                res = ts.best, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                tracing = false;
                has_res = true;
            }
        }
        const uint64_t c1 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        if (has_res) {
            has_res = false;
#if BDPT_DEEP_RNG && BDPT_RING_AHEAD
            // the draws of this step past 227 are read from the ring: generate them first
            if (L.rng.n + BDPT_RING_AHEAD >= 227 && !mt_ring_ahead(L.rng) && P->fr.diag)
                gadd(P->fr.diag + kDiagErrors, 1ull);
#endif
            const uint64_t r0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t act = resolve<COUNT>(L, res, rt, ru, rv, P->sc, P->fr, P->fb, cnt);
            if (COUNT && first_active_lane()) cnt.c[20] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - r0);
            advance<COUNT>(L, act, P->sc, P->fr, P->fb, ls, cnt);
            if (BDPT_RR == 1) long_walk = L.state != ST_IDLE && L.c.depth > BDPT_EXPRESS_DEPTH;
        }
        if (COUNT && first_active_lane()) {
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
            cnt.c[12] += static_cast<uint32_t>(c1 - c0);
            cnt.c[13] += static_cast<uint32_t>(c2 - c1);
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
    if (COUNT) {
        if (lane0()) cnt.c[14] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - clock0);
        flush_counts(cnt, kp.counters);
    }
}

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
