// Wavefront schedule of the BDPT path — the default render path on MI355X.
//
// The megakernel (bdpt_kernels.hip) keeps every sample's state in registers
// next to the traversal, so one kernel needs the registers of both and runs at
// 3 waves per SIMD, too few to hide the dependent node loads of a BVH walk.
// Here the two halves are separate kernels that ping-pong over a pool of path
// slots whose state lives in HBM:
//
//   bdpt_shade_kernel  one thread per slot (coalesced state access): applies
//                      the result of the slot's last query (resolve), runs the
//                      integrator to the next query (advance), and starts a new
//                      camera sample when the slot's sample is done.
//   bdpt_trace_kernel  persistent and lean (more waves per SIMD): waves claim
//                      chunks of 64 slots, probe which hold a query, and hand
//                      those to idle lanes, refilling finished lanes while the
//                      rest of the wave keeps walking the 4-wide hierarchy.
//
// No queues: a slot's pending query is its ray record (min_t NaN = none;
// min_t < 0 = shadow ray, |min_t| the reference's value). Work is claimed from
// 64 partitioned counters (samples for shade, slot chunks for trace) so no
// single atomic address serialises the chip.
//
// Per pass every active slot has exactly one query, so a sample's sequence of
// queries — and every arithmetic operation on it — is the megakernel's (and
// the reference's); only the order of framebuffer additions differs.
//
// Slot state, HBM (float4 chunks, chunk k of slot s at lane[k * nslots + s]):
//   c0 rng a0 a1 b n   c1 pixel, state | pure << 8, steps, prim_tri
//   c2 cam_d, vc       c3 tp, vcm        c4 Li, depth      c5 hit p, dist
//   c6 hit n, mat      c7 hit wo, shape  c8 pend, pend_px  c9 nl, ci
// ray[2 s] = (o, min_t), ray[2 s + 1] = (d, max_t); res[s] = (t, u, v, leaf-
// order triangle index or -1; occluded 1 / -1 for shadow rays).
#include <hip/hip_runtime.h>

#include "bdpt_path.hpp"

namespace bdpt {
namespace dev {

constexpr int kShadeBlock = 256;
constexpr int kTraceBlock = 256;
#ifndef BDPT_TRACE_WAVES
#define BDPT_TRACE_WAVES 8  // waves per SIMD of the trace kernel
#endif
#ifndef BDPT_TRACE_LDS
#define BDPT_TRACE_LDS 8  // traversal-stack entries per lane in LDS (deeper ones in HBM)
#endif
#ifndef BDPT_REFILL_MIN
#define BDPT_REFILL_MIN 16  // idle lanes that trigger a wave's refill
#endif
constexpr int kTraceLds = BDPT_TRACE_LDS;
constexpr int kLaneChunks = 10;

struct WfParams {
    DevScene sc;
    DevFrame fr;
    float* fb;
    float* lv;
    uint2* gstack;
    float4* lane;     // kLaneChunks * nslots
    float4* ray;      // 2 * nslots
    float4* res;      // nslots
    unsigned long long* wctr;  // kParts sample counters + exhausted mask (bit p: partition p done)
    uint32_t* tctr;            // by parity p, 160 words at 160 p: [q] slot cursors (q < kParts), [64, 65] done
                               // mask lo / hi, [96 + q] "issued a query" flags of the shade pass
    unsigned long long* counters;
    uint32_t* sstack;  // shade kernel's link-stack overflow (entries >= shade_lds), or null
    uint32_t nslots;
    uint32_t trace_lanes;
    int32_t shade_lds;  // link-stack entries per lane in the shade kernel's dynamic LDS
};

__device__ __forceinline__ float4 f4(f3 a, float w) { return make_float4(a.x, a.y, a.z, w); }
__device__ __forceinline__ float4 f4i(int a, int b, int c, int d) {
    return make_float4(__int_as_float(a), __int_as_float(b), __int_as_float(c), __int_as_float(d));
}

__device__ __forceinline__ void load_lane(Lane& L, const WfParams& P, uint32_t s, float4 c1) {
    const uint32_t n = P.nslots;
    const float4* b = P.lane + s;
    const float4 c0 = gld4(b), c2 = gld4(b + 2 * n), c3 = gld4(b + 3 * n), c4 = gld4(b + 4 * n),
                 c5 = gld4(b + 5 * n), c6 = gld4(b + 6 * n), c7 = gld4(b + 7 * n), c8 = gld4(b + 8 * n),
                 c9 = gld4(b + 9 * n);
    L.rng = LazyMT{__float_as_uint(c0.x), __float_as_uint(c0.y), __float_as_uint(c0.z), __float_as_uint(c0.w)};
    L.c.pixel = __float_as_int(c1.x);
    const uint32_t sp = __float_as_uint(c1.y);
    L.state = sp & 0xffu;
    L.c.pure = (sp >> 8) & 1u;
    L.c.steps = __float_as_int(c1.z);
    L.c.prim_tri = __float_as_int(c1.w);
    L.c.cam_d = xyz(c2), L.c.vc = c2.w;
    L.c.tp = xyz(c3), L.c.vcm = c3.w;
    L.c.Li = xyz(c4), L.c.depth = __float_as_int(c4.w);
    L.h.p = xyz(c5), L.h.dist = c5.w;
    L.h.n = xyz(c6), L.h.mat = __float_as_int(c6.w);
    L.h.wo = xyz(c7), L.h.shape = __float_as_int(c7.w);
    L.c.pend = xyz(c8), L.c.pend_px = __float_as_int(c8.w);
    L.c.nl = __float_as_int(c9.x), L.c.ci = __float_as_int(c9.y);
    const float4 r0 = gld4(P.ray + 2 * s), r1 = gld4(P.ray + 2 * s + 1);
    L.ray = Ray{xyz(r0), xyz(r1), fabsf(r0.w), r1.w};
}

__device__ __forceinline__ void store_lane(const Lane& L, const WfParams& P, uint32_t s) {
    const uint32_t n = P.nslots;
    float4* b = P.lane + s;
    gst4(b, make_float4(__uint_as_float(L.rng.a0), __uint_as_float(L.rng.a1), __uint_as_float(L.rng.b),
                        __uint_as_float(L.rng.n)));
    gst4(b + n, f4i(L.c.pixel, static_cast<int>(L.state | (L.c.pure ? 0x100u : 0u)), L.c.steps, L.c.prim_tri));
    gst4(b + 2 * n, f4(L.c.cam_d, L.c.vc));
    gst4(b + 3 * n, f4(L.c.tp, L.c.vcm));
    gst4(b + 4 * n, f4(L.c.Li, __int_as_float(L.c.depth)));
    gst4(b + 5 * n, f4(L.h.p, L.h.dist));
    gst4(b + 6 * n, f4(L.h.n, __int_as_float(L.h.mat)));
    gst4(b + 7 * n, f4(L.h.wo, __int_as_float(L.h.shape)));
    gst4(b + 8 * n, f4(L.c.pend, __int_as_float(L.c.pend_px)));
    gst4(b + 9 * n, f4i(L.c.nl, L.c.ci, 0, 0));
    // min_t > 0 on every query the state machine issues; its sign marks shadow rays
    gst4(P.ray + 2 * s, f4(L.ray.o, is_shadow_state(L.state) ? -L.ray.min_t : L.ray.min_t));
    gst4(P.ray + 2 * s + 1, f4(L.ray.d, L.ray.max_t));
}

__device__ __forceinline__ void flush_wave_counts(const Counts& cnt, unsigned long long* out) {
    for (int i = 0; i < kCounters; i++) {
        unsigned long long v = cnt.c[i];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0 && v) atomicAdd(out + i, v);
    }
}

// Queries the trace kernel does not take: rays whose reciprocal direction or
// origin is not finite (the 4-wide tree's monotone-slab argument needs it),
// rays the reference culls at the root (min_t > max_t), and every query under
// BDPT_FLAG_FULL_TRAVERSAL. They are answered here, exactly as the reference
// walks its own binary tree; all others go to the trace queue.
template <bool FULL>
__device__ __forceinline__ bool needs_exact(const Ray& r) {
    return FULL || r.min_t > r.max_t || !ray_inv(r).fast;
}

// A 64-bit value made wave-uniform (readfirstlane works on 32-bit words; the
// halves are zero-extended — a sign-extended low word would fake set bits).
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v & 0xffffffffu)));
    const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(v >> 32)));
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

constexpr int kParts = 64;  // partitions of the sample range / slot range, one counter each

// Takes up to popc(want) new sample indices for the wanting lanes of the wave
// from the partitioned sample counters (start at partition `part`, move on when
// one is exhausted). Returns the lane's sample index or ~0 when none is left.
__device__ __forceinline__ uint64_t claim_samples(bool want, const WfParams& P, int part) {
    const uint64_t total = P.fr.total_samples;
    unsigned long long* const done = P.wctr + kParts;
    const int lane = threadIdx.x & 63;
    uint64_t pend = __ballot(want);
    uint64_t mine = ~0ull;
    for (int tries = 0; pend && tries < 2 * kParts; tries++) {
        const uint64_t dmask = uniform_u64(__atomic_load_n(done, __ATOMIC_RELAXED));
        if (dmask == ~0ull) break;
        if ((dmask >> part) & 1ull) {
            part = (part + 1) & (kParts - 1);
            continue;
        }
        const uint64_t lo = total * static_cast<uint64_t>(part) / kParts,
                       hi = total * static_cast<uint64_t>(part + 1) / kParts;
        const int n = __popcll(pend);
        unsigned long long b = 0;
        if (lane == 0) b = atomicAdd(P.wctr + part, static_cast<unsigned long long>(n));
        b = __shfl(b, 0);
        const uint64_t avail = lo + b >= hi ? 0 : hi - (lo + b);
        if (want && ((pend >> lane) & 1ull)) {
            const uint64_t rank = __popcll(pend & ((1ull << lane) - 1ull));
            if (rank < avail) mine = lo + b + rank;
        }
        pend &= ~__ballot(mine != ~0ull);
        if (avail < static_cast<uint64_t>(n)) {  // partition exhausted
            if (lane == 0) atomicOr(done, 1ull << part);
            part = (part + 1) & (kParts - 1);
        }
    }
    return mine;
}

// Shade pass: one thread per slot.
template <bool FULL, bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void bdpt_shade_kernel(const WfParams* __restrict__ pp, int parity) {
    const WfParams& P = *pp;
    scene_tables_to_lds(P.sc);
    uint32_t* const shade_stack = g_scene_lds + P.sc.lds_words;  // after the scene tables
    const uint32_t s = blockIdx.x * kShadeBlock + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < kParts + 2) P.tctr[160 * parity + threadIdx.x] = 0;  // this pass's trace
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    const uint64_t clock0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    const bool valid = s < P.nslots;
    __shared__ LaneCold cold_mem[kShadeBlock];
    Lane L(cold_mem[threadIdx.x]);
    L.state = ST_IDLE;
    L.c.pixel = 0;
    bool was_active = false;
    if (valid) {
        const float4 c1 = gld4(P.lane + P.nslots + s);
        if ((__float_as_uint(c1.y) & 0xffu) != ST_IDLE) {
            was_active = true;
            load_lane(L, P, s, c1);
            const float4 rs = gld4(P.res + s);
            const LightStore ls = light_store(P.lv, P.fr.rr_depth, s);
            const uint32_t act = resolve<COUNT>(L, __float_as_int(rs.w), rs.x, rs.y, rs.z, P.sc, P.fr, P.fb, cnt);
            advance<COUNT>(L, act, P.sc, P.fr, P.fb, ls, cnt);
            run_deferred<COUNT>(L, P.sc, P.fr, P.fb, ls, cnt);
        }
    }
    // Slots whose sample is done take the next one.
    const bool want = valid && L.state == ST_IDLE;
    if (__ballot(want)) {
        const uint64_t my = claim_samples(want, P, static_cast<int>((blockIdx.x * (kShadeBlock / 64) +
                                                                     (threadIdx.x >> 6)) & (kParts - 1)));
        if (want && my != ~0ull) start_sample(L, my, P.fr);
    }
    if (valid && L.state != ST_IDLE && needs_exact<FULL>(L.ray)) {  // rare, divergent (all under FULL)
        const LinkStack lstk{shade_stack + threadIdx.x, kShadeBlock, P.shade_lds, P.sstack, P.nslots, s};
        const LightStore ls = light_store(P.lv, P.fr.rr_depth, s);
        do {
            const bool any = is_shadow_state(L.state);
            if (COUNT) cnt.c[any ? 1 : 0]++;
            TravResult q{-1, L.ray.max_t, 0.f, 0.f, 0u, 0u, 0u};
            if (!(L.ray.min_t > L.ray.max_t)) q = traverse_binary<COUNT, LinkStack>(P.sc, L.ray, any, !FULL, lstk);
            if (COUNT) cnt.c[2] += q.nodes, cnt.c[3] += q.tris, cnt.c[15] += q.exact;
            const uint32_t act = resolve<COUNT>(L, q.best, q.t, q.u, q.v, P.sc, P.fr, P.fb, cnt);
            advance<COUNT>(L, act, P.sc, P.fr, P.fb, ls, cnt);
            run_deferred<COUNT>(L, P.sc, P.fr, P.fb, ls, cnt);
        } while (L.state != ST_IDLE && needs_exact<FULL>(L.ray));
        was_active = true;
    }
    if (__ballot(valid && L.state != ST_IDLE) && (threadIdx.x & 63) == 0)
        P.tctr[160 * parity + 96 + (blockIdx.x & (kParts - 1))] = 1u;  // tells the host work is left
    if (valid && L.state != ST_IDLE) {
        store_lane(L, P, s);
    } else if (was_active) {  // no query: idle state, and a NaN min_t the trace pass skips
        gst4(P.lane + P.nslots + s, f4i(L.c.pixel, ST_IDLE, 0, 0));
        gst4(P.ray + 2 * s, make_float4(0.f, 0.f, 0.f, __builtin_nanf("")));
    }
    if (COUNT) {
        if ((threadIdx.x & 63) == 0) cnt.c[13] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - clock0);
        flush_wave_counts(cnt, P.counters);
    }
}

// Trace pass: persistent. A wave claims 64-slot chunks from partitioned
// cursors, probes which slots hold a query, and deals them to its idle lanes
// (through a per-wave LDS table) whenever enough lanes are idle.
template <bool COUNT>
__global__ __launch_bounds__(kTraceBlock, BDPT_TRACE_WAVES) void bdpt_trace_kernel(const WfParams* __restrict__ pp,
                                                                                     int parity) {
    const WfParams& P = *pp;
    __shared__ uint2 stack_mem[kTraceLds * kTraceBlock];
    __shared__ uint8_t deal[kTraceBlock / 64][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const Stack stk{stack_mem + threadIdx.x, kTraceBlock, kTraceLds, P.gstack, P.trace_lanes,
                    blockIdx.x * kTraceBlock + threadIdx.x};
    uint32_t* const cur = P.tctr + 160 * parity;
    if (blockIdx.x == 0 && threadIdx.x < kParts) P.tctr[160 * (1 - parity) + 96 + threadIdx.x] = 0;  // next shade
    uint32_t* const done = cur + kParts;  // [0] bits 0..31, [1] bits 32..63
    const uint32_t nslots = P.nslots;
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    const uint64_t clock0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    bool has = false, any = false;
    uint32_t slot = 0;
    Ray r{};
    RayInv ri{};
    TravState ts{};
    bool exhausted = false;  // wave-uniform
    const TravScene tsc = trav_scene(P.sc);
    int part = static_cast<int>((blockIdx.x * (kTraceBlock / 64) + wave) & (kParts - 1));
    uint64_t pending = 0;  // wave-uniform: probed slots of the chunk not dealt yet
    uint32_t cbase = 0;
    for (;;) {
        if (!exhausted) {
            const uint64_t idle = __ballot(!has);
            const int n = __popcll(idle);
            if (n >= BDPT_REFILL_MIN || n == 64) {
                while (pending == 0 && !exhausted) {
                    const uint64_t dm =
                        uniform_u64(static_cast<uint64_t>(__atomic_load_n(done, __ATOMIC_RELAXED)) |
                                    (static_cast<uint64_t>(__atomic_load_n(done + 1, __ATOMIC_RELAXED)) << 32));
                    if (dm == ~0ull) {
                        exhausted = true;
                        break;
                    }
                    if ((dm >> part) & 1ull) {
                        part = (part + 1) & (kParts - 1);
                        continue;
                    }
                    const uint32_t lo = static_cast<uint32_t>(static_cast<uint64_t>(nslots) * part / kParts),
                                   hi = static_cast<uint32_t>(static_cast<uint64_t>(nslots) * (part + 1) / kParts);
                    uint32_t b = 0;
                    if (lane == 0) b = atomicAdd(cur + part, 64u);
                    b = __shfl(b, 0);
                    if (lo + b >= hi) {
                        if (lane == 0) atomicOr(done + (part >> 5), 1u << (part & 31));
                        part = (part + 1) & (kParts - 1);
                        continue;
                    }
                    cbase = lo + b;
                    bool act = false;
                    if (cbase + lane < hi) act = !__builtin_isnan(gld4(P.ray + 2 * (cbase + lane)).w);
                    pending = __ballot(act);
                }
                if (pending) {
                    // lane j holding the rank-k pending slot deals it to the rank-k idle lane
                    const uint32_t rank_p = static_cast<uint32_t>(__popcll(pending & ((1ull << lane) - 1ull)));
                    const bool take = ((pending >> lane) & 1ull) && rank_p < static_cast<uint32_t>(n);
                    if (take) deal[wave][rank_p] = static_cast<uint8_t>(lane);
                    __builtin_amdgcn_wave_barrier();
                    const uint32_t rank_i = static_cast<uint32_t>(__popcll(idle & ((1ull << lane) - 1ull)));
                    const uint32_t dealt = static_cast<uint32_t>(__popcll(pending));
                    if (!has && rank_i < dealt) {
                        slot = cbase + deal[wave][rank_i];
                        const float4 r0 = gld4(P.ray + 2 * slot), r1 = gld4(P.ray + 2 * slot + 1);
                        any = r0.w < 0.f;
                        r = Ray{xyz(r0), xyz(r1), fabsf(r0.w), r1.w};
                        if (COUNT) cnt.c[any ? 1 : 0]++;
                        ri = ray_inv(r);  // finite and min_t <= max_t: the shade kernel took the others
                        ts = trav_begin(tsc, r);
                        has = true;
                    }
                    __builtin_amdgcn_wave_barrier();
                    pending &= ~__ballot(take);
                }
            }
        }
        if (!__ballot(has)) {
            if (exhausted) break;
            continue;
        }
        if (has && trav_step<COUNT>(tsc, r, ri, any, ts, stk, cnt)) {
            gst4(P.res + slot, make_float4(ts.best_t, ts.best_u, ts.best_v, __int_as_float(ts.best)));
            has = false;
        }
    }
    if (COUNT) {
        if (lane == 0) cnt.c[12] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - clock0);
        flush_wave_counts(cnt, P.counters);
    }
}

}  // namespace dev

// ------------------------------------------------------------ host launchers
size_t wf_params_bytes() { return sizeof(dev::WfParams); }
int wf_lane_chunks() { return dev::kLaneChunks; }
int wf_trace_block() { return dev::kTraceBlock; }
int wf_trace_lds_stack() { return dev::kTraceLds; }
int wf_shade_block() { return dev::kShadeBlock; }
int wf_parts() { return dev::kParts; }

int wf_trace_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::bdpt_trace_kernel<false>, dev::kTraceBlock, 0) !=
            hipSuccess ||
        n <= 0)
        n = 1;
    return n;
}

// Fills the parameter block (device buffer `dparams`, stream-ordered).
hipError_t wf_set_params(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lv, uint2* gstack,
                         float4* lane, float4* ray, float4* res, unsigned long long* wctr, uint32_t* tctr,
                         unsigned long long* counters, uint32_t* sstack, uint32_t nslots, uint32_t trace_lanes,
                         int shade_lds, void* dparams, hipStream_t stream) {
    const dev::WfParams host{sc,       fr,     fb,     lv,          gstack,   lane, ray, res, wctr,
                             tctr,     counters, sstack, nslots, trace_lanes, shade_lds};
    return hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
}

// One pass: shade (resolve + advance + refill + enqueue), then trace.
hipError_t wf_launch_pass(const void* dparams, uint32_t flags, uint32_t nslots, int trace_grid, int shade_lds,
                          uint32_t p_lds_words, int64_t pass, hipStream_t stream) {
    const int parity = static_cast<int>(pass & 1);
    const bool full = (flags & 2u) != 0, count = (flags & 1u) != 0;
    const dev::WfParams* p = static_cast<const dev::WfParams*>(dparams);
    const dim3 gs((nslots + dev::kShadeBlock - 1) / dev::kShadeBlock), bs(dev::kShadeBlock);
    const size_t lds = sizeof(uint32_t) * (dev::kShadeBlock * static_cast<size_t>(shade_lds) + p_lds_words);
    if (full && count) hipLaunchKernelGGL((dev::bdpt_shade_kernel<true, true>), gs, bs, lds, stream, p, parity);
    else if (full) hipLaunchKernelGGL((dev::bdpt_shade_kernel<true, false>), gs, bs, lds, stream, p, parity);
    else if (count) hipLaunchKernelGGL((dev::bdpt_shade_kernel<false, true>), gs, bs, lds, stream, p, parity);
    else hipLaunchKernelGGL((dev::bdpt_shade_kernel<false, false>), gs, bs, lds, stream, p, parity);
    const dim3 gt(trace_grid), bt(dev::kTraceBlock);
    if (count) hipLaunchKernelGGL((dev::bdpt_trace_kernel<true>), gt, bt, 0, stream, p, parity);
    else hipLaunchKernelGGL((dev::bdpt_trace_kernel<false>), gt, bt, 0, stream, p, parity);
    return hipGetLastError();
}

}  // namespace bdpt
