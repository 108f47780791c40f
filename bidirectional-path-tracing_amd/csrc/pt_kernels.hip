// HIP kernel for the reference's other offline integrator, PathTracerIntegrator
// (src/integrators/path.h): the explicit path tracer (Russian roulette past
// rrDepth, indirect re-sampling while an emitter is hit, direct light from
// emitter samples and BSDF samples combined with the balance heuristic) and the
// implicit one. It runs on the BDPT path's substrate — the same 4-wide
// traversal with the reference's exact hit semantics, BSDFs, emitter sampling,
// camera rays and per-(pixel, sample) MT19937 seeding — as a separate
// persistent kernel, so the BDPT megakernel's register allocation is untouched.
//
// The reference recursion (recursiveExplicit calls itself BEFORE computing its
// own level's direct light, so the random-number order is: level d's Russian
// roulette and indirect sample(s), then everything below, then level d's
// direct light) runs as a per-lane state machine with an explicit stack of
// levels in HBM. Path length is unbounded under Russian roulette, so the
// generator is the lazy MT19937 of the BDPT path for the first 227 draws and,
// for the rare longer samples, a 624-word ring of this lane's untempered
// outputs in HBM (u[n + 624] = u[n + 397] ^ twist(u[n], u[n + 1])).
#include <hip/hip_runtime.h>

#include <cstring>

#ifndef BDPT_BSDF_TABLE
#define BDPT_BSDF_TABLE 0  // the path / direct frame kernels read the LDS table only
#endif
#include "bdpt_path.hpp"

namespace bdpt {
namespace dev {

// ------------------------------------------------------------- generator
struct PtRng {
    LazyMT m;          // draws 0 .. 226 need no memory
    uint32_t seed;
    uint32_t* ring;    // this lane's 624 words: word k at ring[k * stride]
    uint32_t stride;
};

// Output n >= 227 of std::mt19937(seed) from the lane's ring (mt_ring_step).
__device__ BDPT_NOINLINE uint32_t pt_u32_slow(PtRng& r) { return mt_ring_step(r.m, r.seed, r.ring, r.stride); }
__device__ __forceinline__ float next1(PtRng& r) {
#if BDPT_SAMPLER_STATE
    const uint32_t u = mt_state_u32();  // the caller's std::mt19937 (single-sample build)
    r.m.n++;
#else
    const uint32_t u = r.m.n < 227 ? mt_next_u32(r.m) : pt_u32_slow(r);
#endif
    const float f = static_cast<float>(u) / 4294967296.0f;  // generate_canonical (random.tcc:3348-3380)
    return f >= 1.0f ? 0x1.fffffep-1f : f;
}
__device__ __forceinline__ F2 next2(PtRng& r) {
    F2 o;
    o.x = next1(r);
    o.y = next1(r);
    return o;
}

// ------------------------------------------------------------ parameters
struct PtSettings {
    int32_t is_explicit, max_depth, rr_depth;
    float rr_prob;
    int32_t emitter_samples, bsdf_samples;
    int32_t max_levels;  // capacity of the level stack
    int32_t direct;      // 1..5: DirectIntegrator with samplingStrategy area, solidAngle,
                         // cosineHemisphere, bsdf, mis (direct.h:430-442); 0: the path tracer
};
enum : int32_t { DI_AREA = 1, DI_SOLID_ANGLE = 2, DI_COSINE = 3, DI_BSDF = 4, DI_MIS = 5 };

struct PtParams {
    DevScene sc;
    DevFrame fr;
    PtSettings ps;
    float* fb;
    float4* levels;       // per slot max_levels x 5 float4
    uint32_t* ring;       // 624 words per slot, word-major
    uint2* gstack;        // traversal-stack overflow
    uint32_t nslots;
    unsigned long long* work;
    unsigned long long* counters;  // [0] closest rays (counting pass), [1] level-stack overflows,
                                   // [2] samples past 227 draws, [3] past 624 draws, [7] RNG draws (counting pass)
    float* li_out;                 // single-sample launch: Li is written here instead of the framebuffer
};

enum : uint32_t {  // the query a lane waits on / the step it resumes at
    PQ_NONE = 0,
    PQ_PRIMARY,  // render(): primary hit (path.h:238)
    PQ_IND,      // explicit indirect sample (path.h:90)
    PQ_DIRE,     // explicit direct light, emitter sample (path.h:134)
    PQ_DIRB,     // explicit direct light, BSDF sample (path.h:162)
    PQ_IMP,      // implicit (path.h:43)
    PQ_DI_E,     // direct integrator, emitter / cosine sample (direct.h:177, :216, :275, :345)
    PQ_DI_B,     // direct integrator, BSDF sample (direct.h:249, :387)
};

struct PtLane {
    PtRng rng;
    uint32_t q;  // PQ_*
    bool busy;
    Ray ray;
    Hit h;                      // the current level's vertex
    int depth, pixel;
    // current level (explicit)
    float rr, pdf, cum;
    uint32_t nsamp;
    f3 f, ind, eest, best;
    int i;                      // direct-light sample counter
    // pending direct-light query
    int e_shape;
    float e_cos, e_d2, e_pdf, e_apdf;
    f3 e_wil, b_f, wiw;
    float b_pdf;
    int e_id;                   // direct integrator: the sampled emitter
};

__device__ __forceinline__ f3 emission_of(const DevScene& sc, int mat) { return ld3(bsdf_of(sc, mat).emission); }

__device__ __forceinline__ float balance_heuristic(float nf, float fPdf, float ng, float gPdf) {  // path.h:31-34
    const float f = nf * fPdf, g = ng * gPdf;
    return div_cr(f, f + g);
}

// Level stack record d of the lane: the level's vertex and its indirect sample.
__device__ __forceinline__ float4* level_at(const PtParams& P, uint32_t slot, int d) {
    return P.levels + (static_cast<size_t>(slot) * P.ps.max_levels + static_cast<uint32_t>(d)) * 5;
}
__device__ __forceinline__ void push_level(const PtParams& P, uint32_t slot, const PtLane& L) {
    float4* q = level_at(P, slot, L.depth);
    gst4(q, make_float4(L.h.p.x, L.h.p.y, L.h.p.z, L.rr));
    gst4(q + 1, make_float4(L.h.n.x, L.h.n.y, L.h.n.z, L.pdf));
    gst4(q + 2, make_float4(L.h.wo.x, L.h.wo.y, L.h.wo.z, __int_as_float(L.h.mat)));
    gst4(q + 3, make_float4(L.f.x, L.f.y, L.f.z, __int_as_float(L.h.shape)));
    gst4(q + 4, make_float4(__uint_as_float(L.nsamp), L.cum, 0.f, 0.f));
}
__device__ __forceinline__ void pop_level(const PtParams& P, uint32_t slot, PtLane& L) {
    const float4* q = level_at(P, slot, L.depth);
    const float4 a = gld4(q), b = gld4(q + 1), c = gld4(q + 2), d = gld4(q + 3), e = gld4(q + 4);
    L.h.p = xyz(a), L.rr = a.w;
    L.h.n = xyz(b), L.pdf = b.w;
    L.h.wo = xyz(c), L.h.mat = __float_as_int(c.w);
    L.f = xyz(d), L.h.shape = __float_as_int(d.w);
    L.nsamp = __float_as_uint(e.x), L.cum = e.y;
}

__device__ __forceinline__ Ray pt_ray(f3 o, f3 d) {
    return Ray{o, d, kEpsilon, __builtin_inff()};  // Ray(hit.p, wiW, Epsilon, infinity)
}

// Finishes the sample: rgb[p] += Li * (1 / spp) (renderer.cpp:202, one sample at a time).
__device__ __forceinline__ void pt_finish(PtLane& L, const PtParams& P, f3 Li) {
    if (P.li_out) {  // Integrator::render(ray, sampler) returns Li to its caller
        P.li_out[0] = Li.x, P.li_out[1] = Li.y, P.li_out[2] = Li.z;
    } else if (Li.x != 0.f || Li.y != 0.f || Li.z != 0.f) {
        const float inv_spp = 1.f / static_cast<float>(P.fr.spp);
        float* px = P.fb + 3 * static_cast<size_t>(L.pixel);
        gadd(px + 0, Li.x * inv_spp);
        gadd(px + 1, Li.y * inv_spp);
        gadd(px + 2, Li.z * inv_spp);
    }
    if (L.rng.m.n > 227) gadd(P.counters + 2, 1ull);  // the sample ran on the ring generator
    if (L.rng.m.n > 624) gadd(P.counters + 3, 1ull);  // ... past its first wrap
    L.busy = false;
    L.q = PQ_NONE;
}

// quadratic + raySphereIntersect (direct.h:17-67) in double, as there: true
// when a root lies strictly inside (min_t, max_t).
__device__ BDPT_NOINLINE bool ray_sphere_hit(Ray r, f3 center, float radius) {
    const f3 no = r.o - center;
    const double cc = static_cast<double>(dot(no, no) - (radius * radius));
    const double b = static_cast<double>(dot(no, r.d)) * 2.0;
    const double a = static_cast<double>(dot(r.d, r.d));
    const double disc = b * b - 4 * a * cc;
    double t0, t1;
    if (disc > 0) {
        const double sq = __builtin_sqrt(disc);
        const double inv2a = 1 / (2 * a);
        t0 = (-b + sq) * inv2a;
        t1 = (-b - sq) * inv2a;
    } else if (disc == 0) {
        t0 = (-b + __builtin_sqrt(disc)) / (2 * a);
        t1 = t0;
    } else {
        return false;
    }
    const double lo = r.min_t, hi = r.max_t;
    return (t0 > lo && t0 < hi) || (t1 > lo && t1 < hi);
}
// Warp::squareToUniformSphere (math.h:119-127)
__device__ __forceinline__ f3 uniform_sphere(F2 u) {
    const float phi = u.x * kPi * 2.0f;
    const float cosTheta = 1.f - (2.f * u.y);
    const float sinTheta = sqrt_cr(glibc_fmaxf(1.f - cosTheta * cosTheta, 0.f));
    const SinCos sc = glibc_sincosf2(phi);
    return mk(sinTheta * sc.c, sinTheta * sc.s, cosTheta);
}
// sampleSphereBySolidAngle (direct.h:109-141)
__device__ __forceinline__ f3 sphere_solid_angle(F2 u, f3 p, f3 center, float radius, float& pdf) {
    const f3 cdir = normalize(center - p);
    const f3 dd = center - p;
    const float sin2 = radius * radius / dot(dd, dd);
    const float cosMax = sqrt_cr(glibc_fmaxf(0.f, 1.f - sin2));
    const float cosTheta = (1.f - u.x) + (u.x * cosMax);
    const float phi = u.y * kPi * 2.0f;
    const float sinTheta = sqrt_cr(glibc_fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    const SinCos sc = glibc_sincosf2(phi);
    pdf = kInvTwoPi * rcp_cr(1.f - cosMax);
    return world_at(cdir, mk(sinTheta * sc.c, sinTheta * sc.s, cosTheta));
}

enum : int {  // explicit-level steps between queries
    PS_ENTER,       // recursiveExplicit entry: Russian roulette (path.h:67-74)
    PS_IND_SAMPLE,  // indirect: sample the BSDF, trace (path.h:86-92)
    PS_DIRE,        // direct light, next emitter sample (path.h:120-153)
    PS_DIRB,        // direct light, next BSDF sample (path.h:156-186)
    PS_LEVEL_DONE,  // Lr = direct + indirect, RR scaling, return (path.h:187-198)
    PS_RETURN,      // hand Lr to the caller level (path.h:106) or finish the sample
    PS_IMP_LEVEL,   // recursiveImplicit entry (path.h:36-44)
    PS_IMP_RETURN,  // Li * brdfCosTheta * (1.0 / pdf) up the implicit recursion
    PS_DI_EMIT,     // direct integrator: next emitter / cosine sample
    PS_DI_BSDF,     // direct integrator: next BSDF sample
    PS_WAIT,        // a query was issued
};

// Runs the lane from step `ps` until it issues a query or finishes its sample.
#ifndef PT_INLINE_ADVANCE
#define PT_INLINE_ADVANCE 1  // pt_advance inlined: the lane state stays in registers (not scratch)
#endif
// The overlapped walk / advance schedule (as the BDPT megakernel's) runs for
// the path tracer (+9 % on Caustic, 512²×64); the direct integrator's one-level
// samples are faster without it (1439 vs 1334 Msamples/s).
#ifndef PT_SHADE_READY
#define PT_SHADE_READY 56
#endif
#ifndef PT_TRAV_SPLIT
#define PT_TRAV_SPLIT 8
#endif
#ifndef PT_WALK_UNROLL
#define PT_WALK_UNROLL 1  // extra interior-node steps per walk iteration, after either kind of step (path +0.8 %)
#endif
#ifndef PT_EARLY_COS
#define PT_EARLY_COS 1  // emitter samples rejected on the cosine (dot(v, n), the frame z) before the shading frame is built (+0.7 % path tracer)
#endif
#ifndef PT_ROOT_LDS
#define PT_ROOT_LDS 1  // the overlapped schedule's walks start two levels down (RootLds, as the BDPT megakernel)
#endif
#ifndef PT_WAVES_PER_EU
#define PT_WAVES_PER_EU 4  // 128 VGPRs, 4 blocks of 256 lanes per CU
#endif
#if PT_INLINE_ADVANCE
__device__ __forceinline__
#else
__device__
#endif
void pt_advance(PtLane& L, int ps, f3 Lr, const PtParams& P, uint32_t slot) {
    const DevScene& sc = P.sc;
    const PtSettings& S = P.ps;
    for (int guard = 0; guard < 1 << 20; guard++) {
        switch (ps) {
            case PS_ENTER: {
                L.rr = next1(L.rng);
                const bool enter = L.depth < S.max_depth ||
                                   (S.max_depth == -1 && (L.depth < S.rr_depth || L.rr < S.rr_prob));
                if (!enter) {
                    Lr = mk(0.f, 0.f, 0.f);
                    ps = PS_RETURN;
                    break;
                }
                L.nsamp = 0;
                L.ind = mk(0.f, 0.f, 0.f);
                ps = PS_IND_SAMPLE;
                break;
            }
            case PS_IND_SAMPLE: {
                const F2 u = next2(L.rng);
                f3 wi;
                L.f = bsdf_sample(bsdf_of(sc, L.h.mat), L.h.wo, u, wi, L.pdf);
                L.ray = pt_ray(L.h.p, world_at(L.h.n, wi));
                L.nsamp++;
                L.q = PQ_IND;
                return;
            }
            case PS_DIRE: {
                if (L.i >= S.emitter_samples) {
                    if (S.emitter_samples != 0) L.eest = L.eest / static_cast<float>(S.emitter_samples);
                    L.i = 0;
                    ps = PS_DIRB;
                    break;
                }
                L.i++;
                float epdf, eapdf;
                f3 en, ep;
                const int id = sample_emitter(sc, L.rng, epdf, en, ep, eapdf);
                const f3 wiW = normalize(ep - L.h.p);
#if PT_EARLY_COS
                const f3 dd = L.h.p - ep;  // glm::distance2(positionOut, hit.p)
                const float d2 = dot(dd, dd);
                const float cosOut = dot(-wiW, en);
                if (cosOut > 0.f && dot(wiW, L.h.n) > 0.f) {  // dot(v, n) = the frame's z (to_local)
                    const f3 wil = local_at(L.h.n, wiW);
#else
                const f3 wil = local_at(L.h.n, wiW);
                const f3 dd = L.h.p - ep;  // glm::distance2(positionOut, hit.p)
                const float d2 = dot(dd, dd);
                const float cosOut = dot(-wiW, en);
                if (cosOut > 0.f && wil.z > 0.f) {
#endif
                    L.e_shape = emitter_of(sc, id).shape;
                    L.e_cos = cosOut, L.e_d2 = d2, L.e_pdf = epdf, L.e_apdf = eapdf, L.e_wil = wil;
                    L.ray = pt_ray(L.h.p, wiW);
                    L.q = PQ_DIRE;
                    return;
                }
                break;  // next emitter sample
            }
            case PS_DIRB: {
                if (L.i >= S.bsdf_samples) {
                    if (S.bsdf_samples != 0) L.best = L.best / static_cast<float>(S.bsdf_samples);
                    ps = PS_LEVEL_DONE;
                    break;
                }
                L.i++;
                const F2 u = next2(L.rng);
                f3 wi;
                float pdf;
                const f3 f = bsdf_sample(bsdf_of(sc, L.h.mat), L.h.wo, u, wi, pdf);
                if (!is_zero(f)) {
                    L.b_f = f, L.b_pdf = pdf;
                    L.wiw = world_at(L.h.n, wi);
                    L.ray = pt_ray(L.h.p, L.wiw);
                    L.q = PQ_DIRB;
                    return;
                }
                break;
            }
            case PS_LEVEL_DONE: {
                const f3 direct = L.eest + L.best;
                Lr = direct + L.ind;
                if (S.max_depth == -1 && !(L.depth < S.rr_depth) && (L.rr < S.rr_prob)) Lr = Lr * rcp_cr(S.rr_prob);
                ps = PS_RETURN;
                break;
            }
            case PS_RETURN: {
                if (L.depth == 0) {
                    pt_finish(L, P, Lr);
                    return;
                }
                L.depth--;
                pop_level(P, slot, L);
                // indirectEstimator = Li * brdfCosTheta * (1/pdf) * (1/nSamples) * (1/cumRRProb) (path.h:106)
                L.ind = ((Lr * L.f) * rcp_cr(L.pdf)) * rcp_cr(static_cast<float>(L.nsamp));
                L.ind = L.ind * rcp_cr(L.cum);
                L.eest = mk(0.f, 0.f, 0.f), L.best = mk(0.f, 0.f, 0.f);
                L.i = 0;
                ps = PS_DIRE;
                break;
            }
            case PS_IMP_LEVEL: {
                if (!(L.depth < S.max_depth)) {
                    Lr = mk(0.f, 0.f, 0.f);
                    ps = PS_IMP_RETURN;
                    break;
                }
                const F2 u = next2(L.rng);
                f3 wi;
                L.f = bsdf_sample(bsdf_of(sc, L.h.mat), L.h.wo, u, wi, L.pdf);
                L.wiw = world_at(L.h.n, wi);
                L.ray = pt_ray(L.h.p, L.wiw);
                L.q = PQ_IMP;
                return;
            }
            case PS_IMP_RETURN: {
                if (L.depth == 0) {
                    pt_finish(L, P, Lr);
                    return;
                }
                L.depth--;
                pop_level(P, slot, L);
                Lr = (Lr * L.f) * rcp_cr(L.pdf);  // Li * brdfCosTheta * (1.0 / pdf) (path.h:50, :56)
                ps = PS_IMP_RETURN;
                break;
            }
            case PS_DI_EMIT: {  // renderArea / renderSolidAngle / renderCosineHemisphere / renderMIS
                const int st = S.direct;
                if (st == DI_BSDF) {
                    ps = PS_DI_BSDF;
                    break;
                }
                if (L.i >= S.emitter_samples) {
                    if (st == DI_MIS) {
                        if (S.emitter_samples != 0) L.eest = L.eest / static_cast<float>(S.emitter_samples);
                        else L.eest = mk(0.f, 0.f, 0.f);
                        L.i = 0;
                        ps = PS_DI_BSDF;
                        break;
                    }
                    pt_finish(L, P, L.ind / static_cast<float>(S.emitter_samples));  // Lr /= m_emitterSamples
                    return;
                }
                L.i++;
                if (st == DI_COSINE) {  // direct.h:214-229
                    const f3 local = cosine_hemisphere(next2(L.rng));
                    L.e_wil = local;
                    L.ray = pt_ray(L.h.p, normalize(world_at(L.h.n, local)));
                    L.q = PQ_DI_E;
                    return;
                }
                float epdf;
                const uint32_t n = static_cast<uint32_t>(sc.nemit);
                uint32_t id = static_cast<uint32_t>(next1(L.rng) * static_cast<float>(n));  // selectEmitter
                id = id < n - 1 ? id : n - 1;
                epdf = 1.f / static_cast<float>(n);
                const EmitterRecord& e = emitter_of(sc, static_cast<int>(id));
                const f3 center = ld3(e.center);
                const F2 u = next2(L.rng);
                if (st == DI_AREA) {  // direct.h:160-190, sampleSphereByArea :94-107
                    const f3 ne = uniform_sphere(u);
                    const f3 pos = ne * e.radius + center;
                    const f3 wiW = normalize(pos - L.h.p);
                    const float pdf = 1.f / (((4 * kPi) * e.radius) * e.radius);
                    const f3 dd = L.h.p - pos;
                    const float d2 = dot(dd, dd);
                    const float cosOut = dot(-wiW, ne);
#if PT_EARLY_COS
                    if (cosOut <= 0.f || dot(wiW, L.h.n) <= 0.f) break;
                    const f3 wil = local_at(L.h.n, wiW);
#else
                    const f3 wil = local_at(L.h.n, wiW);
                    if (cosOut <= 0.f || wil.z <= 0.f) break;
#endif
                    L.e_id = static_cast<int>(id), L.e_pdf = epdf, L.e_apdf = pdf, L.e_wil = wil;
                    L.e_cos = cosOut * rcp_cr(d2);  // areaToSolidAngle
                    L.ray = Ray{L.h.p, wiW, kEpsilon, sqrt_cr(d2) - kEpsilon};
                    L.q = PQ_DI_E;
                    return;
                }
                float pdf;  // solid angle (direct.h:262-309) or MIS (:333-372)
                const f3 wiW = sphere_solid_angle(u, L.h.p, center, e.radius, pdf);
#if PT_EARLY_COS
                if (dot(wiW, L.h.n) <= 0.f) break;
                const f3 wil = local_at(L.h.n, wiW);
#else
                const f3 wil = local_at(L.h.n, wiW);
                if (wil.z <= 0.f) break;
#endif
                L.e_id = static_cast<int>(id), L.e_pdf = epdf, L.e_apdf = pdf, L.e_wil = wil;
                const f3 dc = center - L.h.p;
                L.ray = Ray{L.h.p, wiW, kEpsilon, st == DI_SOLID_ANGLE ? sqrt_cr(dot(dc, dc)) + kEpsilon
                                                                       : __builtin_inff()};
                L.q = PQ_DI_E;
                return;
            }
            case PS_DI_BSDF: {  // renderBSDF (direct.h:245-260) / renderMIS (:382-418)
                if (L.i >= S.bsdf_samples) {
                    if (S.direct == DI_BSDF) {
                        pt_finish(L, P, L.ind / static_cast<float>(S.bsdf_samples));  // Lr /= m_bsdfSamples
                        return;
                    }
                    if (S.bsdf_samples != 0) L.best = L.best / static_cast<float>(S.bsdf_samples);
                    else L.best = mk(0.f, 0.f, 0.f);
                    pt_finish(L, P, L.ind + (L.eest + L.best));  // Lr += emitterEstimator + bsdfEstimator
                    return;
                }
                L.i++;
                f3 wi;
                float pdf;
                L.b_f = bsdf_sample(bsdf_of(sc, L.h.mat), L.h.wo, next2(L.rng), wi, pdf);
                L.b_pdf = pdf;
                L.ray = pt_ray(L.h.p, world_at(L.h.n, wi));
                L.q = PQ_DI_B;
                return;
            }
            default:
                return;
        }
    }
    pt_finish(L, P, mk(0.f, 0.f, 0.f));  // unreachable guard
}

// Applies the closest-hit result of the lane's query and continues.
template <bool COUNT>
__device__ __forceinline__ void pt_resolve(PtLane& L, int res, float t, float u, float v, const PtParams& P,
                                           uint32_t slot, Counts& cnt) {
    const DevScene& sc = P.sc;
    const PtSettings& S = P.ps;
    bool hit = res >= 0 && t <= L.ray.max_t && t >= L.ray.min_t;  // accel.h:133
    Hit vis;
    vis.mat = 0, vis.shape = 0;  // a value-initialised SurfaceInteraction on a miss (path.h:84)
    if (hit) shade_hit(sc, res, u, v, t, L.ray.d, vis);
    const uint32_t q = L.q;
    L.q = PQ_NONE;
    const f3 zero = mk(0.f, 0.f, 0.f);
    switch (q) {
        case PQ_PRIMARY: {  // render / renderExplicit / renderImplicit (path.h:204-245)
            if (!hit) return pt_finish(L, P, zero);
            const f3 le = emission_of(sc, vis.mat);
            if (!is_zero(le)) return pt_finish(L, P, le);
            L.h = vis;
            L.depth = 0;
            if (S.direct) {
                L.i = 0;
                L.ind = zero, L.eest = zero, L.best = zero;  // Lr, emitterEstimator, bsdfEstimator
                return pt_advance(L, PS_DI_EMIT, zero, P, slot);
            }
            return pt_advance(L, S.is_explicit ? PS_ENTER : PS_IMP_LEVEL, zero, P, slot);
        }
        case PQ_IND: {  // the do-while of path.h:82-95 and the recursion test of :98-108
            const bool emitter = !is_zero(emission_of(sc, vis.mat));
            if (emitter && next1(L.rng) < 0.95f) return pt_advance(L, PS_IND_SAMPLE, zero, P, slot);
            L.cum = L.nsamp > 1 ? 0.95f : 1.f;
            L.eest = zero, L.best = zero;
            L.i = 0;
            if (hit && !is_zero(L.f) && !emitter) {
                if (L.depth + 1 >= S.max_levels) {  // out of level stack: flagged, the sample ends
                    gadd(P.counters + 1, 1ull);
                    return pt_finish(L, P, zero);
                }
                push_level(P, slot, L);
                L.h = vis;
                L.depth++;
                return pt_advance(L, PS_ENTER, zero, P, slot);
            }
            return pt_advance(L, PS_DIRE, zero, P, slot);  // no recursion: indirectEstimator stays 0
        }
        case PQ_DIRE: {  // path.h:134-151
            if (hit && shape_id(vis.shape) == L.e_shape) {
                const f3 Li = emission_of(sc, vis.mat);
                const BsdfRecord& b = bsdf_of(sc, L.h.mat);
                const float a2s = L.e_cos * rcp_cr(L.e_d2);
                const float bsdfPdf = bsdf_pdf(b, L.e_wil, L.h.wo);
                const float w = balance_heuristic(static_cast<float>(S.emitter_samples),
                                                  (L.e_apdf * L.e_pdf) * rcp_cr(a2s),
                                                  static_cast<float>(S.bsdf_samples), bsdfPdf);
                f3 c = (Li * w) * bsdf_eval(b, L.e_wil, L.h.wo);
                c = ((c * rcp_cr(L.e_apdf)) * rcp_cr(L.e_pdf)) * a2s;
                L.eest = L.eest + c;
            }
            return pt_advance(L, PS_DIRE, zero, P, slot);
        }
        case PQ_DIRB: {  // path.h:162-184
            if (hit) {
                const f3 Li = emission_of(sc, vis.mat);
                const int eid = shape_emitter_of(sc, shape_id(vis.shape));
                if (!is_zero(Li) && eid >= 0) {
                    const EmitterRecord& e = emitter_of(sc, eid);
                    const float emitterPdf = 1.f / static_cast<float>(sc.nemit);
                    const float emitterAreaPdf = rcp_cr(e.area);
                    const f3 dd = L.h.p - vis.p;  // glm::distance2(visibilityInteraction.p, hit.p)
                    const float d2 = dot(dd, dd);
                    const f3 e1 = xyz(gld4(sc.tri + 3 * static_cast<size_t>(res) + 1));
                    const f3 e2 = xyz(gld4(sc.tri + 3 * static_cast<size_t>(res) + 2));
                    const f3 ng = normalize(cross(e1, e2));  // frameNg.n (accel.h:162)
                    const float cosOut = dot(-L.wiw, ng);
                    if (cosOut > 0.f) {
                        const float a2s = cosOut * rcp_cr(d2);
                        const float w = balance_heuristic(static_cast<float>(S.bsdf_samples), L.b_pdf,
                                                          static_cast<float>(S.emitter_samples),
                                                          (emitterPdf * emitterAreaPdf) * rcp_cr(a2s));
                        L.best = L.best + ((Li * w) * L.b_f) * rcp_cr(L.b_pdf);
                    }
                }
            }
            return pt_advance(L, PS_DIRB, zero, P, slot);
        }
        case PQ_IMP: {  // path.h:45-59
            if (!hit) return pt_advance(L, PS_IMP_RETURN, zero, P, slot);
            const f3 le = emission_of(sc, vis.mat);
            if (is_zero(le)) {
                if (L.depth + 1 >= S.max_levels) {
                    gadd(P.counters + 1, 1ull);
                    return pt_finish(L, P, zero);
                }
                push_level(P, slot, L);
                L.h = vis;
                L.depth++;
                return pt_advance(L, PS_IMP_LEVEL, zero, P, slot);
            }
            const f3 Li = dot(vis.n, -L.wiw) > 0.f ? le : zero;
            return pt_advance(L, PS_IMP_RETURN, (Li * L.f) * rcp_cr(L.pdf), P, slot);
        }
        case PQ_DI_E: {
            const int st = S.direct;
            const BsdfRecord& b = bsdf_of(sc, L.h.mat);
            if (st == DI_COSINE) {  // direct.h:221-227
                if (hit)
                    L.ind = L.ind + (emission_of(sc, vis.mat) * bsdf_eval(b, L.e_wil, L.h.wo)) *
                                        rcp_cr(cosine_hemisphere_pdf(L.e_wil));
                return pt_advance(L, PS_DI_EMIT, zero, P, slot);
            }
            const EmitterRecord& e = emitter_of(sc, L.e_id);
            if (st == DI_AREA) {  // direct.h:180-187: unoccluded up to the sampled point
                if (!hit) {
                    f3 c = ld3(e.radiance) * bsdf_eval(b, L.e_wil, L.h.wo);
                    c = ((c * rcp_cr(L.e_apdf)) * rcp_cr(L.e_pdf)) * L.e_cos;
                    L.ind = L.ind + c;
                }
                return pt_advance(L, PS_DI_EMIT, zero, P, slot);
            }
            // solid angle / MIS: the emitter's shape hit first, or nothing hit and the ray meets the sphere
            const bool lit = hit ? shape_id(vis.shape) == e.shape : ray_sphere_hit(L.ray, ld3(e.center), e.radius);
            if (lit) {
                if (st == DI_SOLID_ANGLE) {  // direct.h:283-306
                    const f3 c = (ld3(e.radiance) * bsdf_eval(b, L.e_wil, L.h.wo)) * rcp_cr(L.e_apdf);
                    L.ind = L.ind + c * rcp_cr(L.e_pdf);
                } else {  // direct.h:350-370
                    const float bsdfPdf = bsdf_pdf(b, L.e_wil, L.h.wo);
                    const float w = balance_heuristic(static_cast<float>(S.emitter_samples), L.e_apdf * L.e_pdf,
                                                      static_cast<float>(S.bsdf_samples), bsdfPdf);
                    const f3 c = ((ld3(e.radiance) * bsdf_eval(b, L.e_wil, L.h.wo)) * w) * rcp_cr(L.e_apdf);
                    L.eest = L.eest + c * rcp_cr(L.e_pdf);
                }
            }
            return pt_advance(L, PS_DI_EMIT, zero, P, slot);
        }
        case PQ_DI_B: {
            if (hit) {
                const f3 Le = emission_of(sc, vis.mat);
                if (S.direct == DI_BSDF) {  // direct.h:253-256: Le * brdfCosTheta * (1.0 / pdf)
                    L.ind = L.ind + (Le * L.b_f) * rcp_cr(L.b_pdf);
                } else if (!is_zero(Le)) {  // direct.h:390-414
                    const int eid = shape_emitter_of(sc, shape_id(vis.shape));
                    if (eid >= 0) {
                        const EmitterRecord& e = emitter_of(sc, eid);
                        const f3 dd = L.h.p - ld3(e.center);
                        const float sin2 = e.radius * e.radius / dot(dd, dd);
                        const float cosMax = sqrt_cr(glibc_fmaxf(0.f, 1.f - sin2));
                        float esap = kInvTwoPi * rcp_cr(1.f - cosMax);
                        esap = esap * (1.f / static_cast<float>(sc.nemit));
                        const float w = balance_heuristic(static_cast<float>(S.bsdf_samples), L.b_pdf,
                                                          static_cast<float>(S.emitter_samples), esap);
                        L.best = L.best + ((Le * L.b_f) * w) * rcp_cr(L.b_pdf);
                    }
                }
            }
            return pt_advance(L, PS_DI_BSDF, zero, P, slot);
        }
        default: return;
    }
}

#if !BDPT_SAMPLER_STATE
// SLACK: the overlapped walk's interior boxes with the ambiguity slack
// (DevScene::node_slack, per render on the host; bdpt_frame_kernel's parameter)
template <bool COUNT, bool OVERLAP, bool SLACK = true>
__global__ __launch_bounds__(256, PT_WAVES_PER_EU) void pt_frame_kernel(const PtParams* __restrict__ pp) {
    const PtParams& P = *pp;
    __shared__ uint2 stack_mem[kLdsStack * 256];
#if PT_ROOT_LDS
    __shared__ RootLds root_lds;  // the walk's first two node tests at query issue (bdpt_device.hpp)
    const bool root_in_lds = OVERLAP && root_lds_usable(P.sc);
    if (OVERLAP) root_lds_fill(root_lds, P.sc);
#endif
    scene_tables_to_lds(P.sc);
    const uint32_t slot = blockIdx.x * 256 + threadIdx.x;
    const Stack stk{stack_mem + threadIdx.x, 256, kLdsStack, P.gstack, P.nslots, slot};
    const int lane = threadIdx.x & 63;
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    cnt.m[0] = cnt.m[1] = cnt.m[2] = 0;
    cnt.q[0] = cnt.q[1] = cnt.q[2] = cnt.q[3] = 0;
    PtLane L;
    L.busy = false;
    L.q = PQ_NONE;
    L.rng.ring = P.ring + static_cast<size_t>(slot) * 624;  // slot-major (DevScene::mt_ring)
    L.rng.stride = 1;
    const uint64_t total = P.fr.total_samples;
    bool exhausted = false;
    const TravScene tsc = trav_scene(P.sc);
    bool tracing = false, has_res = false;
    TravState ts{};
    RayInv ri{};
    int res = -1;
    float rt = 0.f, ru = 0.f, rv = 0.f;
    for (;;) {
        if (!exhausted) {  // refill idle lanes: one atomic per wave
            const uint64_t idle = __ballot(!L.busy);
            if (idle) {
                const int n = popc64(idle);
                const int leader = __ffsll(static_cast<unsigned long long>(idle)) - 1;
                unsigned long long base = 0;
                if (lane == leader) base = gadd(P.work, static_cast<unsigned long long>(n));
                base = __shfl(base, leader);
                if (!L.busy) {
                    const uint64_t s = base + popc64(idle & ((1ull << lane) - 1ull));
                    if (s < total) {
                        L.rng.seed = sample_seed(s, P.fr, L.pixel);
                        mt_seed(L.rng.m, L.rng.seed);
                        const f3 d = camera_dir(P.fr, L.pixel, L.rng.m);  // draws 0, 1 (< 227)
                        L.ray = Ray{mk(P.fr.cam_o[0], P.fr.cam_o[1], P.fr.cam_o[2]), d, 1.f, 1000.f};
                        L.q = PQ_PRIMARY;
                        L.busy = true;
                    }
                }
                if (base + n >= total) exhausted = true;
            }
        }
        if (__ballot(L.busy) == 0) {
            if (exhausted) break;
            continue;
        }
        if constexpr (OVERLAP) {
        // The BDPT megakernel's overlapped schedule: a lane keeps walking its
        // query across iterations; lanes with a finished query wait until
        // PT_SHADE_READY of the wave have one, then advance together.
        if (L.busy && !tracing && !has_res) {
            if (COUNT) cnt.c[0]++;
            // no near cull for a query leaving the vertex nearly parallel to its triangle (cull_near_for)
            ri = ray_inv(L.ray, (L.q != PQ_PRIMARY && graze_exempt(L.ray.d, L.h.n, L.h.shape)) ? kNoCullNear : kCullNear);
            if (L.ray.min_t > L.ray.max_t) {  // the reference culls the root (bvh.h:277, :287)
                res = -1, rt = L.ray.max_t, ru = rv = 0.f;
                has_res = true;
            } else if (!ri.fast || far_origin(P.sc, L.ray.o)) {  // the reference's tree, unculled
                const TravResult q = traverse_binary<COUNT, Stack>(P.sc, L.ray, false, false, stk);
                if (COUNT) cnt.c[2] += q.nodes, cnt.c[3] += q.tris, cnt.c[15] += q.exact;
                res = q.best, rt = q.t, ru = q.u, rv = q.v;
                has_res = true;
            } else {
                ts = trav_begin(tsc, L.ray);
                tracing = true;
#if PT_ROOT_LDS
                if (root_in_lds && !walk_begin_lds<COUNT, SLACK>(root_lds, L.ray, ri, false, ts, stk, cnt)) {
                    res = -1, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;  // no child hit: a miss
                    tracing = false;
                    has_res = true;
                }
#endif
            }
        }
        for (;;) {
            const uint64_t tr = __ballot(tracing);
            if (!tr) break;
            if (popc64(__ballot(has_res)) >= PT_SHADE_READY) break;
            const bool at_leaf = (ts.link & kLeafBit) != 0;
            const uint64_t lv = __ballot(tracing && at_leaf);
            const bool do_leaf = popc64(lv) * 4 >= popc64(tr & ~lv) * PT_TRAV_SPLIT;
            bool fin = tracing && at_leaf == do_leaf && trav_step<COUNT, SLACK>(tsc, L.ray, ri, false, ts, stk, cnt);
            // PT_WALK_UNROLL more node steps for lanes now at an interior node (bdpt_frame_kernel's BDPT_UNROLL_ANY)
#pragma unroll
            for (int k = 0; k < PT_WALK_UNROLL; k++)
                if (tracing && !fin && !(ts.link & kLeafBit)) fin = trav_step<COUNT, SLACK>(tsc, L.ray, ri, false, ts, stk, cnt);
            if (fin) {
                res = ts.best, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                tracing = false;
                has_res = true;
            }
        }
        if (has_res) {
            has_res = false;
            pt_resolve<COUNT>(L, res, rt, ru, rv, P, slot, cnt);
            if (COUNT && !L.busy) cnt.c[7] += L.rng.m.n;
        }
        } else if (L.busy) {
            if (COUNT) cnt.c[0]++;
            float t = 0.f, u = 0.f, v = 0.f;
            const int res = traverse<false, COUNT>(P.sc, L.ray, false, stk, t, u, v, cnt);
            pt_resolve<COUNT>(L, res, t, u, v, P, slot, cnt);
            if (COUNT && !L.busy) cnt.c[7] += L.rng.m.n;
        }
    }
    if (COUNT) flush_counts(cnt, P.counters);
}

#endif  // !BDPT_SAMPLER_STATE

#if BDPT_SAMPLER_STATE
// One PathTracerIntegrator / DirectIntegrator::render(ray, sampler) call on one
// lane (path.h:235-245, direct.h:449-462), single-sample build (sample_state.hip):
// the sampler is the caller's std::mt19937 state (P.sc.mt_ring, mt_state_u32).
// out = Li.xyz, draws taken.
__global__ __launch_bounds__(64) void pt_sample_kernel(const PtParams* __restrict__ pp, Ray ray,
                                                       float* __restrict__ out) {
    const PtParams& P = *pp;
    __shared__ uint2 stack_mem[kLdsStack * 64];
    scene_tables_to_lds(P.sc);
    if (threadIdx.x != 0) return;
    const Stack stk{stack_mem, 64, kLdsStack, P.gstack, 1, 0};
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    cnt.m[0] = cnt.m[1] = cnt.m[2] = 0;
    cnt.q[0] = cnt.q[1] = cnt.q[2] = cnt.q[3] = 0;
    // Value-initialised: with a partly uninitialised lane record this one-lane
    // build returned garbage in Li.x (0x5a5a5a5a) although every field is
    // assigned before it is read on the reference's control flow (measured on
    // gfx950, ROCm 7.2; the frame kernel is unaffected).
    PtLane L{};
    L.rng.ring = P.ring;
    L.rng.stride = 1;
    L.rng.seed = 0;
    L.rng.m = LazyMT{0u, 0u, 0u, 0u};  // unused: next1 draws from the caller's state
    L.pixel = 0;
    L.ray = ray;
    L.q = PQ_PRIMARY;
    L.busy = true;
    while (L.busy) {
        float t = 0.f, u = 0.f, v = 0.f;
        const int res = traverse<false, false>(P.sc, L.ray, false, stk, t, u, v, cnt);
        pt_resolve<false>(L, res, t, u, v, P, 0, cnt);
    }
    out[3] = __uint_as_float(L.rng.m.n);
}

#endif  // BDPT_SAMPLER_STATE

}  // namespace dev

// ------------------------------------------------------------ host side
#if !BDPT_SAMPLER_STATE
size_t pt_params_bytes() { return sizeof(dev::PtParams); }
int pt_block() { return 256; }
int pt_lds_stack() { return dev::kLdsStack; }

int pt_blocks_per_cu(size_t dyn_lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::pt_frame_kernel<false, true>, 256, dyn_lds) != hipSuccess ||
        n <= 0)
        n = 1;
    return n;
}

hipError_t launch_pt(const dev::DevScene& sc, const dev::DevFrame& fr, const int32_t settings[8], float* fb,
                     float4* levels, uint32_t* ring, uint2* gstack, uint32_t nslots, unsigned long long* work,
                     unsigned long long* counters, int grid, hipStream_t stream, void* dparams) {
    dev::PtParams host{};
    host.sc = sc;
    host.fr = fr;
    host.ps.is_explicit = settings[0];
    host.ps.max_depth = settings[1];
    host.ps.rr_depth = settings[2];
    std::memcpy(&host.ps.rr_prob, &settings[3], 4);
    host.ps.emitter_samples = settings[4];
    host.ps.bsdf_samples = settings[5];
    host.ps.max_levels = settings[6];
    host.ps.direct = settings[7];
    host.fb = fb, host.levels = levels, host.ring = ring, host.gstack = gstack, host.nslots = nslots;
    host.work = work, host.counters = counters, host.li_out = nullptr;
    hipError_t e = hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    const dev::PtParams* kp = static_cast<const dev::PtParams*>(dparams);
    const size_t lds = 4 * static_cast<size_t>(sc.lds_words);
    const bool count = (fr.flags & 1u) != 0, overlap = host.ps.direct == 0, slack = sc.node_slack != 0;
    // (the non-overlapped walk, traverse(), reads node_slack itself)
    if (count && overlap && slack) hipLaunchKernelGGL((dev::pt_frame_kernel<true, true, true>), dim3(grid), dim3(256), lds, stream, kp);
    else if (count && overlap) hipLaunchKernelGGL((dev::pt_frame_kernel<true, true, false>), dim3(grid), dim3(256), lds, stream, kp);
    else if (count) hipLaunchKernelGGL((dev::pt_frame_kernel<true, false>), dim3(grid), dim3(256), lds, stream, kp);
    else if (overlap && slack) hipLaunchKernelGGL((dev::pt_frame_kernel<false, true, true>), dim3(grid), dim3(256), lds, stream, kp);
    else if (overlap) hipLaunchKernelGGL((dev::pt_frame_kernel<false, true, false>), dim3(grid), dim3(256), lds, stream, kp);
    else hipLaunchKernelGGL((dev::pt_frame_kernel<false, false>), dim3(grid), dim3(256), lds, stream, kp);
    return hipGetLastError();
}

#else
// sc.mt_ring = the device copy of the caller's std::mt19937 state (625 words).
hipError_t launch_pt_sample(const dev::DevScene& sc, const dev::DevFrame& fr, const int32_t settings[8],
                            float4* levels, uint32_t* ring, uint2* gstack, const dev::Ray& ray, float* out,
                            unsigned long long* counters, hipStream_t stream, void* dparams) {
    dev::PtParams host{};
    host.sc = sc;
    host.fr = fr;
    host.ps.is_explicit = settings[0];
    host.ps.max_depth = settings[1];
    host.ps.rr_depth = settings[2];
    std::memcpy(&host.ps.rr_prob, &settings[3], 4);
    host.ps.emitter_samples = settings[4];
    host.ps.bsdf_samples = settings[5];
    host.ps.max_levels = settings[6];
    host.ps.direct = settings[7];
    host.fb = nullptr, host.levels = levels, host.ring = ring, host.gstack = gstack, host.nslots = 1;
    host.work = nullptr, host.counters = counters, host.li_out = out;
    hipError_t e = hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    const dev::PtParams* kp = static_cast<const dev::PtParams*>(dparams);
    hipLaunchKernelGGL(dev::pt_sample_kernel, dim3(1), dim3(64), 4 * static_cast<size_t>(sc.lds_words), stream, kp,
                       ray, out);
    return hipGetLastError();
}
#endif  // BDPT_SAMPLER_STATE

}  // namespace bdpt
