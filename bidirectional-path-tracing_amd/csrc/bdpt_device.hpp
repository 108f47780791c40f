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
constexpr int kCounters = 12;

// ------------------------------------------------------------------ inputs
struct DevScene {
    const float4* __restrict__ tri;
    const float4* __restrict__ shade;
    const float4* __restrict__ nodes;
    const BsdfRecord* __restrict__ bsdf;
    const EmitterRecord* __restrict__ emit;
    const float4* __restrict__ emit_tri;
    const float* __restrict__ emit_cdf;
    const int32_t* __restrict__ shape_emitter;
    uint32_t root_link;
    int32_t nemit;
};

struct DevFrame {
    CameraConstants cam;
    float cam_o[3];
    int32_t W, H, spp, rr_depth, strategy;
    uint32_t seed_base;
    int32_t row_offset, row_stride, nrows;
    uint32_t flags;
    uint64_t total_samples;  // nrows * W * spp
};

struct Ray {
    f3 o, d;
    float min_t, max_t;
};

// Hit record = the parts of SurfaceInteraction (core.h:173-180) the path reads.
struct Hit {
    f3 p, wo, wi;
    f3 s, t, n;  // frameNs
    float dist;
    int mat, shape;
};

// ------------------------------------------------------------------ sampler
// std::mt19937(seed) + uniform_real_distribution<float> (math.h:63-76). A BDPT
// sample draws at most 10 + 8 (rrDepth - 1) numbers (< 227 for rrDepth <= 28),
// all from the first twist, so output n is computed lazily from the seeding
// recurrence: out_n = temper(x[n+397] ^ twist(x[n], x[n+1])). State: x[n],
// x[n+1], x[n+397] and n.
struct LazyMT {
    uint32_t a0, a1, b, n;
};

__device__ __forceinline__ uint32_t mt_init_step(uint32_t x, uint32_t i) { return 1812433253u * (x ^ (x >> 30)) + i; }

__device__ __forceinline__ void mt_seed(LazyMT& r, uint32_t seed) {
    uint32_t x = seed;
    r.a0 = x;
    x = mt_init_step(x, 1);
    r.a1 = x;
#pragma unroll 4
    for (uint32_t i = 2; i <= 397; i++) x = mt_init_step(x, i);
    r.b = x;
    r.n = 0;
}

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

// generate_canonical<float, 24> (libstdc++ 11 random.tcc:3348-3380).
__device__ __forceinline__ float next1(LazyMT& r) {
    float f = static_cast<float>(mt_next_u32(r)) / 4294967296.0f;
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
    return mk(sinTheta * glibc_cosf(phi), sinTheta * glibc_sinf(phi), cosTheta);
}
// squareToUniformDiskConcentric + squareToCosineHemisphere (math.h:153-192)
__device__ __forceinline__ f3 cosine_hemisphere(F2 u) {
    float rx = (2.f * u.x) - 1.f;
    float ry = (2.f * u.y) - 1.f;
    float dx = 0.f, dy = 0.f;
    if (!(rx == 0 && ry == 0)) {
        float radius, phi;
        if ((rx * rx) > (ry * ry)) {
            radius = rx;
            phi = (kPi * 0.25f) * (ry * (1.f / rx));
        } else {
            radius = ry;
            phi = (kPi * 0.5f) - ((kPi * 0.25f) * (rx * (1.f / ry)));
        }
        dx = radius * glibc_cosf(phi);
        dy = radius * glibc_sinf(phi);
    }
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
    return mk(sinTheta * glibc_cosf(phi), sinTheta * glibc_sinf(phi), cosTheta);
}
__device__ __forceinline__ float phong_lobe_pdf(f3 v, float ex) {
    return v.z >= 0.f ? (ex + 2) * kInvTwoPi * glibc_powf(v.z, ex) : 0.f;
}
// squareToUniformTriangle (math.h:229-234)
__device__ __forceinline__ F2 uniform_triangle(F2 s) {
    float u = sqrt_cr(1.f - s.x);
    return F2{1 - u, u * s.y};
}

// -------------------------------------------------------------------- frame
// Frame(n) with coordinateSystem (core.h:155-157, math.h:42-51): t = c, s = cross(c, n).
__device__ __forceinline__ void make_frame(f3 a, f3& s, f3& t) {
    if (fabsf(a.x) > fabsf(a.y)) {
        float inv = 1.f / sqrt_cr(a.x * a.x + a.z * a.z);
        t = mk(a.z * inv, 0.f, -a.x * inv);
    } else {
        float inv = 1.f / sqrt_cr(a.y * a.y + a.z * a.z);
        t = mk(0.f, a.z * inv, -a.y * inv);
    }
    s = cross(t, a);
}
__device__ __forceinline__ f3 to_local(f3 s, f3 t, f3 n, f3 v) { return mk(dot(v, s), dot(v, t), dot(v, n)); }
__device__ __forceinline__ f3 to_world(f3 s, f3 t, f3 n, f3 v) { return (s * v.x + t * v.y) + n * v.z; }
__device__ __forceinline__ f3 reflect_z(f3 d) { return mk(-d.x, -d.y, d.z); }

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

// Fast form of the same decision: t = (l - o) * RN(1/d) differs from the
// reference's RN((l - o) / d) by at most ~1.8e-7 |t| (three roundings). With
// per-axis intervals [lo_i, hi_i], the reference's test is "every cross pair
// lo_i <= hi_j (i != j) holds" (the swaps make lo_i <= hi_i). Each cross pair is
// decided with a slack of 1e-6 (|lo_i| + |hi_j|) — 5x the error bound — and any
// pair inside the slack, or any non-finite value, defers to slab() above, so
// the hit / miss outcome is always the reference's.
enum : int { kSlabMiss = 0, kSlabHit = 1, kSlabAmbiguous = 2 };
__device__ __forceinline__ int cross_le(float a, float b) {
    const float d = b - a, s = 1e-6f * (fabsf(a) + fabsf(b));
    return d > s ? kSlabHit : (d < -s ? kSlabMiss : kSlabAmbiguous);
}
__device__ __forceinline__ int slab_fast(float lx, float ly, float lz, float hx, float hy, float hz, f3 o, f3 inv,
                                         float& tn, float& tf) {
    const float x0 = (lx - o.x) * inv.x, x1 = (hx - o.x) * inv.x;
    const float y0 = (ly - o.y) * inv.y, y1 = (hy - o.y) * inv.y;
    const float z0 = (lz - o.z) * inv.z, z1 = (hz - o.z) * inv.z;
    const float nan_probe = ((x0 + x1) + (y0 + y1)) + (z0 + z1);  // NaN if any t is NaN (or +inf meets -inf)
    if (nan_probe != nan_probe) return kSlabAmbiguous;           // the reference's NaN rules live in slab()
    const float lox = fminf(x0, x1), hix = fmaxf(x0, x1);
    const float loy = fminf(y0, y1), hiy = fmaxf(y0, y1);
    const float loz = fminf(z0, z1), hiz = fmaxf(z0, z1);
    tn = fmaxf(fmaxf(lox, loy), loz);
    tf = fminf(fminf(hix, hiy), hiz);
    const int c1 = cross_le(loy, hix), c2 = cross_le(loz, hix), c3 = cross_le(lox, hiy);
    const int c4 = cross_le(lox, hiz), c5 = cross_le(loy, hiz), c6 = cross_le(loz, hiy);
    if (c1 == kSlabMiss || c2 == kSlabMiss || c3 == kSlabMiss || c4 == kSlabMiss || c5 == kSlabMiss ||
        c6 == kSlabMiss)
        return kSlabMiss;
    if ((c1 & c2 & c3 & c4 & c5 & c6) == kSlabHit) return kSlabHit;
    return kSlabAmbiguous;  // includes NaN / inf operands (every comparison false)
}

__device__ __forceinline__ bool box_test(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r,
                                         f3 inv, float& tn, float& tf) {
    const int f = slab_fast(lx, ly, lz, hx, hy, hz, r.o, inv, tn, tf);
    if (f != kSlabAmbiguous) return f == kSlabHit;
    return slab(lx, ly, lz, hx, hy, hz, r, tn, tf);
}

// rayTriangleIntersect (core.h:379-400) + accel.h:43's t > 1e-3.
__device__ __forceinline__ bool tri_test(const float4* __restrict__ tri, uint32_t i, const Ray& r, float& t, float& u,
                                         float& v) {
    const f3 v0 = xyz(tri[3 * i]), v1 = xyz(tri[3 * i + 1]), v2 = xyz(tri[3 * i + 2]);
    const f3 e1 = v1 - v0, e2 = v2 - v0;
    const f3 pvec = cross(r.d, e2);
    const float det = dot(e1, pvec);
    if (fabsf(det) < kEpsilon) return false;
    const float invDet = 1.f / det;
    const f3 tvec = r.o - v0;
    u = dot(tvec, pvec) * invDet;
    if (u < 0.f || u > 1.f) return false;
    const f3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * invDet;
    if (v < 0.f || u + v > 1.f) return false;
    t = dot(e2, qvec) * invDet;
    return t >= kTriMinT;
}

// Traversal stack: one column per thread in LDS (entry k of thread x at
// base[k * stride + x], conflict-free); entries are node links. 40 entries x
// 4 B x 1024 threads fill the 160 KiB of a CU at 16 waves.
struct Stack {
    uint32_t* base;
    int stride;
    __device__ __forceinline__ void put(int k, uint32_t link) { base[k * stride] = link; }
    __device__ __forceinline__ uint32_t get(int k) const { return base[k * stride]; }
};

// Conservative distance culling. The reference never culls by distance
// (bbhits stay 0, bvh.h:265-337): its result is the minimum-t triangle among
// ALL boxes the line crosses, first-found (= lowest leaf index) on ties. Boxes
// entered beyond best + margin, or exited before t = 5e-4, cannot hold a
// triangle that changes that result.
__device__ __forceinline__ float cull_far(float best) { return best + fabsf(best) * 1e-3f + 1e-4f; }
constexpr float kCullNear = 5e-4f;

struct Counts {
    uint32_t c[kCounters];
};

// SIMD-efficiency probe: true on the lowest active lane of the wave only.
__device__ __forceinline__ bool first_active_lane() {
    return (__lane_id()) == static_cast<unsigned>(__ffsll(static_cast<unsigned long long>(__ballot(1))) - 1);
}

// BVH::getIntersection (bvh.h:259-352) for both query kinds, in ONE inlined
// loop so the megakernel carries a single copy of the traversal:
//   closest (any == false): the minimum-t triangle, ties to the lowest leaf
//     index (= first found by the reference's left-first DFS); returns the leaf
//     index or -1 and the hit's t, u, v.
//   any (any == true): returns 1 if some triangle hits inside [min_t, max_t]
//     (the occlusion early-out at bvh.h:300-302), else -1.
template <bool FULL, bool COUNT>
__device__ __forceinline__ int traverse(const DevScene& sc, const Ray& r, bool any, Stack stk, float& bt, float& bu,
                                        float& bv, Counts& cnt) {
    float best_t = r.max_t, best_u = 0.f, best_v = 0.f;
    int best = -1;
    if (r.min_t > best_t) return -1;  // the root's entry mint is min_t (bvh.h:277, :287)
    uint32_t link = sc.root_link;
    int sp = 0;
    const f3 inv = mk(1.f / r.d.x, 1.f / r.d.y, 1.f / r.d.z);
    for (;;) {
        if (COUNT) {
            cnt.c[8]++;
            if (first_active_lane()) cnt.c[9]++;
        }
        if (link & kLeafBit) {
            const uint32_t start = (link >> 3) & 0x0fffffffu, count = link & 7u;
            bool done = false;
            for (uint32_t k = 0; k < count; k++) {
                const uint32_t i = start + k;
                float t, u, v;
                if (COUNT) cnt.c[3]++;
                if (tri_test(sc.tri, i, r, t, u, v)) {
                    if (any) {
                        if (t <= r.max_t && t >= r.min_t) {
                            best = 1;
                            done = true;
                            break;
                        }
                    } else if (t < best_t || (t == best_t && best >= 0 && static_cast<int>(i) < best)) {
                        best_t = t, best = static_cast<int>(i), best_u = u, best_v = v;
                    }
                }
            }
            if (done) break;
        } else {
            if (COUNT) cnt.c[2]++;
            const float4* nd = sc.nodes + 4 * static_cast<size_t>(link);
            const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2], q3 = nd[3];
            float tn0, tf0, tn1, tf1;
            bool h0 = box_test(q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, r, inv, tn0, tf0);
            bool h1 = box_test(q1.z, q1.w, q2.x, q2.y, q2.z, q2.w, r, inv, tn1, tf1);
            const uint32_t l0 = __float_as_uint(q3.x), l1 = __float_as_uint(q3.y);
            if (!FULL) {
                const float far = cull_far(any ? r.max_t : best_t);
                h0 = h0 && !(tn0 > far) && !(tf0 < kCullNear);
                h1 = h1 && !(tn1 > far) && !(tf1 < kCullNear);
            }
            if (h0 && h1) {
                const bool swap = !FULL && (tn1 < tn0);
                stk.put(sp++, swap ? l0 : l1);
                link = swap ? l1 : l0;
                continue;
            }
            if (h0) { link = l0; continue; }
            if (h1) { link = l1; continue; }
        }
        if (sp == 0) break;
        link = stk.get(--sp);
    }
    bt = best_t, bu = best_u, bv = best_v;
    return best;
}

// AcceleratorBVH::intersect's shading of a closest hit (accel.h:133-166).
__device__ __forceinline__ void shade_hit(const DevScene& sc, int i, float u, float v, float t, f3 dir, Hit& h) {
    const f3 v0 = xyz(sc.tri[3 * i]), v1 = xyz(sc.tri[3 * i + 1]), v2 = xyz(sc.tri[3 * i + 2]);
    const float4 s0 = sc.shade[3 * i], s1 = sc.shade[3 * i + 1], s2 = sc.shade[3 * i + 2];
    const float w = 1 - u - v;
    h.p = (v0 * w + v1 * u) + v2 * v;
    h.n = normalize((xyz(s0) * w + xyz(s1) * u) + xyz(s2) * v);
    make_frame(h.n, h.s, h.t);
    h.wo = to_local(h.s, h.t, h.n, -dir);
    h.wi = mk(0.f, 0.f, 0.f);
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

// MixtureBSDF::eval == PhongBSDF::eval (mixture.h:59-75, phong.h:56-71).
// With Ks == 0 the specular term is (0 * (n + 2)) * INV_TWOPI * powf(c, n) = +0
// (powf of c in [0, 1] is finite), and val + 0 == val: skipping it is exact.
__device__ __forceinline__ f3 glossy_eval(const BsdfRecord& b, f3 wi, f3 wo) {
    f3 val = mk(0.f, 0.f, 0.f);
    if (wi.z >= 0.f && wo.z >= 0.f) {
        val = val + ld3(b.kd) * kInvPi;
        if (b.ks[0] != 0.f || b.ks[1] != 0.f || b.ks[2] != 0.f) {
            const float ex = b.exponent;
            const float c = glibc_fminf(glibc_fmaxf(dot(wi, reflect_z(wo)), 0.f), 1.f);
            val = val + ((ld3(b.ks) * (ex + 2)) * kInvTwoPi) * glibc_powf(c, ex);
        }
        val = val * b.scale;
        val = val * wi.z;
    }
    return val;
}

__device__ BDPT_NOINLINE f3 bsdf_eval(const BsdfRecord& b, f3 wi, f3 wo) {
    if (b.kind == BSDF_DIFFUSE) {  // diffuse.h:35-43
        if (wi.z >= 0.f && wo.z >= 0.f) return (ld3(b.kd) * kInvPi) * wi.z;
        return mk(0.f, 0.f, 0.f);
    }
    if (b.kind == BSDF_MIXTURE || b.kind == BSDF_PHONG) return glossy_eval(b, wi, wo);
    return mk(0.f, 0.f, 0.f);  // delta lobes (perfectmirror.h:41-47, glass.h:55-59)
}

__device__ __forceinline__ float phong_part_pdf(const BsdfRecord& b, f3 wi, f3 wo) {
    f3 rs, rt;
    const f3 rn = reflect_z(wo);
    make_frame(rn, rs, rt);
    return phong_lobe_pdf(to_local(rs, rt, rn, wi), b.exponent);
}

// With specw == 0, pdfPhong * 0 = +0 (pdfPhong is finite and >= 0) and
// 0 + pdfDiffuse * (1 - 0) == pdfDiffuse: skipping the Phong lobe is exact.
__device__ BDPT_NOINLINE float bsdf_pdf(const BsdfRecord& b, f3 wi, f3 wo) {
    if (b.kind == BSDF_DIFFUSE) return cosine_hemisphere_pdf(wi);  // diffuse.h:45-50
    if (b.kind == BSDF_MIXTURE) {                                  // mixture.h:78-100
        const float pd = cosine_hemisphere_pdf(wi);
        if (b.specw == 0.f) return pd;
        const float pp = phong_part_pdf(b, wi, wo);
        return (pp * b.specw) + (pd * (1.f - b.specw));
    }
    if (b.kind == BSDF_PHONG) return phong_part_pdf(b, wi, wo);  // phong.h:73-83
    return 0.f;
}

// glass.h:40-53
__device__ __forceinline__ float fresnel_dielectric(float eta_i, float eta_t, float cos_i, float cos_t) {
    const float eta = eta_i / eta_t;
    const float sin2_t = eta * eta * (glibc_fmaxf(0.f, 1.f - cos_i * cos_i));
    if (sin2_t >= 1.f) return 1.f;
    const float rpar = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    const float rper = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (rpar * rpar + rper * rper) * 0.5f;
}

// BSDF::sample: sets wi, returns f*cos, writes the solid-angle pdf.
__device__ BDPT_NOINLINE f3 bsdf_sample(const BsdfRecord& b, f3 wo, F2 u, f3& wi, float& pdf) {
    switch (b.kind) {
        case BSDF_DIFFUSE:  // diffuse.h:52-61
            wi = cosine_hemisphere(u);
            pdf = cosine_hemisphere_pdf(wi);
            return bsdf_eval(b, wi, wo);
        case BSDF_MIRROR:  // perfectmirror.h:49-59
            pdf = 1.f;
            wi = reflect_z(wo);
            return mk(1.f, 1.f, 1.f);
        case BSDF_GLASS: {  // glass.h:67-108 (pdf 1, no eta^2 scaling)
            pdf = 1.f;
            const bool entering = wo.z > 0.f;
            float eta_i = 1.f, eta_t = b.ior;
            if (!entering) { float q = eta_i; eta_i = eta_t; eta_t = q; }
            const float eta = eta_i / eta_t;
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
        case BSDF_MIXTURE: {  // mixture.h:102-151
            f3 val;
            if (u.x < b.specw) {
                const F2 ns{u.x / b.specw, u.y};
                f3 rs, rt;
                const f3 rn = reflect_z(wo);
                make_frame(rn, rs, rt);
                wi = to_world(rs, rt, rn, phong_lobe(ns, b.exponent));
                val = bsdf_eval(b, wi, wo);
            } else {
                const F2 ns{(u.x - b.specw) / (1.f - b.specw), u.y};
                wi = cosine_hemisphere(ns);
                val = bsdf_eval(b, wi, wo);
            }
            pdf = bsdf_pdf(b, wi, wo);
            return val;
        }
        case BSDF_PHONG: {  // phong.h:85-100
            f3 rs, rt;
            const f3 rn = reflect_z(wo);
            make_frame(rn, rs, rt);
            const f3 ls = phong_lobe(u, b.exponent);
            pdf = phong_lobe_pdf(ls, b.exponent);
            wi = to_world(rs, rt, rn, ls);
            return bsdf_eval(b, wi, wo);
        }
        default:  // null BSDF (illum 5): the reference dereferences nullptr
            pdf = 0.f;
            wi = mk(0.f, 0.f, 0.f);
            return mk(0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ bool is_delta(const BsdfRecord& b) { return (b.type & kTypeDelta) != 0; }

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

// selectEmitter + sampleEmitterPosition (integrator.cpp:46-51, :73-100): 4 draws.
__device__ __forceinline__ const EmitterRecord& sample_emitter(const DevScene& sc, LazyMT& rng, float& emitter_pdf,
                                                              f3& n, f3& pos, float& pos_pdf) {
    const float u0 = next1(rng);
    uint32_t id = static_cast<uint32_t>(u0 * static_cast<float>(sc.nemit));
    id = id < static_cast<uint32_t>(sc.nemit - 1) ? id : static_cast<uint32_t>(sc.nemit - 1);
    emitter_pdf = 1.f / static_cast<float>(sc.nemit);
    const EmitterRecord& e = sc.emit[id];
    const int f = cdf_sample(sc.emit_cdf + e.cdf_offset, e.nfaces + 1, next1(rng));
    const F2 uv = uniform_triangle(next2(rng));
    const float4* q = sc.emit_tri + 5 * static_cast<size_t>(e.face_offset + f);
    const float4 a = q[0], b = q[1], c = q[2], d = q[3], g = q[4];
    const f3 v0 = mk(a.x, a.y, a.z), v1 = mk(a.w, b.x, b.y), v2 = mk(b.z, b.w, c.x);
    const f3 n0 = mk(c.y, c.z, c.w), n1 = mk(d.x, d.y, d.z), n2 = mk(d.w, g.x, g.y);
    const float w = 1 - uv.x - uv.y;
    pos = (v0 * w + v1 * uv.x) + v2 * uv.y;
    n = normalize((n0 * w + n1 * uv.x) + n2 * uv.y);
    pos_pdf = 1.f / e.area;
    return e;
}

}  // namespace dev
}  // namespace bdpt
