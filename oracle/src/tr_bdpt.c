/* TEST INFRASTRUCTURE (oracle): the BDPT hot path restated in C, line by line
 * in the reference's arithmetic order (single precision, no FMA contraction).
 *
 * Reference: JackMinn/Bidirectional-Path-Tracing
 *   sampler          src/core/math.h:63-76 (+ libstdc++ 11 generate_canonical,
 *                    bits/random.tcc:3348-3380; std::mt19937)
 *   warps            src/core/math.h:136-234
 *   frame            src/core/core.h:152-167, math.h:42-51
 *   triangle test    src/core/core.h:379-400, accel.h:27-52
 *   BVH traversal    externals/bvh.h:33-69 (slab test), :259-352 (DFS)
 *   closest hit      src/core/accel.h:125-172
 *   BSDFs            src/bsdfs/diffuse.h:35-61, perfectmirror.h:33-59,
 *                    glass.h:40-108, mixture.h:59-151, phong.h:56-100
 *   emitter helpers  src/core/integrator.cpp:46-100, math.h:107-111
 *   BDPT             src/integrators/bdpt.h:46-505 (NO_RR 1 or 0, BDPT / LT / PT strategy)
 *   driver           src/core/renderer.cpp:143-210 with per-(pixel, sample)
 *                    seeds (SURVEY.md §8(c) parity convention)
 */
#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "tr_internal.h"

/* ---------------------------------------------------------------- counters */
/* [0] closest rays, [1] shadow rays, [2] interior visits, [3] triangle tests,
 * [4] light vertices stored, [5] light-vertex reads (connectVertices calls),
 * [6] splats, [7] RNG draws, [8] eye walks whose first intersect re-traces the
 * primary ray (bdpt.h:70 repeats :225; the GPU reuses that hit instead). */
static __thread int64_t g_ctr[TRO_NUM_COUNTERS];
void tro_counters(int64_t out[TRO_NUM_COUNTERS], int reset) {
    for (int i = 0; i < TRO_NUM_COUNTERS; i++) out[i] = g_ctr[i];
    if (reset) memset(g_ctr, 0, sizeof g_ctr);
}

/* ----------------------------------------------------------------- sampler */
typedef struct {
    uint32_t mt[624];
    int idx;
} tr_sampler;

static void mt_seed(tr_sampler* s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < 624; i++) s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->idx = 624;
}

static uint32_t mt_next(tr_sampler* s) {
    if (s->idx >= 624) {
        for (int k = 0; k < 624; k++) {
            uint32_t y = (s->mt[k] & 0x80000000u) | (s->mt[(k + 1) % 624] & 0x7fffffffu);
            s->mt[k] = s->mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        s->idx = 0;
    }
    uint32_t y = s->mt[s->idx++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* Sampler::next (math.h:70): uniform_real_distribution<float>(0,1) over
 * generate_canonical<float,24>: float(u) / 2^32, clamped below 1. */
static float s_next(tr_sampler* s) {
    g_ctr[7]++;
    float r = (float)mt_next(s) / 4294967296.0f;
    if (r >= 1.0f) r = 0x1.fffffep-1f;
    return r * (1.0f - 0.0f) + 0.0f;
}
typedef struct { float x, y; } v2;
static v2 s_next2d(tr_sampler* s) {
    v2 r;
    r.x = s_next(s);
    r.y = s_next(s);
    return r;
}

uint32_t tro_mt19937_nth(uint32_t seed, int n) {
    tr_sampler s;
    mt_seed(&s, seed);
    uint32_t u = 0;
    for (int i = 0; i <= n; i++) u = mt_next(&s);
    return u;
}
float tro_sampler_nth(uint32_t seed, int n) {
    tr_sampler s;
    mt_seed(&s, seed);
    float u = 0;
    for (int i = 0; i <= n; i++) u = s_next(&s);
    return u;
}
float tro_sinf(float x) { return tr_sinf(x); }
float tro_cosf(float x) { return tr_cosf(x); }
float tro_powf(float x, float y) { return tr_powf(x, y); }

/* ------------------------------------------------------------------- warps */
/* math.h:136-144 */
static v3 sq_uniform_hemisphere(v2 u) {
    float phi = u.x * TR_PI * 2.0f;
    float cosTheta = u.y;
    float sinTheta = sqrtf(tr_fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    return V3(sinTheta * tr_cosf(phi), sinTheta * tr_sinf(phi), cosTheta);
}
/* math.h:153-180 */
static v2 sq_disk_concentric(v2 u) {
    float phi, radius;
    float rX = (2.f * u.x) - 1.f;
    float rY = (2.f * u.y) - 1.f;
    v2 r = {0.f, 0.f};
    if (rX == 0 && rY == 0) return r;
    if ((rX * rX) > (rY * rY)) {
        radius = rX;
        phi = (TR_PI * 0.25f) * (rY * (1.f / rX));
    } else {
        radius = rY;
        phi = (TR_PI * 0.5f) - ((TR_PI * 0.25f) * (rX * (1.f / rY)));
    }
    r.x = radius * tr_cosf(phi);
    r.y = radius * tr_sinf(phi);
    return r;
}
/* math.h:182-192 */
static v3 sq_cosine_hemisphere(v2 u) {
    v2 d = sq_disk_concentric(u);
    float z = 1.0f - (d.x * d.x + d.y * d.y);
    z = tr_fmaxf(z, 0.f);
    z = sqrtf(z);
    return V3(d.x, d.y, z);
}
/* math.h:194-208 */
static float cosine_pdf(v3 v) { return v.z >= 0.f ? v.z * TR_INV_PI : 0.f; }
/* math.h:210-219 */
static v3 sq_phong_lobe(v2 u, float exponent) {
    float cosTheta = tr_powf(u.x, 1.f / (exponent + 2));
    float sinTheta = sqrtf(tr_fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    float phi = u.y * 2.f * TR_PI;
    return V3(sinTheta * tr_cosf(phi), sinTheta * tr_sinf(phi), cosTheta);
}
/* math.h:221-227 */
static float phong_lobe_pdf(v3 v, float exponent) {
    return v.z >= 0.f ? (exponent + 2) * TR_INV_TWOPI * tr_powf(v.z, exponent) : 0.f;
}
/* math.h:229-234 */
static v2 sq_uniform_triangle(v2 s) {
    float u = sqrtf(1.f - s.x);
    v2 r = {1 - u, u * s.y};
    return r;
}

/* ------------------------------------------------------------------- frame */
typedef struct { v3 s, t, n; } frame_t;
/* Frame(n) + coordinateSystem (core.h:155-157, math.h:42-51) */
static frame_t make_frame(v3 a) {
    frame_t f;
    f.n = a;
    v3 c;
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.f / sqrtf(a.x * a.x + a.z * a.z);
        c = V3(a.z * invLen, 0.f, -a.x * invLen);
    } else {
        float invLen = 1.f / sqrtf(a.y * a.y + a.z * a.z);
        c = V3(0.f, a.z * invLen, -a.y * invLen);
    }
    f.t = c;
    f.s = vcross(c, a);
    return f;
}
static v3 to_local(const frame_t* f, v3 v) { return V3(vdot(v, f->s), vdot(v, f->t), vdot(v, f->n)); }
/* s * v.x + t * v.y + n * v.z (core.h:161-163) */
static v3 to_world(const frame_t* f, v3 v) { return vadd(vadd(vscale(f->s, v.x), vscale(f->t, v.y)), vscale(f->n, v.z)); }

/* ---------------------------------------------------------------- geometry */
typedef struct {
    v3 o, d;
    float min_t, max_t;
} ray_t;

typedef struct {
    v3 p, wo, wi;
    float t;
    int shape, prim, mat;
    frame_t fs; /* frameNs */
    v3 ng;      /* frameNg.n (read by the path tracer's BSDF-sampled direct light, path.h:177) */
} hit_t;

/* A value-initialised SurfaceInteraction (all zero): what the reference's
 * intersect leaves behind on a miss (matID 0, shapeID 0). */
static hit_t zero_hit(void) {
    hit_t h;
    memset(&h, 0, sizeof h);
    return h;
}

static inline v3 tri_v(const tro_scene* s, int t, int c) {
    const float* p = s->tv + 9 * (size_t)t + 3 * c;
    return V3(p[0], p[1], p[2]);
}
static inline v3 tri_n(const tro_scene* s, int t, int c) {
    const float* p = s->tn + 9 * (size_t)t + 3 * c;
    return V3(p[0], p[1], p[2]);
}

/* rayTriangleIntersect (core.h:379-400) + the t > 1e-3 filter of accel.h:43
 * (a double comparison in the reference). */
static int tri_intersect(const tro_scene* s, int tri, const ray_t* r, float* tt, float* uu, float* vv) {
    g_ctr[3]++;
    v3 v0 = tri_v(s, tri, 0), v1 = tri_v(s, tri, 1), v2 = tri_v(s, tri, 2);
    v3 v0v1 = vsub(v1, v0);
    v3 v0v2 = vsub(v2, v0);
    v3 pvec = vcross(r->d, v0v2);
    float det = vdot(v0v1, pvec);
    if (fabsf(det) < TR_EPSILON) return 0;
    float invDet = 1 / det;
    v3 tvec = vsub(r->o, v0);
    float u = vdot(tvec, pvec) * invDet;
    if (u < 0 || u > 1) return 0;
    v3 qvec = vcross(tvec, v0v1);
    float v = vdot(r->d, qvec) * invDet;
    if (v < 0 || u + v > 1) return 0;
    float t = vdot(v0v2, qvec) * invDet;
    if (!((double)t > 1e-3)) return 0;
    *tt = t;
    *uu = u;
    *vv = v;
    return 1;
}

/* BBox::intersect (bvh.h:33-69): a line/slab test; tnear/tfar never written. */
static int bbox_hit(const tro_node* n, const ray_t* r) {
    float tmin = (n->bmin[0] - r->o.x) / r->d.x;
    float tmax = (n->bmax[0] - r->o.x) / r->d.x;
    if (tmin > tmax) { float x = tmin; tmin = tmax; tmax = x; }
    float tymin = (n->bmin[1] - r->o.y) / r->d.y;
    float tymax = (n->bmax[1] - r->o.y) / r->d.y;
    if (tymin > tymax) { float x = tymin; tymin = tymax; tymax = x; }
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (n->bmin[2] - r->o.z) / r->d.z;
    float tzmax = (n->bmax[2] - r->o.z) / r->d.z;
    if (tzmin > tzmax) { float x = tzmin; tzmin = tzmax; tzmax = x; }
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    return 1;
}

/* BVH::getIntersection (bvh.h:259-352). Returns the hit triangle id or -1.
 * With occlusion set it returns 1 on the first hit inside [min_t, max_t]. */
static int bvh_query(const tro_scene* s, const ray_t* r, int occlusion, float* bt, float* bu, float* bv) {
    float best_t = r->max_t;
    int best = -1;
    float best_u = 0, best_v = 0;
    struct { int i; float mint; } todo[64];
    int sp = 0;
    todo[0].i = 0;
    todo[0].mint = r->min_t;
    while (sp >= 0) {
        int ni = todo[sp].i;
        float near = todo[sp].mint;
        sp--;
        const tro_node* node = &s->nodes[ni];
        if (near > best_t) continue;
        if (node->right_offset == 0) {
            for (uint32_t o = 0; o < node->nprims; ++o) {
                int tri = s->order[node->start + o];
                float t, u, v;
                if (tri_intersect(s, tri, r, &t, &u, &v)) {
                    if (occlusion && t <= r->max_t && t >= r->min_t) return 1;
                    if (t < best_t) {
                        best_t = t;
                        best = tri;
                        best_u = u;
                        best_v = v;
                    }
                }
            }
        } else {
            g_ctr[2]++;
            int c0 = bbox_hit(&s->nodes[ni + 1], r);
            int c1 = bbox_hit(&s->nodes[ni + node->right_offset], r);
            /* bbhits stay 0: the left child is always "closer" (bvh.h:317-338) */
            if (c0 && c1) {
                todo[++sp].i = ni + (int)node->right_offset;
                todo[sp].mint = 0.f;
                todo[++sp].i = ni + 1;
                todo[sp].mint = 0.f;
            } else if (c0) {
                todo[++sp].i = ni + 1;
                todo[sp].mint = 0.f;
            } else if (c1) {
                todo[++sp].i = ni + (int)node->right_offset;
                todo[sp].mint = 0.f;
            }
        }
    }
    if (occlusion) return 0;
    *bt = best_t;
    *bu = best_u;
    *bv = best_v;
    return best;
}

/* AcceleratorBVH::intersect (accel.h:125-172). */
static int scene_intersect(const tro_scene* s, const ray_t* r, hit_t* h) {
    g_ctr[0]++;
    float t, u, v;
    int tri = bvh_query(s, r, 0, &t, &u, &v);
    if (tri < 0) return 0;
    if (!(t <= r->max_t && t >= r->min_t)) return 0;
    v3 v0 = tri_v(s, tri, 0), v1 = tri_v(s, tri, 1), v2 = tri_v(s, tri, 2);
    v3 n0 = tri_n(s, tri, 0), n1 = tri_n(s, tri, 1), n2 = tri_n(s, tri, 2);
    float w = 1 - u - v;
    h->t = t;
    h->shape = s->tshape[tri];
    h->prim = s->tprim[tri];
    h->p = vadd(vadd(vscale(v0, w), vscale(v1, u)), vscale(v2, v));
    h->ng = vnormalize(vcross(vsub(v1, v0), vsub(v2, v0)));
    h->fs = make_frame(vnormalize(vadd(vadd(vscale(n0, w), vscale(n1, u)), vscale(n2, v))));
    h->wo = to_local(&h->fs, vneg(r->d));
    h->wi = V3(0, 0, 0);
    h->mat = s->tmat[tri];
    return 1;
}

/* BDPTIntegrator::visibilityQuery (bdpt.h:498-505): true = occluded. */
static int visibility_query(const tro_scene* s, v3 start, v3 end) {
    g_ctr[1]++;
    v3 dir = vsub(end, start);
    float dist = sqrtf(vdot(dir, dir));
    dir = vdivs(dir, dist);
    ray_t r = {start, dir, TR_EPSILON, dist - 0.00001f};
    float t, u, v;
    return bvh_query(s, &r, 1, &t, &u, &v);
}

/* ------------------------------------------------------------------- BSDFs */
static inline v3 reflect_local(v3 d) { return V3(-d.x, -d.y, d.z); }

/* MixtureBSDF::eval / PhongBSDF::eval (mixture.h:59-75, phong.h:56-71) */
static v3 glossy_eval(const tro_bsdf* b, const hit_t* h) {
    v3 val = V3(0.f, 0.f, 0.f);
    if (h->wi.z >= 0.f && h->wo.z >= 0.f) {
        val = vadd(val, vscale(b->kd, TR_INV_PI));
        float ex = b->exponent;
        float cosTheta = tr_fminf(tr_fmaxf(vdot(h->wi, reflect_local(h->wo)), 0.f), 1.f);
        val = vadd(val, vscale(vscale(vscale(b->ks, ex + 2), TR_INV_TWOPI), tr_powf(cosTheta, ex)));
        val = vscale(val, b->scale);
        val = vscale(val, h->wi.z);
    }
    return val;
}
static float phong_pdf_only(const tro_bsdf* b, const hit_t* h) {
    frame_t rs = make_frame(reflect_local(h->wo));
    v3 bs = to_local(&rs, h->wi);
    return phong_lobe_pdf(bs, b->exponent);
}

static v3 bsdf_eval(const tro_bsdf* b, const hit_t* h) {
    switch (b->kind) {
        case TRB_DIFFUSE:
            /* diffuse.h:35-43 */
            if (h->wi.z >= 0.f && h->wo.z >= 0.f) return vscale(vscale(b->kd, TR_INV_PI), h->wi.z);
            return V3(0, 0, 0);
        case TRB_MIXTURE:
        case TRB_PHONG:
            return glossy_eval(b, h);
        default: /* mirror.h:41-47, glass.h:55-59: delta lobes evaluate to 0 */
            return V3(0, 0, 0);
    }
}

static float bsdf_pdf(const tro_bsdf* b, const hit_t* h) {
    switch (b->kind) {
        case TRB_DIFFUSE:
            return cosine_pdf(h->wi);
        case TRB_MIXTURE: {
            /* mixture.h:78-100 */
            float pdfPhong = phong_pdf_only(b, h);
            float pdfDiffuse = cosine_pdf(h->wi);
            return (pdfPhong * b->specw) + (pdfDiffuse * (1.f - b->specw));
        }
        case TRB_PHONG:
            return phong_pdf_only(b, h);
        default:
            return 0.f;
    }
}

/* FresnelDielectric (glass.h:40-53) */
static float fresnel_dielectric(float eta_i, float eta_t, float cos_i, float cos_t) {
    float eta = eta_i / eta_t;
    float sin2_t = eta * eta * (tr_fmaxf(0.f, 1.f - cos_i * cos_i));
    if (sin2_t >= 1.f) return 1.f;
    float rParallel = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    float rPerpendicular = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (rParallel * rParallel + rPerpendicular * rPerpendicular) * 0.5f;
}

/* BSDF::sample: sets h->wi, writes *pdf, returns f*cos. */
static v3 bsdf_sample(const tro_bsdf* b, hit_t* h, v2 u, float* pdf) {
    switch (b->kind) {
        case TRB_DIFFUSE: {
            /* diffuse.h:52-61 */
            h->wi = sq_cosine_hemisphere(u);
            *pdf = cosine_pdf(h->wi);
            return bsdf_eval(b, h);
        }
        case TRB_MIRROR:
            /* perfectmirror.h:49-59 */
            *pdf = 1.f;
            h->wi = reflect_local(h->wo);
            return V3(1.f, 1.f, 1.f);
        case TRB_GLASS: {
            /* glass.h:67-108 */
            *pdf = 1;
            int entering = h->wo.z > 0.f;
            float eta_i = 1.f, eta_t = b->ior;
            if (!entering) { float x = eta_i; eta_i = eta_t; eta_t = x; }
            float eta = eta_i / eta_t;
            float sin2_i = tr_fmaxf(0.f, 1.f - h->wo.z * h->wo.z);
            float sin2_t = eta * eta * sin2_i;
            float cos_t = sqrtf(tr_fmaxf(0.f, 1.f - sin2_t));
            cos_t = entering ? -cos_t : cos_t;
            float fresnel = fresnel_dielectric(eta_i, eta_t, fabsf(h->wo.z), fabsf(cos_t));
            if (u.x < fresnel) {
                h->wi = reflect_local(h->wo);
                return V3(1.f, 1.f, 1.f);
            }
            h->wi = V3(eta * -h->wo.x, eta * -h->wo.y, cos_t);
            return b->tf;
        }
        case TRB_MIXTURE: {
            /* mixture.h:102-151 */
            v3 val;
            if (u.x < b->specw) {
                v2 ns = {u.x / b->specw, u.y};
                frame_t rs = make_frame(reflect_local(h->wo));
                v3 bs = sq_phong_lobe(ns, b->exponent);
                h->wi = to_world(&rs, bs);
                val = bsdf_eval(b, h);
            } else {
                v2 ns = {(u.x - b->specw) / (1.f - b->specw), u.y};
                h->wi = sq_cosine_hemisphere(ns);
                val = bsdf_eval(b, h);
            }
            *pdf = bsdf_pdf(b, h);
            return val;
        }
        case TRB_PHONG: {
            /* phong.h:85-100 */
            frame_t rs = make_frame(reflect_local(h->wo));
            v3 bs = sq_phong_lobe(u, b->exponent);
            *pdf = phong_lobe_pdf(bs, b->exponent);
            h->wi = to_world(&rs, bs);
            return bsdf_eval(b, h);
        }
        default:
            abort(); /* null BSDF: the reference dereferences nullptr here */
    }
}

static inline const tro_bsdf* bsdf_of(const tro_scene* s, const hit_t* h) { return &s->bsdf[h->mat]; }
static inline int is_delta(const tro_bsdf* b) { return (b->type & TRT_DELTA) != 0; }

/* ------------------------------------------------------------ emitter help */
/* Integrator::selectEmitter (integrator.cpp:46-51) */
static int select_emitter(const tro_scene* s, float u, float* pdf) {
    size_t id = (size_t)(u * (float)s->nemit);
    if (id > (size_t)(s->nemit - 1)) id = (size_t)(s->nemit - 1);
    *pdf = 1.f / (float)s->nemit;
    return (int)id;
}
/* Distribution1D::sample (math.h:107-111): upper_bound then clamp. */
static int dist_sample(const tro_emitter* e, float u) {
    int lo = 0, hi = e->ncdf;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (u < e->cdf[mid]) hi = mid; else lo = mid + 1;
    }
    int i = lo - 1;
    if (i < 0) i = 0;
    if (i > e->ncdf - 2) i = e->ncdf - 2;
    return i;
}
/* Integrator::sampleEmitterPosition (integrator.cpp:73-100) */
static void sample_emitter_position(const tro_scene* s, tr_sampler* smp, const tro_emitter* e, v3* n, v3* pos,
                                    float* pdf) {
    int prim = dist_sample(e, s_next(smp));
    v2 uv = sq_uniform_triangle(s_next2d(smp));
    int tri = s->shape_first[e->shape] + prim;
    v3 v0 = tri_v(s, tri, 0), v1 = tri_v(s, tri, 1), v2 = tri_v(s, tri, 2);
    float w = 1 - uv.x - uv.y;
    *pos = vadd(vadd(vscale(v0, w), vscale(v1, uv.x)), vscale(v2, uv.y));
    v3 n0 = tri_n(s, tri, 0), n1 = tri_n(s, tri, 1), n2 = tri_n(s, tri, 2);
    *n = vnormalize(vadd(vadd(vscale(n0, w), vscale(n1, uv.x)), vscale(n2, uv.y)));
    *pdf = 1.f / e->area;
}

/* ---------------------------------------------------------------- BDPT */
typedef struct {
    hit_t hit;
    v3 throughput;
    float vcm, vc, rr;
} pvert_t; /* PathVertex (bdpt.h:24-35) */

typedef struct {
    const tro_scene* s;
    int W, H, spp, rr_depth;
    v3 cam_o, cam_fwd;
    m4 w2c, c2clip, ndc2screen;
    float vnear;
    float* fb;
    int strategy; /* tro_params.strategy */
    const tro_params* p;
} ctx_t;

/* splatToImagePlane (bdpt.h:485-496). static_cast<int> of a NaN or an
 * out-of-range value is INT_MIN on x86 (cvttss2si). */
static int f2i_x86(float f) {
    if (!(f > -2147483648.f && f < 2147483648.f)) return (int)0x80000000u;
    return (int)f;
}
static void splat_to_image_plane(const ctx_t* c, v3 p, int* x, int* y) {
    v4 uv = {p.x, p.y, p.z, 1.f};
    uv = tr_m4v4(&c->w2c, uv);
    uv = tr_m4v4(&c->c2clip, uv);
    float w = uv.w;
    uv.x = uv.x / w; uv.y = uv.y / w; uv.z = uv.z / w; uv.w = uv.w / w;
    uv = tr_m4v4(&c->ndc2screen, uv);
    *x = f2i_x86(uv.x);
    *y = f2i_x86(uv.y);
}

/* connectToCamera (bdpt.h:295-371) */
static void connect_to_camera(const ctx_t* c, const pvert_t* lv) {
    const tro_scene* s = c->s;
    v3 cameraForward = c->cam_fwd;
    v3 e2l = vsub(lv->hit.p, c->cam_o);
    float invDistanceSquared = 1.f / vdot(e2l, e2l);
    e2l = vscale(e2l, sqrtf(invDistanceSquared));
    int xPixel, yPixel;
    splat_to_image_plane(c, lv->hit.p, &xPixel, &yPixel);
    if (xPixel < 0 || yPixel < 0 || xPixel >= c->W || yPixel >= c->H) return;
    float cosCamera = vdot(cameraForward, e2l);
    if (cosCamera <= 0.f) return;
    hit_t be = lv->hit;
    be.wi = to_local(&be.fs, vneg(e2l));
    const tro_bsdf* b = bsdf_of(s, &be);
    v3 bsdfCosTheta = bsdf_eval(b, &be);
    if (veq0(bsdfCosTheta) || be.wi.z <= 0.f) return;
    if (visibility_query(s, c->cam_o, lv->hit.p)) return;
    float vnear = c->vnear;
    float imagePointToCameraDist = vnear / cosCamera;
    float imageAreaToCameraSolidAngle = imagePointToCameraDist * imagePointToCameraDist / cosCamera;
    float cameraSolidAngleToSurfaceArea = be.wi.z * invDistanceSquared;
    float imageAreaToSurfaceArea = imageAreaToCameraSolidAngle * cameraSolidAngleToSurfaceArea;
    float surfaceAreaToImageArea = 1.f / imageAreaToSurfaceArea;
    int nlight = c->W * c->H;
    v3 radiance = vmul(lv->throughput, vscale(bsdfCosTheta, 1.f / be.wi.z));
    radiance = vscale(radiance, 1.f / surfaceAreaToImageArea);
    radiance = vscale(radiance, 1.f / (float)nlight);
    radiance = vscale(radiance, 1.f / (float)c->spp);
    float reversePdf_a = 1.f * imageAreaToSurfaceArea;
    hit_t rh = be;
    rh.wi = be.wo;
    rh.wo = be.wi;
    float prevRev = bsdf_pdf(b, &rh) * lv->rr;
    float lightWeight = (reversePdf_a / (float)nlight) * (lv->vcm + prevRev * lv->vc);
    float eyeWeight = 0.f;
    float misWeight = 1.f / (lightWeight + 1.f + eyeWeight);
    if (c->strategy == 0) radiance = vscale(radiance, misWeight); /* bdpt.h:355-357 */
    int pixel = yPixel * c->W + xPixel;
    g_ctr[6]++;
    c->fb[3 * (size_t)pixel + 0] += radiance.x;
    c->fb[3 * (size_t)pixel + 1] += radiance.y;
    c->fb[3 * (size_t)pixel + 2] += radiance.z;
}

/* connectToLight (bdpt.h:374-430) */
static v3 connect_to_light(const ctx_t* c, const pvert_t* ev, tr_sampler* smp) {
    const tro_scene* s = c->s;
    float emitterPdf;
    int id = select_emitter(s, s_next(smp), &emitterPdf);
    const tro_emitter* e = &s->emit[id];
    v3 en, ep;
    float emitterPositionPdf;
    sample_emitter_position(s, smp, e, &en, &ep, &emitterPositionPdf);
    v3 dir = vsub(ev->hit.p, ep);
    float d2 = vdot(dir, dir);
    dir = vscale(dir, 1.f / sqrtf(d2));
    hit_t be = ev->hit;
    be.wi = to_local(&be.fs, vneg(dir));
    float cosAtLight = vdot(en, dir);
    float cosAtEye = be.wi.z;
    if (cosAtLight <= 0.f || cosAtEye <= 0.f) return V3(0, 0, 0);
    float pdf_a = emitterPdf * emitterPositionPdf;
    float pdf_w = pdf_a * d2 / cosAtLight;
    float emitterDirectionPdf_w = TR_INV_TWOPI;
    const tro_bsdf* b = bsdf_of(s, &be);
    v3 Li = vmul(vmul(vscale(bsdf_eval(b, &be), 1.f / pdf_w), ev->throughput), e->radiance);
    if (veq0(Li)) return V3(0, 0, 0);
    if (visibility_query(s, ev->hit.p, ep)) return V3(0, 0, 0);
    float lightPathReversePdf_w = bsdf_pdf(b, &be) * ev->rr;
    float lightWeight = lightPathReversePdf_w / pdf_w;
    hit_t rh = be;
    rh.wi = be.wo;
    rh.wo = be.wi;
    float eyePrevRev = bsdf_pdf(b, &rh) * ev->rr;
    float eyeCurRev_a = cosAtEye * (1.f / d2) * emitterDirectionPdf_w;
    float eyeWeight = eyeCurRev_a * (ev->vcm + eyePrevRev * ev->vc);
    float misWeight = 1.f / (lightWeight + 1.f + eyeWeight);
    return c->strategy == 0 ? vscale(Li, misWeight) : Li; /* bdpt.h:426-428 */
}

/* connectVertices (bdpt.h:434-483) */
static v3 connect_vertices(const ctx_t* c, const pvert_t* lv, const pvert_t* ev) {
    const tro_scene* s = c->s;
    g_ctr[5]++;
    v3 dir = vsub(ev->hit.p, lv->hit.p);
    float invD2 = 1.f / vdot(dir, dir);
    dir = vscale(dir, sqrtf(invD2));
    hit_t lh = lv->hit, eh = ev->hit;
    lh.wi = to_local(&lh.fs, dir);
    eh.wi = to_local(&eh.fs, vneg(dir));
    float cosL = lh.wi.z, cosE = eh.wi.z;
    if (cosL <= 0.f || cosE <= 0.f) return V3(0, 0, 0);
    if (visibility_query(s, ev->hit.p, lv->hit.p)) return V3(0, 0, 0);
    const tro_bsdf* bl = bsdf_of(s, &lh);
    const tro_bsdf* be = bsdf_of(s, &eh);
    v3 Li = vmul(bsdf_eval(bl, &lh), bsdf_eval(be, &eh));
    Li = vmul(Li, vscale(vmul(lv->throughput, ev->throughput), invD2));
    float eyePathReversePdf_w = bsdf_pdf(bl, &lh) * lv->rr;
    { v3 x = lh.wi; lh.wi = lh.wo; lh.wo = x; }
    float lightPathPrevRev = bsdf_pdf(bl, &lh) * lv->rr;
    float lightPathReversePdf_w = bsdf_pdf(be, &eh) * ev->rr;
    eh.wo = eh.wi;
    eh.wi = ev->hit.wo;
    float eyePathPrevRev = bsdf_pdf(be, &eh) * ev->rr;
    float lightPathReversePdf_a = lightPathReversePdf_w * cosL * invD2;
    float eyePathReversePdf_a = eyePathReversePdf_w * cosE * invD2;
    float lightWeight = lightPathReversePdf_a * (lv->vcm + lightPathPrevRev * lv->vc);
    float eyeWeight = eyePathReversePdf_a * (ev->vcm + eyePathPrevRev * ev->vc);
    float misWeight = 1.f / (lightWeight + 1.f + eyeWeight);
    return vscale(Li, misWeight);
}

/* ContinuePathRandomWalk (bdpt.h:243-291) */
static int continue_walk(const ctx_t* c, hit_t* h, tr_sampler* smp, float rrp, pvert_t* pv, v3* tp, int* depth,
                         float* vc, float* vcm, ray_t* ray) {
    const tro_bsdf* b = bsdf_of(c->s, h);
    int delta = is_delta(b);
    float pdf;
    v3 f = bsdf_sample(b, h, s_next2d(smp), &pdf);
    pdf *= rrp;
    pv->hit.wi = h->wi;
    float absCosOut = fabsf(h->wi.z);
    if (veq0(f)) return 0;
    *tp = vmul(*tp, vscale(f, 1.f / pdf));
    (*depth)++;
    hit_t rh = *h;
    rh.wi = h->wo;
    rh.wo = h->wi;
    float prevRev = delta ? pdf : bsdf_pdf(b, &rh) * rrp;
    if (delta) {
        *vc = (absCosOut / pdf) * (prevRev * *vc);
        *vcm = 0.f;
    } else {
        *vc = (absCosOut / pdf) * (*vcm + prevRev * *vc);
        *vcm = 1.f / pdf;
    }
    ray->o = h->p;
    ray->d = to_world(&h->fs, h->wi);
    ray->min_t = TR_EPSILON;
    ray->max_t = FLT_MAX;
    return 1;
}

#define MAX_LIGHT_VERTS 1024 /* light vertices kept per sample (the reference's vector is unbounded;
                                 a longer subpath is counted in g_ctr[7]'s overflow twin below) */
static __thread int64_t g_rr_overflow, g_max_light_depth, g_max_eye_depth, g_max_nl;

/* rrProbability (bdpt.h:127-132 / :199-204): 1 before rrDepth, then 0.5 when the
 * throughput's luminance (getLuminance, math.h:56-58: a glm dot) is below 0.01;
 * always 1 under NO_RR = 1 (bdpt.h:18, the reference as shipped). */
static float rr_probability(const ctx_t* c, int depth, v3 tp) {
    if (!c->p->russian_roulette) return 1.f;
    if ((depth + 1) < c->rr_depth) return 1.f;
    return vdot(tp, V3(0.212671f, 0.715160f, 0.072169f)) < 0.01f ? 0.5f : 1.f;
}

/* The loop test `depth < m_rrDepth || (sampler.next() < rrProbability && !NO_RR)`
 * (bdpt.h:68, :188): past rrDepth one draw, then a continuation only with RR on. */
static int walk_continues(const ctx_t* c, int depth, float rrp, tr_sampler* smp) {
    if (depth < c->rr_depth) return 1;
    const float u = s_next(smp);
    return c->p->russian_roulette && u < rrp;
}

int64_t tro_rr_overflow(int reset) {
    int64_t v = g_rr_overflow;
    if (reset) g_rr_overflow = 0;
    return v;
}

void tro_walk_stats(int64_t out[3], int reset) {
    out[0] = g_max_light_depth, out[1] = g_max_eye_depth, out[2] = g_max_nl;
    if (reset) g_max_light_depth = g_max_eye_depth = g_max_nl = 0;
}

/* lightSubpathWalk (bdpt.h:158-217) */
static int light_walk(const ctx_t* c, tr_sampler* smp, pvert_t* lverts) {
    const tro_scene* s = c->s;
    int nl = 0;
    float emitterPdf, emitterAreaPdf, emitterEmissionPdf;
    v3 normalOut, positionOut;
    int id = select_emitter(s, s_next(smp), &emitterPdf);
    const tro_emitter* e = &s->emit[id];
    sample_emitter_position(s, smp, e, &normalOut, &positionOut, &emitterAreaPdf);
    v3 edir = sq_uniform_hemisphere(s_next2d(smp));
    emitterEmissionPdf = TR_INV_TWOPI * emitterAreaPdf;
    emitterAreaPdf *= emitterPdf;
    emitterEmissionPdf *= emitterPdf;
    frame_t lf = make_frame(normalOut);
    ray_t wi = {positionOut, to_world(&lf, edir), TR_EPSILON, FLT_MAX};
    v3 throughput = vscale(vscale(e->radiance, edir.z), 1.f / emitterEmissionPdf);
    float vc = edir.z * (1.f / emitterEmissionPdf);
    float vcm = emitterAreaPdf / emitterEmissionPdf;
    if (edir.z <= 0.f) return 0;
    int depth = 1;
    float rrp = 1.f;
    while (walk_continues(c, depth, rrp, smp)) {
        hit_t hit;
        if (!scene_intersect(s, &wi, &hit)) break;
        float distSquared = hit.t * hit.t;
        float absCosIn = fabsf(hit.wo.z);
        vcm *= (distSquared / absCosIn);
        vc *= (1.f / absCosIn);
        rrp = rr_probability(c, depth, throughput);
        int delta = is_delta(bsdf_of(s, &hit));
        pvert_t lv = {hit, throughput, vcm, vc, rrp};
        if (!delta) connect_to_camera(c, &lv);
        if (!continue_walk(c, &hit, smp, rrp, &lv, &throughput, &depth, &vc, &vcm, &wi)) break;
        if (!delta) {
            if (nl < MAX_LIGHT_VERTS) {
                lverts[nl++] = lv;
                g_ctr[4]++;
            } else {
                g_rr_overflow++;
            }
        }
    }
    if (depth > g_max_light_depth) g_max_light_depth = depth;
    if (nl > g_max_nl) g_max_nl = nl;
    return nl;
}

/* eyeSubpathWalk (bdpt.h:46-155) */
static v3 eye_walk(const ctx_t* c, const pvert_t* lverts, int nl, ray_t ray, tr_sampler* smp) {
    const tro_scene* s = c->s;
    v3 Li = V3(0, 0, 0);
    int pureSpecular = 1;
    float cosCamera = vdot(c->cam_fwd, ray.d);
    float imagePointToCameraDist = c->vnear / cosCamera;
    float imageAreaToCameraSolidAngle = imagePointToCameraDist * imagePointToCameraDist / cosCamera;
    float t1Pdf = 1.f * imageAreaToCameraSolidAngle;
    ray_t wi = ray;
    v3 throughput = V3(1.f, 1.f, 1.f);
    float vc = 0.f;
    float vcm = (float)(c->W * c->H) * (1.f / t1Pdf);
    int depth = 1;
    float rrp = 1.f;
    while (walk_continues(c, depth, rrp, smp)) {
        hit_t hit;
        if (depth == 1 && 1 < c->rr_depth) g_ctr[8]++;
        if (!scene_intersect(s, &wi, &hit)) break;
        float distSquared = hit.t * hit.t;
        float absCosIn = fabsf(hit.wo.z);
        vcm *= (distSquared / absCosIn);
        vc *= (1.f / absCosIn);
        const tro_material* m = &s->mats[hit.mat];
        v3 emission = V3(m->Ke[0], m->Ke[1], m->Ke[2]);
        if (!veq0(emission)) {
            int eid = s->shape_emitter[hit.shape];
            if (eid < 0) abort(); /* reference asserts (integrator.cpp:56) */
            const tro_emitter* e = &s->emit[eid];
            float emitterPdf = 1.f / (float)s->nemit;
            if (depth > 1) {
                v3 contribution = vmul(e->radiance, throughput);
                float pA = 1.f / (e->area * emitterPdf);
                float dirPdf = TR_INV_TWOPI;
                float cameraWeight = pA * vcm + (pA * dirPdf) * vc;
                float misWeight = 1.f / (1.f + cameraWeight);
                if (c->strategy == 2) { /* PATH_TRACING: pure specular paths only (bdpt.h:110-113) */
                    if (pureSpecular) Li = vadd(Li, contribution);
                } else {
                    if (c->strategy == 0 && !pureSpecular) contribution = vscale(contribution, misWeight); /* :95-99 */
                    Li = vadd(Li, contribution);
                }
            } else if (depth == 1) {
                Li = vadd(Li, emission);
            }
            break;
        }
        rrp = rr_probability(c, depth, throughput);
        pvert_t ev = {hit, throughput, vcm, vc, rrp};
        if (!is_delta(bsdf_of(s, &hit))) {
            pureSpecular = 0;
            Li = vadd(Li, connect_to_light(c, &ev, smp));
            if (c->strategy == 0) /* bdpt.h:145-149 */
                for (int i = 0; i < nl; i++) Li = vadd(Li, connect_vertices(c, &lverts[i], &ev));
        }
        if (!continue_walk(c, &hit, smp, rrp, &ev, &throughput, &depth, &vc, &vcm, &wi)) break;
    }
    if (depth > g_max_eye_depth) g_max_eye_depth = depth;
    return Li;
}

/* BDPTIntegrator::render (bdpt.h:219-241) */
static v3 bdpt_render(const ctx_t* c, ray_t ray, tr_sampler* smp) {
    hit_t hit;
    if (!scene_intersect(c->s, &ray, &hit)) return V3(0, 0, 0);
    pvert_t lverts[MAX_LIGHT_VERTS];
    if (c->strategy == 1) { /* LIGHT_TRACING (bdpt.h:229-231): light walk, then Le at the primary hit */
        (void)light_walk(c, smp, lverts);
        const tro_material* m = &c->s->mats[hit.mat];
        return V3(m->Ke[0], m->Ke[1], m->Ke[2]);
    }
    if (c->strategy == 2) return eye_walk(c, lverts, 0, ray, smp); /* PATH_TRACING (:232-233) */
    int nl = light_walk(c, smp, lverts);
    return eye_walk(c, lverts, nl, ray, smp);
}

/* ------------------------------------------------------------ path tracer */
/* PathTracerIntegrator (src/integrators/path.h), the other offline integrator
 * the reference's shipped cbox_bdpt_path.toml selects. */
static v3 emission_of(const tro_scene* s, const hit_t* h) { /* getEmission (integrator.cpp:41-44) */
    const tro_material* m = &s->mats[h->mat];
    return V3(m->Ke[0], m->Ke[1], m->Ke[2]);
}
/* balanceHeuristic (path.h:31-34) */
static float balance_heuristic(float nf, float fPdf, float ng, float gPdf) {
    float f = nf * fPdf, g = ng * gPdf;
    return f / (f + g);
}

/* recursiveImplicit (path.h:36-64). "(1.0 / pdf)" is a double divided and
 * narrowed to float by glm's scalar operator: the correctly rounded 1.f / pdf. */
static v3 pt_implicit(const ctx_t* c, tr_sampler* smp, hit_t* hit, int depth) {
    const tro_scene* s = c->s;
    if (!(depth < c->p->pt_max_depth)) return V3(0, 0, 0);
    v2 u = s_next2d(smp);
    float pdf;
    v3 f = bsdf_sample(bsdf_of(s, hit), hit, u, &pdf);
    hit_t vis = zero_hit();
    v3 wiW = to_world(&hit->fs, hit->wi);
    ray_t r = {hit->p, wiW, TR_EPSILON, INFINITY};
    if (!scene_intersect(s, &r, &vis)) return V3(0, 0, 0);
    float inv = (float)(1.0 / (double)pdf);
    if (veq0(emission_of(s, &vis))) return vscale(vmul(pt_implicit(c, smp, &vis, depth + 1), f), inv);
    v3 Li = emission_of(s, &vis);
    Li = vdot(vis.fs.n, vneg(wiW)) > 0.f ? Li : V3(0, 0, 0);
    return vscale(vmul(Li, f), inv);
}

/* recursiveExplicit (path.h:66-202) */
static v3 pt_explicit(const ctx_t* c, tr_sampler* smp, hit_t* hit, int depth) {
    const tro_scene* s = c->s;
    const tro_params* P = c->p;
    v3 Lr = V3(0, 0, 0);
    float rrSample = s_next(smp);
    v3 indirect = V3(0, 0, 0), direct = V3(0, 0, 0);
    if (depth < P->pt_max_depth || (P->pt_max_depth == -1 && (depth < P->pt_rr_depth || rrSample < P->pt_rr_prob))) {
        { /* indirect estimator (:77-112): re-sample while an emitter is hit, 0.95 each retry */
            unsigned nSamples = 0;
            const float indRRProb = 0.95f;
            float cumRRProb = 1.f;
            hit_t vis;
            int intersects = 0;
            float pdf = 0.f;
            v3 f = V3(0, 0, 0);
            do {
                vis = zero_hit();
                v2 u = s_next2d(smp);
                f = bsdf_sample(bsdf_of(s, hit), hit, u, &pdf);
                v3 wiW = to_world(&hit->fs, hit->wi);
                ray_t r = {hit->p, wiW, TR_EPSILON, INFINITY};
                intersects = scene_intersect(s, &r, &vis);
                nSamples++;
            } while (!veq0(emission_of(s, &vis)) && s_next(smp) < indRRProb);
            cumRRProb = nSamples > 1 ? indRRProb : 1.f;
            if (intersects && !veq0(f) && veq0(emission_of(s, &vis))) {
                v3 Li = pt_explicit(c, smp, &vis, depth + 1);
                indirect = vscale(vscale(vscale(vmul(Li, f), 1.f / pdf), 1.f / (float)nSamples), 1.f / cumRRProb);
            }
        }
        { /* direct estimator (:115-190) */
            v3 emitterEst = V3(0, 0, 0), bsdfEst = V3(0, 0, 0);
            for (int i = 0; i < P->pt_emitter_samples; ++i) {
                float emitterPdf, emitterAreaPdf;
                v3 nOut, pOut;
                int id = select_emitter(s, s_next(smp), &emitterPdf);
                const tro_emitter* e = &s->emit[id];
                sample_emitter_position(s, smp, e, &nOut, &pOut, &emitterAreaPdf);
                v3 wiW = vnormalize(vsub(pOut, hit->p));
                v3 wiLocal = to_local(&hit->fs, wiW);
                v3 dd = vsub(hit->p, pOut); /* glm::distance2(positionOut, hit.p) */
                float lightDistanceSquared = vdot(dd, dd);
                float cosOutgoing = vdot(vneg(wiW), nOut);
                if (cosOutgoing > 0.f && wiLocal.z > 0.f) {
                    ray_t r = {hit->p, wiW, TR_EPSILON, INFINITY};
                    hit_t vis = zero_hit();
                    if (scene_intersect(s, &r, &vis) && vis.shape == e->shape) {
                        v3 Li = emission_of(s, &vis);
                        hit->wi = wiLocal;
                        float a2s = cosOutgoing * (1.f / lightDistanceSquared);
                        const tro_bsdf* b = bsdf_of(s, hit);
                        float bsdfPdf = bsdf_pdf(b, hit);
                        float w = balance_heuristic((float)P->pt_emitter_samples, emitterAreaPdf * emitterPdf * (1.f / a2s),
                                                    (float)P->pt_bsdf_samples, bsdfPdf);
                        v3 t = vmul(vscale(Li, w), bsdf_eval(b, hit));
                        t = vscale(vscale(vscale(t, 1.f / emitterAreaPdf), 1.f / emitterPdf), a2s);
                        emitterEst = vadd(emitterEst, t);
                    }
                }
            }
            emitterEst = P->pt_emitter_samples == 0 ? V3(0, 0, 0) : vdivs(emitterEst, (float)P->pt_emitter_samples);
            for (int i = 0; i < P->pt_bsdf_samples; ++i) {
                v2 u = s_next2d(smp);
                float bsdfPdf;
                v3 f = bsdf_sample(bsdf_of(s, hit), hit, u, &bsdfPdf);
                if (veq0(f)) continue;
                hit_t vis = zero_hit();
                v3 wiW = to_world(&hit->fs, hit->wi);
                ray_t r = {hit->p, wiW, TR_EPSILON, INFINITY};
                if (!scene_intersect(s, &r, &vis)) continue;
                v3 Li = emission_of(s, &vis);
                if (veq0(Li)) continue;
                int eid = s->shape_emitter[vis.shape]; /* getEmitterIDByShapeID (integrator.cpp:53-58) */
                if (eid < 0) abort();                  /* the reference asserts */
                const tro_emitter* e = &s->emit[eid];
                float emitterPdf = 1.f / (float)s->nemit;
                float emitterAreaPdf = 1.f / e->area;
                v3 dd = vsub(hit->p, vis.p); /* glm::distance2(vis.p, hit.p) */
                float lightDistanceSquared = vdot(dd, dd);
                float cosOutgoing = vdot(vneg(wiW), vis.ng);
                if (cosOutgoing > 0.f) {
                    float a2s = cosOutgoing * (1.f / lightDistanceSquared);
                    float w = balance_heuristic((float)P->pt_bsdf_samples, bsdfPdf, (float)P->pt_emitter_samples,
                                                emitterPdf * emitterAreaPdf * (1.f / a2s));
                    bsdfEst = vadd(bsdfEst, vscale(vmul(vscale(Li, w), f), 1.f / bsdfPdf));
                }
            }
            bsdfEst = P->pt_bsdf_samples == 0 ? V3(0, 0, 0) : vdivs(bsdfEst, (float)P->pt_bsdf_samples);
            direct = vadd(emitterEst, bsdfEst);
        }
        Lr = vadd(direct, indirect);
        if (P->pt_max_depth == -1 && !(depth < P->pt_rr_depth) && (rrSample < P->pt_rr_prob))
            Lr = vscale(Lr, 1.f / P->pt_rr_prob);
    }
    return Lr;
}

/* PathTracerIntegrator::render (path.h:235-245) with renderExplicit / renderImplicit (:204-233) */
static v3 pt_render(const ctx_t* c, ray_t ray, tr_sampler* smp) {
    hit_t hit = zero_hit();
    if (!scene_intersect(c->s, &ray, &hit)) return V3(0, 0, 0);
    if (!veq0(emission_of(c->s, &hit))) return emission_of(c->s, &hit);
    return c->p->pt_explicit ? pt_explicit(c, smp, &hit, 0) : pt_implicit(c, smp, &hit, 0);
}

/* -------------------------------------------------------- direct lighting */
/* DirectIntegrator (src/integrators/direct.h): emitters are treated as spheres
 * of their shape's corner mean and AABB half-width (renderer.cpp:349-358). */

/* quadratic + raySphereIntersect (direct.h:17-67), in double as there. */
static int ray_sphere_hit(const ray_t* r, v3 center, float radius) {
    v3 no = vsub(r->o, center);
    double cc = (double)(vdot(no, no) - (radius * radius));
    double b = (double)vdot(no, r->d) * 2.0;
    double a = (double)vdot(r->d, r->d);
    double disc = b * b - 4 * a * cc;
    double t0, t1;
    if (disc > 0) {
        double sq = sqrt(disc);
        double inv2a = 1 / (2 * a);
        t0 = (-b + sq) * inv2a;
        t1 = (-b - sq) * inv2a;
    } else if (disc == 0) {
        t0 = (-b + sqrt(disc)) / (2 * a);
        t1 = t0;
    } else {
        return 0;
    }
    const double lo = r->min_t, hi = r->max_t;
    return (t0 > lo && t0 < hi) || (t1 > lo && t1 < hi);
}
/* Warp::squareToUniformSphere (math.h:119-127) */
static v3 sq_uniform_sphere(v2 u) {
    float phi = u.x * TR_PI * 2.0f;
    float cosTheta = 1.f - (2.f * u.y);
    float sinTheta = tr_sqrtf(fmaxf(1.f - cosTheta * cosTheta, 0.f));
    return V3(sinTheta * tr_cosf(phi), sinTheta * tr_sinf(phi), cosTheta);
}
/* sampleSphereBySolidAngle (direct.h:109-141) */
static v3 sample_sphere_solid_angle(v2 u, v3 p, v3 center, float radius, float* pdf) {
    v3 cdir = vnormalize(vsub(center, p));
    frame_t f = make_frame(cdir);
    v3 dd = vsub(center, p);
    float sin2 = radius * radius / vdot(dd, dd);
    float cosMax = tr_sqrtf(fmaxf(0.f, 1.f - sin2));
    float cosTheta = (1.f - u.x) + (u.x * cosMax);
    float phi = u.y * TR_PI * 2.0f;
    float sinTheta = tr_sqrtf(fmaxf(1.f - (cosTheta * cosTheta), 0.f));
    v3 d = V3(sinTheta * tr_cosf(phi), sinTheta * tr_sinf(phi), cosTheta);
    *pdf = TR_INV_TWOPI * (1.f / (1.f - cosMax));
    return to_world(&f, d);
}

static v3 di_render(const ctx_t* c, ray_t ray, tr_sampler* smp) {
    const tro_scene* s = c->s;
    const tro_params* P = c->p;
    const int es = P->di_emitter_samples, bs = P->di_bsdf_samples, strat = P->di_strategy;
    v3 Lr = V3(0, 0, 0);
    hit_t hit = zero_hit();
    if (!scene_intersect(s, &ray, &hit)) return Lr;
    v3 le = emission_of(s, &hit);
    if (!veq0(le)) return le;
    const tro_bsdf* b = bsdf_of(s, &hit);
    if (strat == 1 || strat == 2) { /* renderArea (:143-195) / renderSolidAngle (:244-311) */
        for (int i = 0; i < es; ++i) {
            float emitterPdf;
            int id = select_emitter(s, s_next(smp), &emitterPdf);
            const tro_emitter* e = &s->emit[id];
            v2 u = s_next2d(smp);
            if (strat == 1) {
                v3 ne = sq_uniform_sphere(u);
                v3 pos = vadd(vscale(ne, e->radius), e->center);
                v3 wiW = vnormalize(vsub(pos, hit.p));
                float pdf = 1.f / (4 * TR_PI * e->radius * e->radius);
                v3 dd = vsub(hit.p, pos);
                float d2 = vdot(dd, dd);
                float cosOut = vdot(vneg(wiW), ne);
                v3 wil = to_local(&hit.fs, wiW);
                if (cosOut <= 0.f || wil.z <= 0.f) continue;
                ray_t r = {hit.p, wiW, TR_EPSILON, tr_sqrtf(d2) - TR_EPSILON};
                hit_t vis = zero_hit();
                if (!scene_intersect(s, &r, &vis)) {
                    hit.wi = wil;
                    float a2s = cosOut * (1.f / d2);
                    v3 t = vmul(e->radiance, bsdf_eval(b, &hit));
                    Lr = vadd(Lr, vscale(vscale(vscale(t, 1.f / pdf), 1.f / emitterPdf), a2s));
                }
            } else {
                float pdf;
                v3 wiW = sample_sphere_solid_angle(u, hit.p, e->center, e->radius, &pdf);
                v3 wil = to_local(&hit.fs, wiW);
                if (wil.z <= 0.f) continue;
                v3 dc = vsub(e->center, hit.p);
                ray_t r = {hit.p, wiW, TR_EPSILON, tr_sqrtf(vdot(dc, dc)) + TR_EPSILON}; /* glm::distance */
                hit_t vis = zero_hit();
                int vh = scene_intersect(s, &r, &vis);
                if ((vh && vis.shape == e->shape) || (!vh && ray_sphere_hit(&r, e->center, e->radius))) {
                    hit.wi = wil;
                    v3 t = vmul(e->radiance, bsdf_eval(b, &hit));
                    Lr = vadd(Lr, vscale(vscale(t, 1.f / pdf), 1.f / emitterPdf));
                }
            }
        }
        return vdivs(Lr, (float)es);
    }
    if (strat == 3) { /* renderCosineHemisphere (:198-233) */
        for (int i = 0; i < es; ++i) {
            v3 local = sq_cosine_hemisphere(s_next2d(smp));
            v3 world = vnormalize(to_world(&hit.fs, local));
            ray_t r = {hit.p, world, TR_EPSILON, INFINITY};
            hit_t vis = zero_hit();
            if (scene_intersect(s, &r, &vis)) {
                hit.wi = local;
                v3 t = vmul(emission_of(s, &vis), bsdf_eval(b, &hit));
                Lr = vadd(Lr, vscale(t, 1.0f / cosine_pdf(local)));
            }
        }
        return vdivs(Lr, (float)es);
    }
    if (strat == 4) { /* renderBSDF (:235-264) */
        for (int i = 0; i < bs; ++i) {
            float pdf;
            v3 f = bsdf_sample(b, &hit, s_next2d(smp), &pdf);
            ray_t r = {hit.p, to_world(&hit.fs, hit.wi), TR_EPSILON, INFINITY};
            hit_t vis = zero_hit();
            if (scene_intersect(s, &r, &vis))
                Lr = vadd(Lr, vscale(vmul(emission_of(s, &vis), f), (float)(1.0 / (double)pdf)));
        }
        return vdivs(Lr, (float)bs);
    }
    if (strat != 5) abort(); /* "Error: wrong strategy" (direct.h:440-441) */
    /* renderMIS (:313-428) */
    v3 eEst = V3(0, 0, 0), bEst = V3(0, 0, 0);
    for (int i = 0; i < es; ++i) {
        float emitterPdf;
        int id = select_emitter(s, s_next(smp), &emitterPdf);
        const tro_emitter* e = &s->emit[id];
        v2 u = s_next2d(smp);
        float pdf;
        v3 wiW = sample_sphere_solid_angle(u, hit.p, e->center, e->radius, &pdf);
        v3 wil = to_local(&hit.fs, wiW);
        if (wil.z <= 0.f) continue;
        ray_t r = {hit.p, wiW, TR_EPSILON, INFINITY};
        hit_t vis = zero_hit();
        int vh = scene_intersect(s, &r, &vis);
        if ((vh && vis.shape == e->shape) || (!vh && ray_sphere_hit(&r, e->center, e->radius))) {
            hit.wi = wil;
            float bsdfPdf = bsdf_pdf(b, &hit);
            float w = balance_heuristic((float)es, pdf * emitterPdf, (float)bs, bsdfPdf);
            v3 t = vscale(vmul(e->radiance, bsdf_eval(b, &hit)), w);
            eEst = vadd(eEst, vscale(vscale(t, 1.f / pdf), 1.f / emitterPdf));
        }
    }
    eEst = es == 0 ? V3(0, 0, 0) : vdivs(eEst, (float)es);
    for (int i = 0; i < bs; ++i) {
        float pdf;
        v3 f = bsdf_sample(b, &hit, s_next2d(smp), &pdf);
        ray_t r = {hit.p, to_world(&hit.fs, hit.wi), TR_EPSILON, INFINITY};
        hit_t vis = zero_hit();
        if (!scene_intersect(s, &r, &vis)) continue;
        v3 Le = emission_of(s, &vis);
        if (veq0(Le)) continue;
        int eid = s->shape_emitter[vis.shape];
        if (eid < 0) abort(); /* the reference asserts */
        const tro_emitter* e = &s->emit[eid];
        v3 dd = vsub(hit.p, e->center);
        float sin2 = e->radius * e->radius / vdot(dd, dd);
        float cosMax = tr_sqrtf(fmaxf(0.f, 1.f - sin2));
        float esap = TR_INV_TWOPI * (1.f / (1.f - cosMax));
        esap *= 1.f / (float)s->nemit;
        float w = balance_heuristic((float)bs, pdf, (float)es, esap);
        bEst = vadd(bEst, vscale(vscale(vmul(Le, f), w), 1.f / pdf));
    }
    bEst = bs == 0 ? V3(0, 0, 0) : vdivs(bEst, (float)bs);
    return vadd(Lr, vadd(eEst, bEst));
}

static v3 integrator_render(const ctx_t* c, ray_t ray, tr_sampler* smp) {
    if (c->p->integrator == 2) return di_render(c, ray, smp);
    return c->p->integrator == 1 ? pt_render(c, ray, smp) : bdpt_render(c, ray, smp);
}

/* ------------------------------------------------------------------ driver */
typedef struct {
    m4 c2w;
    float invW, invH, angle, aspect;
} camdrv_t;

static void setup(ctx_t* c, camdrv_t* cd, const tro_scene* s, const tro_params* p, float* fb) {
    c->s = s;
    c->W = p->width;
    c->H = p->height;
    c->spp = p->spp;
    c->rr_depth = p->rr_depth;
    c->strategy = p->strategy;
    c->p = p;
    c->cam_o = V3(p->eye[0], p->eye[1], p->eye[2]);
    tr_camera_mats(p, &c->w2c, &cd->c2w, &c->c2clip, &c->ndc2screen, &cd->angle, &cd->aspect, &c->cam_fwd, &c->vnear);
    cd->invW = 1.f / (float)p->width;
    cd->invH = 1.f / (float)p->height;
    c->fb = fb;
}

/* Camera ray of renderer.cpp:162-192 (jitter draws first when spp > 1). */
static ray_t camera_ray(const ctx_t* c, const camdrv_t* cd, int pixel, tr_sampler* smp) {
    int j = pixel % c->W;
    int i = pixel / c->W;
    float y = (1.f - ((float)i + 0.5f) * cd->invH) * 2.f - 1.f;
    float x = (((float)j + 0.5f) * cd->invW) * 2.f - 1.f;
    v4 ipp;
    if (c->spp == 1) {
        ipp.x = x * cd->angle * cd->aspect;
        ipp.y = y * cd->angle;
    } else {
        v2 rs = s_next2d(smp);
        rs.x -= 0.5f;
        rs.y -= 0.5f;
        rs.x = rs.x * cd->invW;
        rs.y = rs.y * cd->invH;
        ipp.x = (x + rs.x) * cd->angle * cd->aspect;
        ipp.y = (y + rs.y) * cd->angle;
    }
    ipp.z = -1.f;
    ipp.w = 0.f;
    v4 d4 = tr_m4v4(&cd->c2w, ipp);
    ray_t r = {c->cam_o, vnormalize(V3(d4.x, d4.y, d4.z)), 1.f, 1000.f};
    return r;
}

static inline uint32_t seed_for(uint32_t base, int pixel, int spp, int k) {
    return base + (uint32_t)pixel * (uint32_t)spp + (uint32_t)k;
}

int64_t tro_render(const tro_scene* s, const tro_params* p, float* fb, int row_begin, int row_end, int row_stride) {
    ctx_t c;
    camdrv_t cd;
    setup(&c, &cd, s, p, fb);
    tr_sampler* smp = (tr_sampler*)malloc(sizeof(tr_sampler));
    int64_t n = 0;
    if (row_stride < 1) row_stride = 1;
    for (int row = row_begin; row < row_end && row < p->height; row += row_stride) {
        for (int j = 0; j < p->width; j++) {
            int pixel = row * p->width + j;
            v3 acc = V3(0, 0, 0);
            for (int k = 0; k < p->spp; k++) {
                mt_seed(smp, seed_for(p->seed_base, pixel, p->spp, k));
                ray_t ray = camera_ray(&c, &cd, pixel, smp);
                acc = vadd(acc, integrator_render(&c, ray, smp));
                n++;
            }
            v3 add = vscale(acc, 1.f / (float)p->spp);
            fb[3 * (size_t)pixel + 0] += add.x;
            fb[3 * (size_t)pixel + 1] += add.y;
            fb[3 * (size_t)pixel + 2] += add.z;
        }
    }
    free(smp);
    return n;
}

/* Debugging aid (tools/rr_find.py): samples [s_lo, s_hi) of one image row in the
 * frame kernels' numbering (s = j * spp + k), each added as Li / spp on its own
 * (the GPU's order of adds, not the reference's per-pixel sum). */
int64_t tro_render_row_samples(const tro_scene* s, const tro_params* p, float* fb, int row, int64_t s_lo,
                               int64_t s_hi) {
    ctx_t c;
    camdrv_t cd;
    setup(&c, &cd, s, p, fb);
    tr_sampler* smp = (tr_sampler*)malloc(sizeof(tr_sampler));
    int64_t n = 0;
    for (int64_t q = s_lo; q < s_hi; q++) {
        const int j = (int)(q / p->spp), k = (int)(q % p->spp);
        const int pixel = row * p->width + j;
        mt_seed(smp, seed_for(p->seed_base, pixel, p->spp, k));
        ray_t ray = camera_ray(&c, &cd, pixel, smp);
        const v3 add = vscale(integrator_render(&c, ray, smp), 1.f / (float)p->spp);
        fb[3 * (size_t)pixel + 0] += add.x;
        fb[3 * (size_t)pixel + 1] += add.y;
        fb[3 * (size_t)pixel + 2] += add.z;
        n++;
    }
    free(smp);
    return n;
}

void tro_sample(const tro_scene* s, const tro_params* p, int pixel, int k, float Li[3], float* fb) {
    ctx_t c;
    camdrv_t cd;
    setup(&c, &cd, s, p, fb);
    tr_sampler* smp = (tr_sampler*)malloc(sizeof(tr_sampler));
    mt_seed(smp, seed_for(p->seed_base, pixel, p->spp, k));
    ray_t ray = camera_ray(&c, &cd, pixel, smp);
    v3 L = integrator_render(&c, ray, smp);
    Li[0] = L.x;
    Li[1] = L.y;
    Li[2] = L.z;
    free(smp);
}
