// The lane-decoupled build of the BDPT megakernel ("dq": decoupled connection
// queue). Same per-sample arithmetic and random-number order as
// bdpt_kernels.hip (reference src/integrators/bdpt.h:46-241), different
// schedule: a lane is either an OWNER, running a camera sample's primary ray
// and its two random walks (closest-hit queries only), or a HELPER, running one
// connection task — connectToCamera (bdpt.h:295-371), connectToLight
// (bdpt.h:374-430) or connectVertices with one light vertex (bdpt.h:434-483) —
// whose shadow ray it traces itself and whose contribution it adds to the
// framebuffer (float reassociation only, like every other add here).
//
// An owner at a light vertex writes the vertex record and pushes a camera task;
// at an eye vertex it writes the eye-vertex record (with the emitter sample it
// drew for next-event estimation, bdpt.h:376-381) and pushes 1 + nl tasks; then
// it continues its walk in the same shading step instead of waiting for nl + 1
// shadow rays one after another. Tasks go to a per-block ring in LDS (4-byte
// descriptors); idle lanes pop them, so the connection bodies run for many
// lanes at once and their shadow rays share walks. When the ring is full an
// owner runs the rest of its own tasks itself (the serial schedule of
// bdpt_kernels.hip), so no owner ever waits on another lane.
//
// Records of a sample stay valid until its last task is done: each lane slot
// has two record buffers (samples alternate) and a per-slot count of
// outstanding tasks per buffer; a lane whose next buffer is still referenced
// takes tasks instead of a new sample.
#include <hip/hip_runtime.h>

#define BDPT_BSDF_TABLE 0
#ifndef BDPT_LDS_STACK
#define BDPT_LDS_STACK 6  // one traversal-stack entry less in LDS than the default build: room for the task ring
#endif
#include "bdpt_path.hpp"

namespace bdpt {
namespace dev {

#ifndef BDPT_WAVES_PER_EU
#define BDPT_WAVES_PER_EU 4
#endif
#ifndef BDPT_SHADE_READY
#define BDPT_SHADE_READY 48
#endif
#ifndef BDPT_TRAV_SPLIT
#define BDPT_TRAV_SPLIT 8
#endif
#ifndef BDPT_WALK_UNROLL
#define BDPT_WALK_UNROLL 1
#endif
#ifndef BDPT_DQ_RING
#define BDPT_DQ_RING 512  // task descriptors per block (LDS)
#endif
#ifndef BDPT_DQ_HELPER_WAVES
#define BDPT_DQ_HELPER_WAVES 1  // waves per block whose idle lanes take tasks before new samples
#endif
#ifndef BDPT_DQ_ROUNDS
#define BDPT_DQ_ROUNDS 2  // task-phase rounds per loop iteration (a rejected task's lane pops again; 1 / 2 / 64: 152 / 172 / 166)
#endif
#ifndef BDPT_DQ_HIGH
#define BDPT_DQ_HIGH (BDPT_DQ_RING / 2)  // ring fill above which every idle lane takes tasks
#endif

constexpr int kDqBlock = 256;
constexpr uint32_t kDqRing = BDPT_DQ_RING;
static_assert((kDqRing & (kDqRing - 1)) == 0, "ring size is a power of two");

// Task descriptor: type | owner lane in the block << 2 | record buffer << 10 |
// eye vertex << 11 | light vertex << 17 | self << 23 (an owner running its own task).
enum : uint32_t { T_SPLAT = 0, T_NEE = 1, T_CONN = 2 };
constexpr uint32_t kDescSelf = 1u << 23;
__device__ __forceinline__ uint32_t dq_desc(uint32_t type, uint32_t ol, uint32_t buf, uint32_t e, uint32_t v) {
    return type | (ol << 2) | (buf << 10) | (e << 11) | (v << 17);
}

// Lane states beyond bdpt_path.hpp's: a task's shadow ray from the camera
// (connectToCamera) or from an eye vertex; an owner with own tasks still to run;
// an owner resuming its walk after them.
enum : uint32_t { ST_TSPLAT = 8, ST_TASK = 9, ST_BACKLOG = 10, ST_RESUME = 11, ST_OTSPLAT = 12, ST_OTASK = 13,
                  ST_FINWAIT = 14 };
// ST_OTSPLAT / ST_OTASK: an owner's own task (its descriptor is not kept: the
// owner's LaneCold still holds its sample, prim_tri included)
enum : uint32_t { A_PUSH = 20, A_RESUME_LIGHT, A_RESUME_EYE };

// Owner bookkeeping packed into LaneCold words the decoupled schedule frees:
//   nl word:  bits 0..7 stored light vertices, bit 8 record buffer, bits 9..15 eye records written
//   ci word:  backlog: bits 0..7 next own task, 8..15 end, 16..21 eye record, bit 24 light side
//   rr word:  outstanding tasks of this slot's records, buffer 0 in bits 0..15, buffer 1 in 16..31
//   prim_tri: (task mode) the descriptor being run
struct DqRing {
    uint32_t lock, head, tail, owners;  // owners: samples in flight in the block
    uint32_t e[kDqRing];
};

__device__ __forceinline__ uint32_t& cold_u(float& f) { return *reinterpret_cast<uint32_t*>(&f); }
__device__ __forceinline__ int dq_nl(const LaneCold& c) { return c.nl & 0xff; }
__device__ __forceinline__ uint32_t dq_buf(const LaneCold& c) { return (static_cast<uint32_t>(c.nl) >> 8) & 1u; }
__device__ __forceinline__ uint32_t dq_ne(const LaneCold& c) { return (static_cast<uint32_t>(c.nl) >> 9) & 0x7fu; }

// Record stores: light vertices (64 B, bdpt_path.hpp LightStore layout) and eye
// vertices (128 B: (p, vcm) (n, vc) (wo, pixel) (tp, mat | graze << 24)
// (e_p, emitter pdf x position pdf) (e_n, emitter id) + 32 B pad), slot-major,
// two buffers per slot.
struct DqStores {
    float4* lv;  // [(slot * 2 + buf) * lv_max + v] * 4
    float4* ev;  // [(slot * 2 + buf) * ev_max + e] * 8
    uint32_t lv_max, ev_max;
    __device__ __forceinline__ float4* light(uint32_t slot, uint32_t buf, uint32_t v) const {
        return lv + ((static_cast<size_t>(slot) * 2 + buf) * lv_max + v) * 4;
    }
    __device__ __forceinline__ float4* eye(uint32_t slot, uint32_t buf, uint32_t e) const {
        return ev + ((static_cast<size_t>(slot) * 2 + buf) * ev_max + e) * 8;
    }
};

__device__ __forceinline__ uint32_t dq_load(uint32_t& w) {
    return __hip_atomic_load(&w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void dq_lock(DqRing& q) {
    while (atomicCAS(&q.lock, 0u, 1u) != 0u) __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void dq_unlock(DqRing& q) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __hip_atomic_store(&q.lock, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ------------------------------------------------------------ task execution
// Computes the task in L.c.prim_tri (descriptor) up to its shadow ray: L.ray,
// L.c.pend, L.c.pend_px and the state (ST_TSPLAT / ST_TASK); false when the
// reference would not trace it (cosines, zero contribution, off-image splat).
// Each body restates the megakernel's (bdpt_path.hpp) arithmetic exactly.
template <bool COUNT>
__device__ __forceinline__ bool dq_task(Lane& L, uint32_t d, const DevScene& sc, const DevFrame& fr,
                                        const DqStores& st, Counts& cnt) {
    const uint32_t type = d & 3u, ol = (d >> 2) & 0xffu, buf = (d >> 10) & 1u, e = (d >> 11) & 0x3fu,
                   v = (d >> 17) & 0x3fu;
    const uint32_t oslot = blockIdx.x * kDqBlock + ol;
    const f3 cam_o = mk(fr.cam_o[0], fr.cam_o[1], fr.cam_o[2]);
    // a descriptor outside the records is a schedule bug: counted (bdpt_stats.schedule_errors), never read
    if (type > T_CONN || v >= st.lv_max || e >= st.ev_max) {
        if (fr.diag) gadd(fr.diag + kDiagErrors, 1ull);
        return false;
    }
    if (type == T_SPLAT) {  // connectToCamera (bdpt.h:295-371) of light vertex v
        const float4* q = st.light(oslot, buf, v);
        const float4 a = gld4(q), b = gld4(q + 1), c = gld4(q + 2), dd = gld4(q + 3);
        const f3 p = xyz(a), n = xyz(b), wo = xyz(c), tp = xyz(dd);
        const float vcm = a.w, vc = b.w;
        const BsdfRecord& bs = bsdf_of(sc, __float_as_int(dd.w));
        const f3 fwd = mk(fr.cam.fwd[0], fr.cam.fwd[1], fr.cam.fwd[2]);
        f3 e2l = p - cam_o;
        const float invD2 = rcp_cr(dot(e2l, e2l));
        e2l = e2l * sqrt_cr(invD2);
        int xp, yp;
        splat_pixel(fr.cam, p, xp, yp);
        if (xp < 0 || yp < 0 || xp >= fr.W || yp >= fr.H) return false;
        const float cosCamera = dot(fwd, e2l);
        if (cosCamera <= 0.f) return false;
        if (dot(-e2l, n) <= 0.f) return false;  // wi.z (the frame's z component, to_local)
        const f3 wi = local_for(bs, n, -e2l);
        const EvalPdfs ep = bsdf_eval_pdfs(bs, wi, wo);
        if (is_zero(ep.f)) return false;
        const float dn = div_cr(fr.cam.vnear, cosCamera);
        const float img2solid = div_cr(dn * dn, cosCamera);
        const float img2surf = img2solid * (wi.z * invD2);
        const float surf2img = rcp_cr(img2surf);
        const float nlight = static_cast<float>(fr.W * fr.H);
        f3 rad = tp * (ep.f * rcp_cr(wi.z));
        rad = rad * rcp_cr(surf2img);
        rad = rad * fr.inv_pixels;
        rad = rad * fr.inv_spp;
        const float reversePdf_a = 1.f * img2surf;
        const float lightWeight = div_cr(reversePdf_a, nlight) * (vcm + ep.rev * vc);
        const float mis = rcp_cr(lightWeight + 1.f + 0.f);
        L.c.pend = (fr.strategy == 0) ? rad * mis : rad;
        L.c.pend_px = yp * fr.W + xp;
        L.ray = shadow_ray(cam_o, p);
        L.state = (d & kDescSelf) ? ST_OTSPLAT : ST_TSPLAT;
        return true;
    }
    const float4* qe = st.eye(oslot, buf, e);
    const float4 ea = gld4(qe), eb = gld4(qe + 1), ec = gld4(qe + 2), ed = gld4(qe + 3);
    const f3 ep_ = xyz(ea), en = xyz(eb), ewo = xyz(ec), etp = xyz(ed);
    const float evcm = ea.w, evc = eb.w;
    const uint32_t mw = __float_as_uint(ed.w);
    const BsdfRecord& be = bsdf_of(sc, static_cast<int>(mw & 0xffffffu));
    L.c.pend_px = __float_as_int(ec.w);
    L.h.n = en;  // the shadow ray leaves the eye vertex: its normal and graze code (cull_near_for)
    L.h.shape = static_cast<int>(mw & 0xff000000u);
    if (type == T_NEE) {  // connectToLight (bdpt.h:374-430) with the owner's emitter sample
        const float4 ee = gld4(qe + 4), ef = gld4(qe + 5);
        const f3 e_p = xyz(ee), e_n = xyz(ef);
        const float e_pp = ee.w;  // emitterPdf * position pdf, as the owner formed it
        const EmitterRecord& em = emitter_of(sc, __float_as_int(ef.w));
        f3 dir = ep_ - e_p;
        const float d2 = dot(dir, dir);
        dir = dir * rcp_cr(sqrt_cr(d2));
        const float cosAtLight = dot(e_n, dir);
        const float cosAtEye = dot(-dir, en);
        if (cosAtLight <= 0.f || cosAtEye <= 0.f) return false;
        const f3 wi = local_for(be, en, -dir);
        const float pdf_w = div_cr(e_pp * d2, cosAtLight);
        const EvalPdfs ep = bsdf_eval_pdfs(be, wi, ewo);
        const f3 Li = ((ep.f * rcp_cr(pdf_w)) * etp) * ld3(em.radiance);
        if (is_zero(Li)) return false;
        const float lightWeight = div_cr(ep.fwd, pdf_w);
        const float eyeCurRev_a = cosAtEye * rcp_cr(d2) * kInvTwoPi;
        const float eyeWeight = eyeCurRev_a * (evcm + ep.rev * evc);
        const float mis = rcp_cr(lightWeight + 1.f + eyeWeight);
        L.c.pend = (fr.strategy == 0) ? Li * mis : Li;
        L.ray = shadow_ray(ep_, e_p);
        L.state = (d & kDescSelf) ? ST_OTASK : ST_TASK;
        return true;
    }
    // connectVertices (bdpt.h:434-483) of eye vertex e with light vertex v
    if (COUNT) cnt.c[5]++;
    const float4* ql = st.light(oslot, buf, v);
    const float4 la = gld4(ql), lb = gld4(ql + 1), lc = gld4(ql + 2), ld = gld4(ql + 3);
    const f3 lp = xyz(la), ln = xyz(lb), lwo = xyz(lc), ltp = xyz(ld);
    f3 dir = ep_ - lp;
    const float invD2 = rcp_cr(dot(dir, dir));
    dir = dir * sqrt_cr(invD2);
    const float cosL = dot(dir, ln), cosE = dot(-dir, en);
    if (cosL <= 0.f || cosE <= 0.f) return false;
    const BsdfRecord& bl = bsdf_of(sc, __float_as_int(ld.w));
    const f3 wiL = local_for(bl, ln, dir);
    const f3 wiE = local_for(be, en, -dir);
    const EvalPdfs eL = bsdf_eval_pdfs(bl, wiL, lwo), eE = bsdf_eval_pdfs(be, wiE, ewo);
    f3 Li = eL.f * eE.f;
    Li = Li * ((ltp * etp) * invD2);
    const float lightPathRev_a = eE.fwd * cosL * invD2;
    const float eyePathRev_a = eL.fwd * cosE * invD2;
    const float lightWeight = lightPathRev_a * (la.w + eL.rev * lb.w);
    const float eyeWeight = eyePathRev_a * (evcm + eE.rev * evc);
    const float mis = rcp_cr(lightWeight + 1.f + eyeWeight);
    L.c.pend = Li * mis;
    L.ray = shadow_ray(ep_, lp);
    L.state = (d & kDescSelf) ? ST_OTASK : ST_TASK;
    return true;
}

// Next own task of an owner in backlog mode: the descriptor, or false when
// its backlog is done.
__device__ __forceinline__ bool dq_own_next(LaneCold& c, uint32_t& d) {
    const uint32_t b = static_cast<uint32_t>(c.ci);
    const uint32_t next = b & 0xffu, end = (b >> 8) & 0xffu, e = (b >> 16) & 0x3fu;
    if (next >= end) return false;
    const uint32_t me = threadIdx.x;
    if (b & (1u << 24)) d = dq_desc(T_SPLAT, me, dq_buf(c), 0u, e) | kDescSelf;  // e holds the light vertex
    else d = (next == 0 ? dq_desc(T_NEE, me, dq_buf(c), e, 0u) : dq_desc(T_CONN, me, dq_buf(c), e, next - 1)) | kDescSelf;
    c.ci = static_cast<int>(b + 1u);
    return true;
}

__device__ __forceinline__ bool dq_is_shadow(uint32_t st) {
    return st == ST_TSPLAT || st == ST_TASK || st == ST_OTSPLAT || st == ST_OTASK;
}
__device__ __forceinline__ float dq_cull_near(const Lane& L) {
    const uint32_t st = L.state;
    if (st == ST_PRIMARY || st == ST_TSPLAT || st == ST_OTSPLAT) return kCullNear;
    return graze_exempt(L.ray.d, L.h.n, L.h.shape) ? kNoCullNear : kCullNear;
}

// Eye-side contributions (next-event estimation, vertex connections) go to the
// owner's eye estimate in LDS (LaneCold::Li, three ds_add_f32), as the serial
// schedule adds them to its Li: the owner adds the estimate to the framebuffer
// once, when its sample has ended AND every task of it is done (ST_FINWAIT
// until then; the lane takes ring tasks meanwhile). The sums differ from the
// reference's only in order (float reassociation, like the atomics).
__device__ __forceinline__ void dq_li_add(LaneCold& owner, f3 v) {
    atomicAdd(&owner.Li.x, v.x);
    atomicAdd(&owner.Li.y, v.y);
    atomicAdd(&owner.Li.z, v.z);
}
constexpr uint32_t kFinWait = 1u << 16;  // LaneCold::nl: the owner's sample ended, its tasks are not all done

// The result of the lane's query: owners continue their sample, task lanes add
// the contribution of an unoccluded shadow ray.
template <bool COUNT>
__device__ __forceinline__ uint32_t dq_resolve(Lane& L, int res, float t, float u, float v, const DevScene& sc,
                                               const DevFrame& fr, float* __restrict__ fb, LaneCold* cold,
                                               Counts& cnt) {
    const uint32_t st = L.state;
    if (dq_is_shadow(st)) {
        const bool own = st == ST_OTSPLAT || st == ST_OTASK;
        if (res < 0) {
            if (st == ST_TSPLAT || st == ST_OTSPLAT) {
                if (COUNT) cnt.c[6]++;
                splat_add(fb, L.c.pend_px, L.c.pend);
            } else {
                // Li += contribution of the owner's sample (bdpt.h:140, :150)
                dq_li_add(own ? L.c : cold[(static_cast<uint32_t>(L.c.prim_tri) >> 2) & 0xffu], L.c.pend);
            }
        }
        if (own) {
            L.state = ST_BACKLOG;  // the owner's next own task (or its walk) in the task phase
            return A_DONE;
        }
        const uint32_t d = static_cast<uint32_t>(L.c.prim_tri);
        const uint32_t ol = (d >> 2) & 0xffu, buf = (d >> 10) & 1u;
        atomicSub(&cold_u(cold[ol].rr), 1u << (16 * buf));  // after the Li add (LDS is in order per wave)
        L.state = (static_cast<uint32_t>(L.c.nl) & kFinWait) ? ST_FINWAIT : ST_IDLE;
        return A_DONE;
    }
    bool hit = res >= 0 && t <= L.ray.max_t && t >= L.ray.min_t;  // accel.h:133
    if (hit && st != ST_PRIMARY) shade_hit(sc, res, u, v, t, L.ray.d, L.h);
    uint32_t act;
    switch (st) {
        case ST_PRIMARY:
            if (!hit) act = A_FINISH;
            else {
                L.c.prim_tri = res;
                L.c.Li = mk(t, u, v);
                act = (fr.strategy == 2) ? A_START_EYE : A_START_LIGHT;
            }
            break;
        case ST_LIGHT: act = hit ? A_LIGHT_VERTEX : A_START_EYE; break;
        case ST_EYE: act = hit ? A_EYE_VERTEX : A_FINISH; break;
        case ST_DEFER: act = A_START_EYE; break;
        case ST_RESUME: act = (static_cast<uint32_t>(L.c.ci) & (1u << 24)) ? A_RESUME_LIGHT : A_RESUME_EYE; break;
        default: act = A_DONE;
    }
    if (++L.c.steps > max_steps_per_sample(fr.rr_depth) && act != A_FINISH) act = A_FINISH;
    return act;
}

#define DQ_ACTION(ID, COND)               \
    if (COUNT) tally_action(cnt, (COND)); \
    if (COND) do {                        \
        const ActionClock<COUNT> clk_(cnt, ID);
#define DQ_END \
    }          \
    while (0)

// The owner's shading sweep (one forward pass over the action DAG, as
// bdpt_path.hpp advance()): walks and record writes; the connections are
// pushed as tasks.
template <bool COUNT>
__device__ void dq_advance(Lane& L, uint32_t act, const DevScene& sc, const DevFrame& fr, float* __restrict__ fb,
                           const DqStores& st, DqRing& q, Counts& cnt) {
    const f3 cam_o = mk(fr.cam_o[0], fr.cam_o[1], fr.cam_o[2]);
    const f3 fwd = mk(fr.cam.fwd[0], fr.cam.fwd[1], fr.cam.fwd[2]);
    const uint32_t me = threadIdx.x, slot = blockIdx.x * kDqBlock + me;
    uint32_t ntask = 0, tdesc = 0;  // tasks this lane pushes in A_PUSH: first descriptor, count
    DQ_ACTION(21, act == A_START_EYE) {  // eyeSubpathWalk prologue (bdpt.h:47-65)
        const f3 prim = L.c.Li;
        if (fr.strategy == 1) {  // LIGHT_TRACING: Li = Le at the primary hit (bdpt.h:231)
            const int mat = __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(L.c.prim_tri)).w);
            L.c.Li = ld3(bsdf_of(sc, mat).emission);
            act = A_FINISH;
            break;
        }
        const float cosCamera = dot(fwd, L.c.cam_d);
        const float d = div_cr(fr.cam.vnear, cosCamera);
        const float t1Pdf = 1.f * div_cr(d * d, cosCamera);
        L.c.tp = mk(1.f, 1.f, 1.f);
        L.c.vc = 0.f;
        L.c.vcm = static_cast<float>(fr.W * fr.H) * rcp_cr(t1Pdf);
        L.c.depth = 1;
        L.c.pure = 1u;
        L.c.Li = mk(0.f, 0.f, 0.f);
        L.ray = Ray{cam_o, L.c.cam_d, 1.f, 1000.f};
        act = A_EYE_NEXT;
        if (1 < fr.rr_depth) {  // the eye walk's first hit is the primary hit (bdpt.h:70 repeats :225)
            shade_hit(sc, L.c.prim_tri, prim.y, prim.z, prim.x, L.ray.d, L.h);
            L.c.steps++;
            act = A_EYE_VERTEX;
        }
    } DQ_END;
    DQ_ACTION(22, act == A_EYE_VERTEX) {  // bdpt.h:73-136
        const float dist2 = L.h.dist * L.h.dist;
        const float absCosIn = fabsf(L.h.wo.z);
        L.c.vcm *= div_cr(dist2, absCosIn);
        L.c.vc *= rcp_cr(absCosIn);
        const BsdfRecord& b = bsdf_of(sc, L.h.mat);
        const f3 emission = ld3(b.emission);
        if (!is_zero(emission)) {
            const int eid = shape_emitter_of(sc, shape_id(L.h.shape));
            if (eid >= 0) {
                const EmitterRecord& e = emitter_of(sc, eid);
                const float emitterPdf = sc.inv_nemit;
                if (L.c.depth > 1) {
                    f3 contrib = ld3(e.radiance) * L.c.tp;
                    const float pA = rcp_cr(e.area * emitterPdf);
                    const float camW = pA * L.c.vcm + (pA * kInvTwoPi) * L.c.vc;
                    const float mis = rcp_cr(1.f + camW);
                    // (Li in LDS takes helpers' adds concurrently: atomic adds)
                    if (fr.strategy == 2) {
                        if (L.c.pure) dq_li_add(L.c, contrib);
                    } else {
                        if (!L.c.pure) contrib = contrib * mis;
                        dq_li_add(L.c, contrib);
                    }
                } else if (L.c.depth == 1) {
                    dq_li_add(L.c, emission);
                }
            }
            act = A_FINISH;
            break;
        }
        if (is_delta(b)) {
            act = A_EYE_CONTINUE;
            break;
        }
        L.c.pure = 0u;
        act = A_NEE;
    } DQ_END;
    int e_id = 0, e_graze = 0;
    float e_pdf = 0.f, e_pos_pdf = 0.f;
    f3 e_n = mk(0.f, 0.f, 0.f), e_p = e_n;
    DQ_ACTION(23, act == A_START_LIGHT || act == A_NEE) {  // selectEmitter + sampleEmitterPosition: 4 draws
        e_id = sample_emitter(sc, L.rng, e_pdf, e_n, e_p, e_pos_pdf, &e_graze);
    } DQ_END;
    DQ_ACTION(24, act == A_START_LIGHT) {  // lightSubpathWalk prologue (bdpt.h:158-182): 6 draws
        const EmitterRecord& e = emitter_of(sc, e_id);
        float areaPdf = e_pos_pdf;
        const f3 edir = uniform_hemisphere(next2(L.rng));
        float emissionPdf = kInvTwoPi * areaPdf;
        areaPdf *= e_pdf;
        emissionPdf *= e_pdf;
        f3 fs, ft;
        make_frame(e_n, fs, ft);
        L.ray = Ray{e_p, to_world(fs, ft, e_n, edir), kEpsilon, 3.402823466e+38f};
        L.h.n = e_n;
        L.h.shape = e_graze;
        L.c.tp = (ld3(e.radiance) * edir.z) * rcp_cr(emissionPdf);
        L.c.vc = edir.z * rcp_cr(emissionPdf);
        L.c.vcm = div_cr(areaPdf, emissionPdf);
        L.c.nl = static_cast<int>(static_cast<uint32_t>(L.c.nl) & ~0xffu);  // nl = 0 (buffer, eye count kept)
        L.c.depth = 1;
        if (edir.z <= 0.f) {
            L.state = ST_DEFER;
            act = A_ISSUED;
        } else {
            act = A_LIGHT_NEXT;
        }
    } DQ_END;
    DQ_ACTION(25, act == A_NEE) {  // the eye-vertex record for next-event estimation and the connections
        const uint32_t w = static_cast<uint32_t>(L.c.nl), buf = (w >> 8) & 1u, e = (w >> 9) & 0x7fu;
        float4* r = st.eye(slot, buf, e);
        lv_st(r, make_float4(L.h.p.x, L.h.p.y, L.h.p.z, L.c.vcm));
        lv_st(r + 1, make_float4(L.h.n.x, L.h.n.y, L.h.n.z, L.c.vc));
        lv_st(r + 2, make_float4(L.h.wo.x, L.h.wo.y, L.h.wo.z, __int_as_float(L.c.pixel)));
        lv_st(r + 3, make_float4(L.c.tp.x, L.c.tp.y, L.c.tp.z,
                                 __uint_as_float(static_cast<uint32_t>(L.h.mat) |
                                                 (static_cast<uint32_t>(L.h.shape) & 0xff000000u))));
        lv_st(r + 4, make_float4(e_p.x, e_p.y, e_p.z, e_pdf * e_pos_pdf));
        lv_st(r + 5, make_float4(e_n.x, e_n.y, e_n.z, __int_as_float(e_id)));
        L.c.nl = static_cast<int>(w + (1u << 9));
        ntask = 1u + (fr.strategy == 0 ? static_cast<uint32_t>(w & 0xffu) : 0u);
        tdesc = dq_desc(T_NEE, me, buf, e, 0u);
        act = A_PUSH;
    } DQ_END;
    DQ_ACTION(26, act == A_LIGHT_VERTEX) {  // bdpt.h:193-209: the record connectToCamera and the eye walk read
        const float dist2 = L.h.dist * L.h.dist;
        const float absCosIn = fabsf(L.h.wo.z);
        L.c.vcm *= div_cr(dist2, absCosIn);
        L.c.vc *= rcp_cr(absCosIn);
        act = A_LIGHT_CONTINUE;
        const BsdfRecord& b = bsdf_of(sc, L.h.mat);
        if (is_delta(b)) break;
        const uint32_t w = static_cast<uint32_t>(L.c.nl), buf = (w >> 8) & 1u, nl = w & 0xffu;
        float4* r = st.light(slot, buf, nl);
        lv_st(r, make_float4(L.h.p.x, L.h.p.y, L.h.p.z, L.c.vcm));
        lv_st(r + 1, make_float4(L.h.n.x, L.h.n.y, L.h.n.z, L.c.vc));
        lv_st(r + 2, make_float4(L.h.wo.x, L.h.wo.y, L.h.wo.z, 1.f));
        lv_st(r + 3, make_float4(L.c.tp.x, L.c.tp.y, L.c.tp.z, __int_as_float(L.h.mat)));
        ntask = 1u;
        tdesc = dq_desc(T_SPLAT, me, buf, 0u, nl);
        act = A_PUSH;
    } DQ_END;
    DQ_ACTION(27, act == A_PUSH) {  // the tasks to the block's ring; what does not fit, the owner runs itself
        const uint64_t m = __ballot(true);  // the pushing lanes (the sweep runs for the lanes that shade)
        // exclusive prefix of ntask (< 64) over those lanes, bit by bit from ballots
        const uint64_t below = m & ((1ull << (threadIdx.x & 63)) - 1ull);
        uint32_t pre = 0, total = 0;
#pragma unroll
        for (int bit = 0; bit < 6; bit++) {
            const uint64_t bm = __ballot((ntask >> bit) & 1u);
            pre += static_cast<uint32_t>(__popcll(bm & below)) << bit;
            total += static_cast<uint32_t>(__popcll(bm)) << bit;
        }
        const int leader = __ffsll(static_cast<unsigned long long>(m)) - 1;
        uint32_t base = 0, room = 0;
        if ((threadIdx.x & 63) == static_cast<uint32_t>(leader)) {
            dq_lock(q);
            base = q.tail;
            const uint32_t used = base - q.head;
            room = min(total, kDqRing - used);
            q.tail = base + room;
        }
        base = __shfl(base, leader);
        room = __shfl(room, leader);
        const uint32_t k = pre >= room ? 0u : min(ntask, room - pre);  // this lane's tasks that fit
        const bool light = (tdesc & 3u) == T_SPLAT;
        for (uint32_t i = 0; i < k; i++) {
            const uint32_t d = light ? tdesc : (i == 0 ? tdesc : (tdesc & ~3u) | T_CONN | ((i - 1) << 17));
            q.e[(base + pre + i) & (kDqRing - 1)] = d;
        }
        if (k) atomicAdd(&cold_u(L.c.rr), k << (16 * ((tdesc >> 10) & 1u)));
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): this wave's record stores are done before the publish
        if ((threadIdx.x & 63) == static_cast<uint32_t>(leader)) dq_unlock(q);
        if (k < ntask) {  // backlog: own tasks k .. ntask - 1 (light: the one camera task)
            const uint32_t e = light ? ((tdesc >> 17) & 0x3fu) : ((tdesc >> 11) & 0x3fu);
            L.c.ci = static_cast<int>(k | (ntask << 8) | (e << 16) | (light ? 1u << 24 : 0u));
            L.state = ST_BACKLOG;
            act = A_ISSUED;
        } else {
            act = light ? A_LIGHT_CONTINUE : A_EYE_CONTINUE;
        }
    } DQ_END;
    if (act == A_RESUME_LIGHT) act = A_LIGHT_CONTINUE;
    if (act == A_RESUME_EYE) act = A_EYE_CONTINUE;
    DQ_ACTION(28, act == A_LIGHT_CONTINUE || act == A_EYE_CONTINUE) {  // ContinuePathRandomWalk (bdpt.h:243-291)
        const bool light = act == A_LIGHT_CONTINUE;
        const BsdfRecord& b = bsdf_of(sc, L.h.mat);
        const bool delta = is_delta(b);
        const bool more = continue_walk(b, L.h, L.rng, L.c.tp, L.c.depth, L.c.vc, L.c.vcm, L.ray, 1.f);
        if (!light) {
            act = more ? A_EYE_NEXT : A_FINISH;
        } else if (more) {
            if (!delta) {
                L.c.nl++;  // the stored vertex joins the light subpath (bdpt.h:211-215)
                if (COUNT) cnt.c[4]++;
            }
            act = A_LIGHT_NEXT;
        } else {
            L.state = ST_DEFER;
            act = A_ISSUED;
        }
    } DQ_END;
    DQ_ACTION(29, act == A_LIGHT_NEXT) {  // the loop test of bdpt.h:188
        if (walk_continues(L, fr)) {
            L.state = ST_LIGHT;
            act = A_ISSUED;
        } else {
            L.state = ST_DEFER;
            act = A_ISSUED;
        }
    } DQ_END;
    DQ_ACTION(30, act == A_EYE_NEXT) {  // the loop test of bdpt.h:68
        if (walk_continues(L, fr)) {
            L.state = ST_EYE;
            act = A_ISSUED;
        } else {
            act = A_FINISH;
        }
    } DQ_END;
    DQ_ACTION(31, act == A_FINISH) {  // the sample's walks have ended: its estimate once its tasks are done
        L.c.nl = static_cast<int>(static_cast<uint32_t>(L.c.nl) | kFinWait);
        L.state = ST_FINWAIT;
        act = A_ISSUED;
    } DQ_END;
}
#undef DQ_ACTION
#undef DQ_END

// ------------------------------------------------------------------- kernel
struct DqParams {
    DevScene sc;
    DevFrame fr;
    float* fb;
    float* lv;
    float* ev;
    uint2* gstack;
    uint32_t nslots, ev_max;
    unsigned long long* work;
    unsigned long long* counters;
};

template <bool FULL, bool COUNT, bool SLACK>
__global__ __launch_bounds__(kDqBlock, BDPT_WAVES_PER_EU) void bdpt_frame_kernel_dq(const DqParams* __restrict__ kpp) {
    const DqParams& kp = *kpp;
    __shared__ uint2 stack_mem[kLdsStack * kDqBlock];
    __shared__ RootLds root_lds;
    __shared__ DqRing q;
    if (threadIdx.x == 0) q.lock = q.head = q.tail = q.owners = 0u;
    const bool root_in_lds = !FULL && root_lds_usable(kp.sc);
    if (!FULL) root_lds_fill(root_lds, kp.sc);
    scene_tables_to_lds(kp.sc);  // ends with a barrier (the ring's words too)
    const int lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const Stack stk{stack_mem + threadIdx.x, kDqBlock, kLdsStack, kp.gstack, kp.nslots,
                    blockIdx.x * kDqBlock + threadIdx.x};
    Counts cnt;
    for (int i = 0; i < kCounters; i++) cnt.c[i] = 0;
    cnt.m[0] = cnt.m[1] = cnt.m[2] = 0;
    cnt.q[0] = cnt.q[1] = cnt.q[2] = cnt.q[3] = 0;
    const DqStores st{reinterpret_cast<float4*>(kp.lv), reinterpret_cast<float4*>(kp.ev),
                      static_cast<uint32_t>(kp.fr.lv_max > 1 ? kp.fr.lv_max : 1), kp.ev_max};
    unsigned long long* const work = kp.work;
    const uint64_t total = kp.fr.total_samples;
    __shared__ LaneCold cold_mem[kDqBlock];
    Lane L(cold_mem[threadIdx.x]);
    L.state = ST_IDLE;
    L.c.nl = 0;
    cold_u(L.c.rr) = 0u;
    __syncthreads();
    bool exhausted = false;  // wave-uniform: no samples left for this wave
    uint64_t chunk_base = 0;
    int chunk_pos = 0, chunk_n = 0;
    bool global_done = false;
    uint32_t chunk_x397 = 0;
#if BDPT_EYE_SLOTS
    uint32_t chunk_seq = 0;
    if (lane == 0)
        for (int k = 0; k < BDPT_EYE_SLOTS; k++) wave_eye_slots()[k] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
#endif
    // idle lanes of helper waves take tasks before new samples; the others only above BDPT_DQ_HIGH
    const uint32_t take_at = wave >= 4u - BDPT_DQ_HELPER_WAVES ? 0u : static_cast<uint32_t>(BDPT_DQ_HIGH);
    const TravScene tsc = trav_scene(kp.sc);
    bool tracing = false, has_res = false, q_any = false;
    TravState ts{};
    RayInv ri{};
    int res = -1;
    float rt = 0.f, ru = 0.f, rv = 0.f;
    unsigned long long* const diag = kp.fr.diag;
    if (diag && lane == 0) gmin(diag + kDiagStart, __builtin_amdgcn_s_memrealtime());
    const uint64_t clock0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
        typedef const __attribute__((address_space(4))) DqParams* ConstP;
        uint64_t pa = (uint64_t)(ConstP)kpp;
        asm volatile("" : "+s"(pa));
        const DqParams* P = (const DqParams*)(ConstP)pa;
        // ---- task phase: idle lanes and owners with own tasks get work
        const uint64_t tp0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        for (int round = 0; round < BDPT_DQ_ROUNDS; round++) {
            const uint32_t pend = __hip_atomic_load(&cold_u(L.c.rr), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            {  // owners whose sample ended: its estimate to the framebuffer once its last task is done
                const bool fin = L.state == ST_FINWAIT && ((pend >> (16 * dq_buf(L.c))) & 0xffffu) == 0u;
                const uint64_t fm = __ballot(fin);
                if (fm) {
                    if (fin) {
                        L.c.nl = static_cast<int>(static_cast<uint32_t>(L.c.nl) & ~kFinWait);
                        finish<COUNT>(L, P->fr, P->fb, cnt);  // L.state = ST_IDLE
                    }
                    if (lane == __ffsll(static_cast<unsigned long long>(fm)) - 1)
                        atomicSub(&q.owners, static_cast<uint32_t>(__popcll(fm)));
                }
            }
            const bool own = L.state == ST_BACKLOG;
            const bool waiting = L.state == ST_FINWAIT;  // (may help meanwhile)
            const bool idle = L.state == ST_IDLE;
            if (!__ballot(own || idle || waiting)) break;
            const uint32_t buf_next = dq_buf(L.c) ^ 1u;
            const bool can_sample = idle && !exhausted && ((pend >> (16 * buf_next)) & 0xffffu) == 0u;
            const uint32_t fill = dq_load(q.tail) - dq_load(q.head);  // snapshot (policy only)
            const bool want = (idle && fill > 0u && (fill > take_at || !can_sample)) || (waiting && fill > 0u);
            uint32_t d = 0;
            bool got = false;
            const uint64_t wm = __ballot(want);
            if (wm) {  // pop up to popc(wm) descriptors
                const int leader = __ffsll(static_cast<unsigned long long>(wm)) - 1;
                uint32_t base = 0, k = 0;
                if (lane == leader) {
                    dq_lock(q);
                    base = q.head;
                    k = min(q.tail - base, static_cast<uint32_t>(__popcll(wm)));
                    q.head = base + k;
                }
                base = __shfl(base, leader);
                k = __shfl(k, leader);
                const uint32_t rank = __popcll(wm & ((1ull << lane) - 1ull));
                if (want && rank < k) {
                    d = q.e[(base + rank) & (kDqRing - 1)];
                    got = true;
                }
                if (lane == leader) dq_unlock(q);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // the records behind the descriptors
            }
            if (own) got = dq_own_next(L.c, d);
            bool progressed = got;
            if (got) {
                if (COUNT) cnt.q[own ? 3 : 1]++;
                if (!own) L.c.prim_tri = static_cast<int>(d);  // (an owner's prim_tri is its primary hit)
                if (!dq_task<COUNT>(L, d, P->sc, P->fr, st, cnt)) {  // nothing to trace: done at once
                    if (COUNT) cnt.q[2]++;
                    if (!(d & kDescSelf)) {
                        atomicSub(&cold_u(cold_mem[(d >> 2) & 0xffu].rr), 1u << (16 * ((d >> 10) & 1u)));
                        L.state = waiting ? ST_FINWAIT : ST_IDLE;
                    }
                }
            } else if (own) {  // backlog done: the walk resumes in the next shading step
                L.state = ST_RESUME;
                progressed = true;
            }
            // new samples for idle lanes without a task, from the wave's 64-sample chunk
            const bool ws = can_sample && !got && L.state == ST_IDLE;
            uint64_t sm = __ballot(ws);
            while (sm && !exhausted) {
                if (chunk_pos >= chunk_n) {
                    if (global_done) {
                        exhausted = true;
                        break;
                    }
                    unsigned long long b = 0;
                    if (lane == 0) b = gadd(work, 64ull);
                    b = __shfl(b, 0);
                    if (b >= total) {
                        exhausted = true;
                        break;
                    }
                    chunk_base = b;
                    chunk_n = static_cast<int>(total - b < 64 ? total - b : 64);
                    chunk_pos = 0;
                    global_done = b + 64 >= total;
                    if (global_done && diag && lane == 0) diag[kDiagLastClaim] = __builtin_amdgcn_s_memrealtime();
                    int px;
                    chunk_x397 = mt_x397(sample_seed(b + lane, P->fr, px));
#if BDPT_EYE_SLOTS
                    const int cpx = __shfl(px, 0);
                    if (lane == 0)
                        eye_slot_reset(P->fb, static_cast<int>(chunk_seq % BDPT_EYE_SLOTS), P->fr.spp % 64 == 0 ? cpx : -1);
                    chunk_seq++;
#endif
                }
                const int m = min(__popcll(sm), chunk_n - chunk_pos);
                const int rank = __popcll(sm & ((1ull << lane) - 1ull));
                const uint32_t x397 = __shfl(chunk_x397, (chunk_pos + rank) & 63);
                const bool mine = ((sm >> lane) & 1ull) && rank < m;
                if (mine) {
                    L.c.nl = static_cast<int>(buf_next << 8);  // the other record buffer, nothing stored
                    start_sample<true>(L, chunk_base + chunk_pos + rank, P->fr, x397);
                    progressed = true;
                }
                if (lane == 0 && m > 0) atomicAdd(&q.owners, static_cast<uint32_t>(m));
                chunk_pos += m;
                sm &= ~__ballot(mine);
            }
            if (!__ballot(progressed)) break;
        }
        if (COUNT && (threadIdx.x & 63) == 0) cnt.q[0] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - tp0);
        const bool busy = L.state != ST_IDLE;
        if (!__ballot(busy)) {
            // nothing for this wave now: done once no sample is left, the ring is
            // empty and no owner of the block can push more; else wait for tasks
            if (exhausted && dq_load(q.owners) == 0u && dq_load(q.tail) == dq_load(q.head)) break;
            __builtin_amdgcn_s_sleep(2);
            continue;
        }
        // ---- walk (the overlapped schedule of bdpt_kernels.hip)
        // (an owner still in ST_BACKLOG, when the task phase ran out of rounds, waits for the next one)
        if (busy && !tracing && !has_res && L.state != ST_BACKLOG && L.state != ST_FINWAIT) {
            q_any = dq_is_shadow(L.state);
            if (COUNT && L.state != ST_DEFER && L.state != ST_RESUME) cnt.c[q_any ? 1 : 0]++;
            ri = ray_inv(L.ray, dq_cull_near(L));
            if (L.state == ST_DEFER || L.state == ST_RESUME) {
                res = -1;
                has_res = true;
            } else if (L.ray.min_t > L.ray.max_t) {
                res = -1, rt = L.ray.max_t, ru = rv = 0.f;
                has_res = true;
            } else if (FULL || !ri.fast || far_origin(P->sc, L.ray.o)) {
                const TravResult r = traverse_binary<COUNT, Stack>(P->sc, L.ray, q_any, false, stk);
                if (COUNT) cnt.c[2] += r.nodes, cnt.c[3] += r.tris, cnt.c[15] += r.exact;
                res = r.best, rt = r.t, ru = r.u, rv = r.v;
                has_res = true;
            } else {
                ts = trav_begin(tsc, L.ray);
                tracing = true;
                if (root_in_lds && !walk_begin_lds<COUNT, SLACK>(root_lds, L.ray, ri, q_any, ts, stk, cnt)) {
                    res = -1, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                    tracing = false;
                    has_res = true;
                }
            }
        }
        if (!__ballot(tracing || has_res)) {  // only owners waiting on their tasks (or own tasks next round)
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        const uint64_t c0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        for (;;) {
            const uint64_t tr = __ballot(tracing);
            if (!tr) break;
            const uint64_t ready = __ballot(has_res);
            if (__popcll(ready) >= BDPT_SHADE_READY) break;
            const bool at_leaf = (ts.link & kLeafBit) != 0;
            const uint64_t lv = __ballot(tracing && at_leaf);
            const bool do_leaf = __popcll(lv) * 4 >= __popcll(tr & ~lv) * BDPT_TRAV_SPLIT;
            bool fin = tracing && at_leaf == do_leaf && trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
#pragma unroll
            for (int k = 0; k < BDPT_WALK_UNROLL; k++)
                if (!do_leaf && tracing && !fin && !(ts.link & kLeafBit))
                    fin = trav_step<COUNT, SLACK>(tsc, L.ray, ri, q_any, ts, stk, cnt);
            if (fin) {
                res = ts.best, rt = ts.best_t, ru = ts.best_u, rv = ts.best_v;
                tracing = false;
                has_res = true;
            }
        }
        const uint64_t c1 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
        if (has_res) {
            has_res = false;
            const uint64_t r0 = COUNT ? __builtin_amdgcn_s_memtime() : 0;
            const uint32_t act = dq_resolve<COUNT>(L, res, rt, ru, rv, P->sc, P->fr, P->fb, cold_mem, cnt);
            if (COUNT && first_active_lane()) cnt.c[20] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - r0);
            if (act != A_DONE) dq_advance<COUNT>(L, act, P->sc, P->fr, P->fb, st, q, cnt);
        }
        if (COUNT && first_active_lane()) {
            const uint64_t c2 = __builtin_amdgcn_s_memtime();
            cnt.c[12] += static_cast<uint32_t>(c1 - c0);
            cnt.c[13] += static_cast<uint32_t>(c2 - c1);
        }
    }
#if BDPT_EYE_SLOTS
    if (lane == 0)
        for (int k = 0; k < BDPT_EYE_SLOTS; k++) eye_slot_reset(kp.fb, k, -1);
#endif
    if (diag && lane == 0) gmax(diag + kDiagEnd, __builtin_amdgcn_s_memrealtime());
    if (COUNT) {
        if (lane == 0) cnt.c[14] += static_cast<uint32_t>(__builtin_amdgcn_s_memtime() - clock0);
        flush_counts(cnt, kp.counters);
    }
}

}  // namespace dev

// ------------------------------------------------------------ host launchers
size_t frame_params_bytes_dq() { return sizeof(dev::DqParams); }

hipError_t launch_frame_dq(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, float* evbuf,
                           uint32_t ev_max, uint2* gstack, uint32_t nslots, unsigned long long* work,
                           unsigned long long* counters, int grid, hipStream_t stream, void* dparams) {
    const bool full = (fr.flags & 2u) != 0, count = (fr.flags & 1u) != 0, slack = sc.node_slack != 0;
    const dev::DqParams host{sc, fr, fb, lvbuf, evbuf, gstack, nslots, ev_max, work, counters};
    hipError_t e = hipMemcpyAsync(dparams, &host, sizeof(host), hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    const dev::DqParams* kp = static_cast<const dev::DqParams*>(dparams);
    const dim3 g(grid), b(dev::kDqBlock);
    const size_t lds = 4 * static_cast<size_t>(sc.lds_words);
    if (full && count) hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<true, true, true>), g, b, lds, stream, kp);
    else if (full) hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<true, false, true>), g, b, lds, stream, kp);
    else if (count && slack) hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<false, true, true>), g, b, lds, stream, kp);
    else if (count) hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<false, true, false>), g, b, lds, stream, kp);
    else if (slack) hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<false, false, true>), g, b, lds, stream, kp);
    else hipLaunchKernelGGL((dev::bdpt_frame_kernel_dq<false, false, false>), g, b, lds, stream, kp);
    return hipGetLastError();
}

int frame_kernel_lds_stack_dq() { return dev::kLdsStack; }

int frame_kernel_blocks_per_cu_dq(size_t dyn_lds) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, dev::bdpt_frame_kernel_dq<false, false, false>,
                                                     dev::kDqBlock, dyn_lds) != hipSuccess ||
        n <= 0)
        n = 1;
    return n;
}

}  // namespace bdpt
