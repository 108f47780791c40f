// Per-function entry points of the BDPT hot path, batched on the device: the
// BSDF plugin contract (BSDF::eval / pdf / sample, reference
// src/core/core.h:308-310, src/bsdfs/{diffuse,perfectmirror,glass,mixture,phong}.h),
// GlassBSDF::FresnelDielectric (glass.h:40-53), rayTriangleIntersect
// (core.h:379-400), AcceleratorBVH::intersect and the occlusion query
// (accel.h:125-172, bvh.h:259-352) and BDPTIntegrator::splatToImagePlane
// (bdpt.h:485-496). Each kernel runs exactly the device function the frame
// kernels call, one element per lane, so the parity tests can pin every piece
// of the path against the reference's own functions.
#include <hip/hip_runtime.h>

#include "bdpt_path.hpp"

namespace bdpt {
namespace dev {

constexpr int kKatBlock = 64;

// mode 0: eval (f * cos) -> out[3]; 1: pdf -> out[1]; 2: sample -> out f[3], wi[3], pdf
__global__ __launch_bounds__(kKatBlock) void bsdf_kat_kernel(DevScene sc, int mode, int64_t n,
                                                            const int32_t* __restrict__ mat,
                                                            const float* __restrict__ wo, const float* __restrict__ x,
                                                            float* __restrict__ out) {
    scene_tables_to_lds(sc);
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kKatBlock + threadIdx.x;
    if (i >= n) return;
    const int m = mat[i];
    if (m < 0 || m >= sc.nbsdf) return;
    const BsdfRecord& b = bsdf_of(sc, m);
    const f3 o = mk(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
    if (mode == 0) {
        const f3 f = bsdf_eval(b, mk(x[3 * i], x[3 * i + 1], x[3 * i + 2]), o);
        out[3 * i] = f.x, out[3 * i + 1] = f.y, out[3 * i + 2] = f.z;
    } else if (mode == 1) {
        out[i] = bsdf_pdf(b, mk(x[3 * i], x[3 * i + 1], x[3 * i + 2]), o);
    } else {
        f3 wi;
        float pdf;
        const f3 f = bsdf_sample(b, o, F2{x[2 * i], x[2 * i + 1]}, wi, pdf);
        float* r = out + 7 * i;
        r[0] = f.x, r[1] = f.y, r[2] = f.z, r[3] = wi.x, r[4] = wi.y, r[5] = wi.z, r[6] = pdf;
    }
}

// in: (eta_i, eta_t, cos_i, cos_t) per element
__global__ __launch_bounds__(kKatBlock) void fresnel_kat_kernel(int64_t n, const float* __restrict__ in,
                                                               float* __restrict__ out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kKatBlock + threadIdx.x;
    if (i >= n) return;
    const float* q = in + 4 * i;
    out[i] = fresnel_dielectric(q[0], q[1], q[2], q[3]);
}

// rayTriangleIntersect (no t > 1e-3 acceptance: that is accel.h:43's): in rays
// (o, d, min_t, max_t) and vertices (v0, v1, v2); out (hit, t, u, v).
__global__ __launch_bounds__(kKatBlock) void triangle_kat_kernel(int64_t n, const float* __restrict__ rays,
                                                                const float* __restrict__ verts,
                                                                float* __restrict__ out) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kKatBlock + threadIdx.x;
    if (i >= n) return;
    const float* r = rays + 8 * i;
    const float* v = verts + 9 * i;
    const Ray ray{mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], r[7]};
    const f3 v0 = mk(v[0], v[1], v[2]), v1 = mk(v[3], v[4], v[5]), v2 = mk(v[6], v[7], v[8]);
    float t = 0.f, u = 0.f, w = 0.f;
    const bool hit = tri_test_raw(v0, v1 - v0, v2 - v0, ray, t, u, w);
    float* o = out + 4 * i;
    o[0] = hit ? 1.f : 0.f, o[1] = t, o[2] = u, o[3] = w;
}

// Closest hit (AcceleratorBVH::intersect) or occlusion (bvh->getIntersection(ray,
// &info, true), as visibilityQuery calls it) through the product traversal.
// out per ray (20 words, bdpt_hit): hit (int bits), t, u, v, shapeID, primID, matID (int bits),
// p[3], frameNs.n[3], frameNg.n[3], wo[3], leaf-order triangle index (int bits).
// nrm (optional, 3 per ray): the normal of the surface the ray leaves, for the
// frame kernels' near-cull rule (cull_near_for: a zero normal = a camera
// origin), otri (optional) the triangle of that surface, whose graze code widens
// the threshold as in the frames; without nrm no box is near-culled.
__global__ __launch_bounds__(kKatBlock) void intersect_kat_kernel(DevScene sc, int64_t n, int occlusion,
                                                                 const float* __restrict__ rays,
                                                                 const float* __restrict__ nrm,
                                                                 const int32_t* __restrict__ otri,
                                                                 uint2* __restrict__ gstack, uint32_t nslots,
                                                                 float* __restrict__ out) {
    __shared__ uint2 stack_mem[kLdsStack * kKatBlock];
    scene_tables_to_lds(sc);
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kKatBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t slot = static_cast<uint32_t>(i % nslots);
    const Stack stk{stack_mem + threadIdx.x, kKatBlock, kLdsStack, gstack, nslots, slot};
    const float* r = rays + 8 * i;
    const Ray ray{mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6], r[7]};
    Counts cnt;
    float t = 0.f, u = 0.f, v = 0.f;
    float near = kNoCullNear;
    if (nrm) {
        const f3 sn = mk(nrm[3 * i], nrm[3 * i + 1], nrm[3 * i + 2]);
        const bool camera = sn.x == 0.f && sn.y == 0.f && sn.z == 0.f;
        const int ot = otri ? otri[i] : -1;
        const int code = ot >= 0 ? __float_as_int(gld4(sc.shade + kShadeStride * static_cast<size_t>(ot) + 1).w) : 0;
        near = (camera || !graze_exempt(ray.d, sn, code)) ? kCullNear : kNoCullNear;
    }
    const int res = traverse<false, false>(sc, ray, occlusion != 0, stk, t, u, v, cnt, near);
    float* o = out + 20 * i;
    for (int k = 0; k < 20; k++) o[k] = 0.f;
    if (occlusion) {
        o[0] = __int_as_float(res >= 0 ? 1 : 0);
        return;
    }
    const bool hit = res >= 0 && t <= ray.max_t && t >= ray.min_t;  // accel.h:133
    o[1] = t;
    if (!hit) return;
    Hit h;
    shade_hit(sc, res, u, v, t, ray.d, h);
    const float4* sh = sc.shade + kShadeStride * static_cast<size_t>(res);
    const f3 v0 = xyz(gld4(sc.tri + 3 * static_cast<size_t>(res))), v1 = xyz(gld4(sh + 3)), v2 = xyz(gld4(sh + 4));
    const f3 ng = normalize(cross(v1 - v0, v2 - v0));
    o[0] = __int_as_float(1), o[2] = u, o[3] = v;
    o[4] = __int_as_float(shape_id(h.shape)), o[5] = __int_as_float(__float_as_int(gld4(sh + 2).w)), o[6] = __int_as_float(h.mat);
    o[7] = h.p.x, o[8] = h.p.y, o[9] = h.p.z;
    o[10] = h.n.x, o[11] = h.n.y, o[12] = h.n.z;
    o[13] = ng.x, o[14] = ng.y, o[15] = ng.z;
    o[16] = h.wo.x, o[17] = h.wo.y, o[18] = h.wo.z;
    o[19] = __int_as_float(res);
}

__global__ __launch_bounds__(kKatBlock) void splat_kat_kernel(DevFrame fr, int64_t n, const float* __restrict__ p,
                                                             int32_t* __restrict__ xy) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kKatBlock + threadIdx.x;
    if (i >= n) return;
    int x, y;
    splat_pixel(fr.cam, mk(p[3 * i], p[3 * i + 1], p[3 * i + 2]), x, y);
    xy[2 * i] = x, xy[2 * i + 1] = y;
}

}  // namespace dev

static dim3 kat_grid(int64_t n) { return dim3(static_cast<unsigned>((n + dev::kKatBlock - 1) / dev::kKatBlock)); }

hipError_t launch_bsdf_kat(const dev::DevScene& sc, int mode, int64_t n, const int32_t* mat, const float* wo,
                           const float* x, float* out, hipStream_t st) {
    if (n > 0)
        hipLaunchKernelGGL(dev::bsdf_kat_kernel, kat_grid(n), dim3(dev::kKatBlock), 4 * static_cast<size_t>(sc.lds_words),
                           st, sc, mode, n, mat, wo, x, out);
    return hipGetLastError();
}
hipError_t launch_fresnel_kat(int64_t n, const float* in, float* out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(dev::fresnel_kat_kernel, kat_grid(n), dim3(dev::kKatBlock), 0, st, n, in, out);
    return hipGetLastError();
}
hipError_t launch_triangle_kat(int64_t n, const float* rays, const float* verts, float* out, hipStream_t st) {
    if (n > 0)
        hipLaunchKernelGGL(dev::triangle_kat_kernel, kat_grid(n), dim3(dev::kKatBlock), 0, st, n, rays, verts, out);
    return hipGetLastError();
}
hipError_t launch_intersect_kat(const dev::DevScene& sc, int64_t n, int occlusion, const float* rays, const float* nrm,
                                const int32_t* otri, uint2* gstack, uint32_t nslots, float* out, hipStream_t st) {
    if (n > 0)
        hipLaunchKernelGGL(dev::intersect_kat_kernel, kat_grid(n), dim3(dev::kKatBlock),
                           4 * static_cast<size_t>(sc.lds_words), st, sc, n, occlusion, rays, nrm, otri, gstack,
                           nslots, out);
    return hipGetLastError();
}
hipError_t launch_splat_kat(const dev::DevFrame& fr, int64_t n, const float* p, int32_t* xy, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(dev::splat_kat_kernel, kat_grid(n), dim3(dev::kKatBlock), 0, st, fr, n, p, xy);
    return hipGetLastError();
}

}  // namespace bdpt
