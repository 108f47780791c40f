// Plain-old-data records shared by the host ingest and the HIP kernels.
//
// HBM layout (all arrays 16-byte aligned, read through float4 loads):
//   tri[3*i + c]   (v0, 0), (v1 - v0, 0), (v2 - v0, 0)     triangle i in BVH leaf order; the
//                                                            edges rounded as the reference's test forms them
//   shade[5*i + c] c=0..2: (n_c.x, n_c.y, n_c.z, id_c)       id_0 = matID, id_1 = shapeID,
//                                                            id_2 = primID (int bits)
//                  c=3,4: (v1, 0), (v2, 0)                   for the hit point of a closest hit
//     (host layout; the device copy has kShadeStride float4 per triangle: the
//      same five, then (v0, 0) and padding — one 128-byte line per closest hit)
//   nodes[4*j + q] interior node j (2-wide, both child boxes inline):
//       q0 = c0.min.xyz, c0.max.x   q1 = c0.max.yz, c1.min.xy
//       q2 = c1.min.z, c1.max.xyz   q3 = (link0, link1, 0, 0) as uint bits
//     link: bit 31 set -> leaf, start = (link >> 3) & 0x0fffffff, count = link & 7
//           otherwise  -> index of the child's interior record
//   emit_tri[5*f + q] emitter faces in shape face order (v0 v1 v2 n0 n1 n2 packed)
#pragma once

#include <cstdint>

namespace bdpt {

struct alignas(16) float4_t {
    float x, y, z, w;
};

enum BsdfKind : int32_t {
    BSDF_NULL = 0,     // illum 5: the reference leaves a null BSDF (renderer.cpp:268)
    BSDF_DIFFUSE = 1,  // illum 7: src/bsdfs/diffuse.h
    BSDF_MIRROR = 2,   // illum 3: src/bsdfs/perfectmirror.h
    BSDF_GLASS = 3,    // illum 6: src/bsdfs/glass.h
    BSDF_MIXTURE = 4,  // illum 8: src/bsdfs/mixture.h
    BSDF_PHONG = 5,    // any other illum: src/bsdfs/phong.h
};

// BSDF::EBSDFType bits (reference src/core/core.h:261-295).
constexpr uint32_t kTypeNull = 0x1u, kTypeDiffuseRefl = 0x2u, kTypeGlossyRefl = 0x8u, kTypeDeltaRefl = 0x20u,
                   kTypeDeltaTrans = 0x40u;
constexpr uint32_t kTypeDelta = kTypeNull | kTypeDeltaRefl | kTypeDeltaTrans;

struct BsdfRecord {
    int32_t kind;
    uint32_t type;
    float kd[3], ks[3], tf[3], emission[3];
    float exponent, ior, scale, specw;
};

struct EmitterRecord {
    int32_t shape;
    int32_t nfaces;
    int32_t face_offset;  // into emit_tri (faces)
    int32_t cdf_offset;   // into emit_cdf (nfaces + 1 entries)
    float area;
    float radiance[3];
    // The emitter as a sphere, for DirectIntegrator (direct.h): the shape's corner
    // mean (renderer.cpp:295-304) and AABB max.x - center.x (renderer.cpp:349-353).
    float center[3];
    float radius;
};

struct CameraConstants {
    float w2c[16], c2w[16], c2clip[16], ndc2screen[16];  // column-major (glm)
    float invW, invH, angle, aspect;
    float fwd[3];
    float vnear;
};

// Device shade records: 8 float4 (128 B, line aligned) holding the host record's
// five plus v0 at slot 5, so shading a closest hit reads one cache line instead
// of the 80-byte record (often split over two lines) and v0 from the tri array;
// 5 = the host layout uploaded as is.
#ifndef BDPT_SHADE_WIDE
#define BDPT_SHADE_WIDE 1
#endif
constexpr int kShadeStride = BDPT_SHADE_WIDE ? 8 : 5;
constexpr int kShadeV0 = 5;  // slot of (v0, 0) in a wide record

constexpr uint32_t kLeafBit = 0x80000000u;
// Words per lane slot of the BDPT megakernel's MT19937 ring (DevScene::mt_ring):
// the 624-word ring and the generate-ahead cursor (bdpt_device.hpp, mt_ring_ahead).
constexpr uint32_t kMtRingSlotWords = 640;
// Words per lane slot of the Russian-roulette continuation records (DevFrame::park;
// bdpt_kernels.hip, park_save); the list of parked slots follows the records.
constexpr uint32_t kParkSlotWords = 64;
inline uint32_t make_leaf_link(uint32_t start, uint32_t count) { return kLeafBit | (start << 3) | count; }

}  // namespace bdpt
