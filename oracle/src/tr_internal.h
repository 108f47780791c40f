/* TEST INFRASTRUCTURE (oracle) — internal types shared by tr_scene.c / tr_bdpt.c. */
#ifndef TR_INTERNAL_H
#define TR_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "oracle.h"
#include "tr_mathf.h"

/* reference src/core/platform.h:51-57 */
#define TR_PI 3.14159265358979323846f
#define TR_INV_PI 0.31830988618379067154f
#define TR_INV_TWOPI 0.15915494309189533577f
#define TR_EPSILON 1e-8f

typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;
typedef struct { float m[4][4]; } m4; /* column-major like glm: m[col][row] */

/* BSDF kinds, chosen by MTL illum (reference renderer.cpp:258-271). */
enum { TRB_NULL = 0, TRB_DIFFUSE, TRB_MIRROR, TRB_GLASS, TRB_MIXTURE, TRB_PHONG };
/* reference src/core/core.h:261-300 */
#define TRT_NULL 0x1u
#define TRT_DIFFUSE_REFL 0x2u
#define TRT_GLOSSY_REFL 0x8u
#define TRT_DELTA_REFL 0x20u
#define TRT_DELTA_TRANS 0x40u
#define TRT_DELTA (TRT_NULL | TRT_DELTA_REFL | TRT_DELTA_TRANS)

typedef struct {
    char name[128];
    int illum;
    float Kd[3], Ks[3], Ke[3], Tf[3], Ns, Ni;
    int has_diffuse_tex, has_specular_tex;
} tro_material;

typedef struct {
    int kind;
    unsigned type;
    v3 kd, ks, tf, emission;
    float exponent, ior, scale, specw;
} tro_bsdf;

typedef struct {
    int shape;
    float area;
    v3 radiance;
    int ncdf;
    float* cdf; /* ncdf = faces + 1 */
    v3 center;    /* worldData.shapesCenter (renderer.cpp:295-304): mean of the shape's corners */
    float radius; /* Scene::getShapeRadius (renderer.cpp:349-353): AABB max.x - center.x */
} tro_emitter;

typedef struct {
    float bmin[3], bmax[3];
    uint32_t start, nprims, right_offset;
} tro_node;

struct tro_scene {
    /* triangles in (shape, face) order, as tinyobj emits them */
    int ntri;
    float* tv;     /* [ntri][9] positions v0 v1 v2 */
    float* tn;     /* [ntri][9] normals n0 n1 n2   */
    int* tshape;   /* shape id                      */
    int* tprim;    /* face index within the shape   */
    int* tmat;     /* material id of the face       */
    int nshapes;
    int* shape_first; /* first triangle of each shape */
    int* shape_count;
    int* shape_emitter; /* emitter index for the shape, or -1 */
    int nmat;
    tro_material* mats;
    tro_bsdf* bsdf;
    int nemit;
    tro_emitter* emit;
    /* BVH: build_prims order (triangle ids) and flat preorder nodes */
    int* order;
    int nnodes;
    tro_node* nodes;
    int max_depth;
};

/* glm-order vector helpers (reference externals/glm/glm/detail/func_geometric.inl) */
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* dot: tmp = a*b; (tmp.x + tmp.y) + tmp.z  (func_geometric.inl:59) */
static inline float vdot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
/* cross (func_geometric.inl:74-83) */
static inline v3 vcross(v3 x, v3 y) {
    return V3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}
float tr_sqrtf(float x);
/* normalize: v * (1 / sqrt(dot(v, v)))  (func_geometric.inl:94, func_exponential.inl:138) */
static inline v3 vnormalize(v3 v) { return vscale(v, 1.f / tr_sqrtf(vdot(v, v))); }
static inline int veq0(v3 v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }

void tr_camera_mats(const tro_params* p, m4* w2c, m4* c2w, m4* c2clip, m4* ndc2screen, float* angle, float* aspect,
                    v3* fwd, float* vnear);
v4 tr_m4v4(const m4* m, v4 v);

#endif
