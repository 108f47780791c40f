// Host-side scene ingest for the MI355X BDPT path.
//
// Replaces Scene::load (reference src/core/renderer.cpp:235-315): OBJ/MTL
// parsing with tinyobjloader v1.2.0 semantics (the reference's vendored
// externals/tiny_obj_loader.h, real_t = float, triangulate = true), BSDF
// selection by MTL illum, emitters with per-face area CDFs, and the Fast-BVH
// build (externals/bvh.h:147-247). Triangle order and BVH topology are kept
// bit-identical to the reference because they decide closest-hit ties.
//
// The result is then flattened into the HBM layout the HIP kernels read
// (see DeviceLayout / DESIGN.md "Data layout in HBM").
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "bdpt_amd.h"
#include "bdpt_types.h"

namespace bdpt {

struct Material {
    std::string name;
    int illum = 0;
    float Kd[3] = {0, 0, 0}, Ks[3] = {0, 0, 0}, Ke[3] = {0, 0, 0}, Tf[3] = {0, 0, 0};
    float Ns = 1.f, Ni = 1.f;  // tinyobj InitMaterial defaults (tiny_obj_loader.h:964-999)
    bool has_texture = false;
};

struct Emitter {
    int shape = -1;
    float area = 0.f;
    float radiance[3] = {0, 0, 0};
    std::vector<float> cdf;  // normalized face-area CDF, faces + 1 entries
};

struct FlatNode {  // BVHFlatNode (bvh.h:102-105) without the redundant extent
    float bmin[3], bmax[3];
    uint32_t start, nprims, right_offset;
};

struct HostScene {
    // Triangles in tinyobj (shape, face) order.
    std::vector<float> pos;  // [ntri][9]
    std::vector<float> nrm;  // [ntri][9]
    std::vector<int32_t> tri_shape, tri_prim, tri_mat;
    std::vector<int32_t> shape_first, shape_count, shape_emitter;
    std::vector<Material> materials;
    std::vector<BsdfRecord> bsdfs;
    std::vector<Emitter> emitters;
    // Fast-BVH result: build_prims order and preorder flat nodes.
    std::vector<int32_t> order;
    std::vector<FlatNode> nodes;
    int max_depth = 0;

    size_t num_triangles() const { return tri_shape.size(); }
};

// Returns false and sets `err` on failure (missing file, bad face index, face
// without normal or material, bitmap textures, null BSDF on an emitter test).
bool load_obj_scene(const std::string& obj_path, HostScene& out, std::string& err);

// The same HostScene from the caller's in-memory Scene (core.h:352-358) handed
// over as a bdpt_scene_desc: triangles, materials with their constructed
// constants, emitters with their CDFs and the flattened Fast-BVH, validated.
bool load_desc_scene(const bdpt_scene_desc& desc, HostScene& out, std::string& err);

// Flattened arrays uploaded to HBM (layouts documented in bdpt_types.h).
struct DeviceLayout {
    std::vector<float4_t> tri;      // 3 per triangle, BVH leaf order
    std::vector<float4_t> shade;    // 5 per triangle, BVH leaf order
    std::vector<float4_t> nodes;    // 4 per interior node (the reference's binary tree)
    uint32_t root_link = 0;
    std::vector<float4_t> wnodes;   // 8 per 4-wide traversal node (wide_bvh.hpp)
    std::vector<float4_t> qnodes;   // 4 per node: the same tree compressed (quantize_wide_nodes)
    bool q_ok = false;              // qnodes built (triangle tree, every node on the grid)
    uint32_t wroot_link = 0;
    int wmax_stack = 0, wdepth = 0;
    int64_t wleaves = 0;
    std::vector<float4_t> wtri;     // 3 per triangle in the traversal tree's leaf order (wide_bvh.hpp)
    std::vector<float4_t> lbox;     // 2 per reference leaf: its exact box
    bool tri_tree = true;           // false: traversal leaves = the reference leaves (BDPT_TRAV_TREE=refleaf)
    std::vector<BsdfRecord> bsdfs;
    std::vector<EmitterRecord> emitters;
    std::vector<float4_t> emit_tri; // 5 per emitter face, shape face order
    std::vector<float> emit_cdf;
    std::vector<int32_t> shape_emitter;
};

bool build_device_layout(const HostScene& s, DeviceLayout& out, std::string& err);

// Sets the thread-local message of bdpt_last_error() and returns `code`.
int set_error(int code, const std::string& msg);

// Integrator::save's EXR (utils.h:95-156 via tinyexr): half-float B, G, R
// planes, uncompressed scanlines. rgb = W*H*3 floats, pixel-major, row 0 = top.
bool encode_exr_bgr_half(const float* rgb, int W, int H, std::vector<unsigned char>& out, std::string& err);

// Camera constants (renderer.cpp:140-153, bdpt.h:49-54, :485-489), GLM 0.9.9
// operation order.
void camera_constants(const float eye[3], const float at[3], const float up[3], float fov, int width, int height,
                      CameraConstants& out);

}  // namespace bdpt
