// 4-wide traversal hierarchy over the reference's BVH leaves.
//
// The reference (externals/bvh.h:259-352) visits every node whose box passes
// its slab test (BBox::intersect, bvh.h:33-69) and never culls by distance, so
// a leaf's triangles are tested iff the leaf box and all of its ancestors pass.
// Every Fast-BVH box is the exact union of its primitives' boxes (bvh.h:176-182),
// so a child box lies inside its parent box, and for a ray whose direction has
// no zero component the slab test is monotone under box growth: each per-axis
// t = (l - o) / d is a monotone function of l after rounding, so a child that
// passes implies a parent that passes. Hence for such rays the reference tests
// exactly the leaves whose own box passes — independent of the tree above them.
//
// That frees the hierarchy ABOVE the leaves: this builder groups the
// reference leaves (kept as units: same triangles, same order, same exact box)
// under a binned-SAH tree collapsed to 4-wide nodes (children picked by SAH
// dynamic programming, wide_bvh.cpp DpCollapse). Interior boxes are exact
// unions of leaf boxes and are tested conservatively (an ambiguous fast test
// counts as a hit); the leaf boxes are tested exactly. Rays with a zero or
// non-finite reciprocal direction (where 0/0 = NaN breaks monotonicity) keep
// the reference's binary tree (DeviceLayout::nodes).
//
// Node record, 8 float4 (128 B) per 4-wide node, children in SoA order:
//   q0 lo.x[4]  q1 hi.x[4]  q2 lo.y[4]  q3 hi.y[4]  q4 lo.z[4]  q5 hi.z[4]
//   q6 link[4] (uint bits; kLeafBit | start << 3 | count for a reference leaf,
//               a node index otherwise, kEmptyLink for an unused slot)
//   q7 unused
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "bdpt_types.h"

namespace bdpt {

struct FlatNode;

constexpr int kWideArity = 4;
constexpr uint32_t kEmptyLink = 0xffffffffu;

struct WideBvh {
    std::vector<float4_t> nodes;  // 8 per node
    uint32_t root_link = 0;       // a node index, or a leaf link when the whole scene is one leaf
    int max_stack = 0;            // worst-case traversal stack entries (sum of (arity-1) on a path)
    int depth = 0;
    int64_t leaves = 0;
};

// Builds the hierarchy over the leaves of the reference's flat preorder tree.
bool build_wide_bvh(const std::vector<FlatNode>& flat, WideBvh& out, std::string& err);

// The default traversal hierarchy: a binned-SAH 4-wide tree over single
// triangles (leaves of up to kTriLeafMax, closed by the SAH), boxes padded by
// pad_rel x the scene diagonal. A triangle is a candidate of the reference's
// search iff its REFERENCE leaf box passes BBox::intersect (see above: for rays
// without a zero direction component that is independent of the tree above the
// leaves); the device checks that box exactly, but only for a triangle hit that
// would become the result (or end an occlusion query). Everything else — node
// boxes, leaf grouping, order — is free, so the tree is built for speed:
// against the reference-leaf tree it halves the walk steps and cuts triangle
// tests ~4x on the Cornell scenes (tools/trav_sim.cpp).
//   tri:      3 float4 per triangle in this tree's leaf order: (v0, reference
//             index bits) (e1, reference leaf id bits) (e2, 0)
//   leaf_box: 2 float4 per reference leaf: (lo, 0) (hi, 0) — infinite when the
//             whole reference tree is one leaf (then no box is tested)
constexpr int kTriLeafMax = 4;
constexpr float kTriBoxPad = 1e-4f;  // x scene diagonal: the hit-point tolerance of the culling
struct TriWideBvh {
    WideBvh bvh;
    std::vector<float4_t> tri;
    std::vector<float4_t> leaf_box;
    float pad = 0.f;
};
bool build_wide_bvh_tris(const std::vector<FlatNode>& flat, const std::vector<float4_t>& tri,
                         const std::vector<float4_t>& shade, float pad_rel, TriWideBvh& out, std::string& err);

// Compressed 64-byte node records (4 float4) of the same tree, for the
// BDPT_QNODES=1 kernels: each child box as 8-bit offsets on a per-node,
// per-axis grid of 2^e steps from the node's box minimum, rounded outward, so
// the decoded box contains the exact one (the difference is computed in
// double; its rounding, ~2^-53 of a coordinate, is far inside kTriBoxPad).
//   q0 = (org.x, org.y, org.z, (e_x + 127) | (e_y + 127) << 8 | (e_z + 127) << 16)
//   q1 = (lo.x bytes, hi.x bytes, lo.y bytes, hi.y bytes)   byte c = child c
//   q2 = (lo.z bytes, hi.z bytes, 0, 0)
//   q3 = link[4] (as in the 128-byte record)
// A child bound is org + q * 2^e; the device forms its slab distance as
// fma(q, 2^e / d, (org - o) / d). e is kept in [kQuantExpMin, kQuantExpMax] so
// 2^e / d stays a normal float for |1/d| in [2^-40, 2^96] (RayInv::fast);
// false when a node needs a larger grid (non-finite or > 2.7e8-wide boxes).
constexpr int kQuantExpMin = -80, kQuantExpMax = 20;
bool quantize_wide_nodes(const std::vector<float4_t>& wnodes, std::vector<float4_t>& qnodes);

}  // namespace bdpt
