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
// under a binned-SAH tree collapsed to 4-wide nodes. Interior boxes are exact
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

}  // namespace bdpt
