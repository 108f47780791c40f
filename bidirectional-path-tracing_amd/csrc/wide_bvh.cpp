// Binned-SAH 4-wide hierarchy over the reference's BVH leaves (see wide_bvh.hpp).
#include "wide_bvh.hpp"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>

#include "scene.hpp"

namespace bdpt {
namespace {

struct Box {
    float lo[3], hi[3];
    void clear() {
        for (int a = 0; a < 3; a++) lo[a] = __builtin_inff(), hi[a] = -__builtin_inff();
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], b.lo[a]), hi[a] = std::max(hi[a], b.hi[a]);
    }
    double area() const {
        const double x = std::max(0.0, double(hi[0]) - lo[0]), y = std::max(0.0, double(hi[1]) - lo[1]),
                     z = std::max(0.0, double(hi[2]) - lo[2]);
        return 2.0 * (x * y + y * z + z * x);
    }
};

struct Leaf {
    Box box;
    float c[3];
    uint32_t link;
};

struct BNode {  // binary build node
    Box box;
    int left = -1, right = -1;  // children (binary node ids), -1 for a leaf
    int leaf = -1;              // index into leaves when a leaf (first of `count` consecutive ones)
    int count = 1;
};

constexpr int kMaxBins = 128;
constexpr int kBins = 32;  // SAH bins per axis (BDPT_SAH_BINS overrides, up to kMaxBins)
constexpr int kMaxBinaryDepth = 96;

class Builder {
   public:
    explicit Builder(std::vector<Leaf>& leaves) : L(leaves) {}
    std::vector<BNode> nodes;
    int max_depth = 0;
    bool median_only = false;
    // Leaves of up to max_leaf items, closed by the SAH (leaf cost n * area vs
    // node_cost * area + the best split); max_leaf 1 = one item per leaf.
    int max_leaf = 1;
    double node_cost = 1.0;
    int bins = kBins;

    int build(int b, int e, int depth) {
        max_depth = std::max(max_depth, depth);
        const int id = static_cast<int>(nodes.size());
        nodes.emplace_back();
        Box box;
        box.clear();
        for (int i = b; i < e; i++) box.grow(L[i].box);
        nodes[id].box = box;
        if (e - b == 1) {
            nodes[id].leaf = b;
            return id;
        }
        double split_cost = 0.0;
        const int mid = split(b, e, &split_cost);
        if (e - b <= max_leaf && box.area() * (e - b) <= node_cost * box.area() + split_cost) {
            nodes[id].leaf = b;
            nodes[id].count = e - b;
            return id;
        }
        const int l = build(b, mid, depth + 1);
        const int r = build(mid, e, depth + 1);
        nodes[id].left = l;
        nodes[id].right = r;
        return id;
    }

   private:
    std::vector<Leaf>& L;

    int median(int b, int e, int axis) {
        const int mid = (b + e) / 2;
        std::nth_element(L.begin() + b, L.begin() + mid, L.begin() + e,
                         [axis](const Leaf& x, const Leaf& y) { return x.c[axis] < y.c[axis]; });
        return mid;
    }

    int split(int b, int e, double* cost_out = nullptr) {
        float cl[3], ch[3];
        for (int a = 0; a < 3; a++) cl[a] = __builtin_inff(), ch[a] = -__builtin_inff();
        for (int i = b; i < e; i++)
            for (int a = 0; a < 3; a++) cl[a] = std::min(cl[a], L[i].c[a]), ch[a] = std::max(ch[a], L[i].c[a]);
        int wide_axis = 0;
        for (int a = 1; a < 3; a++)
            if (ch[a] - cl[a] > ch[wide_axis] - cl[wide_axis]) wide_axis = a;
        if (cost_out) *cost_out = __builtin_inf();
        if (median_only || !(ch[wide_axis] > cl[wide_axis])) return median(b, e, wide_axis);
        double best = __builtin_inf();
        int best_axis = -1, best_bin = -1;
        for (int a = 0; a < 3; a++) {
            if (!(ch[a] > cl[a])) continue;
            const double scale = bins / (double(ch[a]) - cl[a]);
            Box bb[kMaxBins];
            int cnt[kMaxBins] = {};
            for (int k = 0; k < bins; k++) bb[k].clear();
            for (int i = b; i < e; i++) {
                int k = static_cast<int>((double(L[i].c[a]) - cl[a]) * scale);
                k = std::min(std::max(k, 0), bins - 1);
                cnt[k]++;
                bb[k].grow(L[i].box);
            }
            double right_area[kMaxBins];
            int right_cnt[kMaxBins];
            Box acc;
            acc.clear();
            int n = 0;
            for (int k = bins - 1; k > 0; k--) {
                acc.grow(bb[k]);
                n += cnt[k];
                right_area[k] = acc.area();
                right_cnt[k] = n;
            }
            acc.clear();
            n = 0;
            for (int k = 0; k < bins - 1; k++) {
                acc.grow(bb[k]);
                n += cnt[k];
                if (n == 0 || right_cnt[k + 1] == 0) continue;
                const double cost = acc.area() * n + right_area[k + 1] * right_cnt[k + 1];
                if (cost < best) best = cost, best_axis = a, best_bin = k;
            }
        }
        if (best_axis < 0) return median(b, e, wide_axis);
        if (cost_out) *cost_out = best;
        const double scale = bins / (double(ch[best_axis]) - cl[best_axis]);
        const float lo = cl[best_axis];
        auto it = std::partition(L.begin() + b, L.begin() + e, [&](const Leaf& x) {
            int k = static_cast<int>((double(x.c[best_axis]) - lo) * scale);
            k = std::min(std::max(k, 0), bins - 1);
            return k <= best_bin;
        });
        const int mid = static_cast<int>(it - L.begin());
        if (mid == b || mid == e) return median(b, e, wide_axis);
        return mid;
    }
};

float u2f(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// Collapses the binary tree to 4-wide nodes (repeatedly opening the interior
// child of largest area) into out.nodes; returns the root link.
// The children of every 4-wide node are chosen by dynamic programming over the
// binary tree to minimise the SAH cost (area-weighted node and triangle tests,
// BDPT_DP_NODE_COST per node test, 1 per triangle; round 3: HardLight +1.6 %,
// Caustic / synth1m +-0.2 %, 13 % fewer nodes). BDPT_WIDE_COLLAPSE=greedy
// restores the earlier rule: open the largest interior child first.
struct DpCollapse {
    std::vector<std::array<double, kWideArity + 1>> dist;  // [j]: best cost of the subtree as <= j children
    std::vector<std::array<int, kWideArity + 1>> cut;      // [j]: 0 = the subtree itself, else slots to the left
    std::vector<double> cost;                              // the subtree as one child (a leaf, or a wide node)
    std::vector<int> wide_cut;                             // a wide node here: slots given to the left child
    void run(const std::vector<BNode>& bn, double node_cost) {
        const size_t n = bn.size();
        dist.assign(n, {});
        cut.assign(n, {});
        cost.assign(n, 0.0);
        wide_cut.assign(n, 1);
        std::function<void(int)> visit = [&](int id) {
            const BNode& b = bn[id];
            const double area = b.box.area();
            if (b.leaf >= 0) {
                cost[id] = area * b.count;
                for (int j = 1; j <= kWideArity; j++) dist[id][j] = cost[id], cut[id][j] = 0;
                return;
            }
            visit(b.left);
            visit(b.right);
            double best = __builtin_inf();
            for (int i = 1; i < kWideArity; i++) {
                const double c = dist[b.left][i] + dist[b.right][kWideArity - i];
                if (c < best) best = c, wide_cut[id] = i;
            }
            cost[id] = area * node_cost + best;
            dist[id][1] = cost[id], cut[id][1] = 0;
            for (int j = 2; j <= kWideArity; j++) {
                dist[id][j] = cost[id], cut[id][j] = 0;
                for (int i = 1; i < j; i++) {
                    const double c = dist[b.left][i] + dist[b.right][j - i];
                    if (c < dist[id][j]) dist[id][j] = c, cut[id][j] = i;
                }
            }
        };
        visit(0);
    }
    void gather(const std::vector<BNode>& bn, int id, int j, std::vector<int>& out) const {
        if (cut[id][j] == 0) {
            out.push_back(id);
            return;
        }
        gather(bn, bn[id].left, cut[id][j], out);
        gather(bn, bn[id].right, j - cut[id][j], out);
    }
};

uint32_t collapse(const std::vector<BNode>& bn, const std::function<uint32_t(const BNode&)>& leaf_link, WideBvh& out) {
    int max_stack = 0, max_depth = 0;
    const char* mode = std::getenv("BDPT_WIDE_COLLAPSE");
    const bool dp = !(mode && std::string(mode) == "greedy");
    DpCollapse D;
    if (dp) {
        const char* nc = std::getenv("BDPT_DP_NODE_COST");
        D.run(bn, nc ? std::max(0.0, std::atof(nc)) : 1.0);
    }
    std::function<uint32_t(int, int, int)> emit = [&](int id, int depth, int stack_above) -> uint32_t {
        std::vector<int> ch;
        if (dp) {
            D.gather(bn, bn[id].left, D.wide_cut[id], ch);
            D.gather(bn, bn[id].right, kWideArity - D.wide_cut[id], ch);
        } else {
            ch = {bn[id].left, bn[id].right};
        }
        while (!dp && static_cast<int>(ch.size()) < kWideArity) {
            int pick = -1;
            double area = -1.0;
            for (int k = 0; k < static_cast<int>(ch.size()); k++)
                if (bn[ch[k]].leaf < 0 && bn[ch[k]].box.area() > area) area = bn[ch[k]].box.area(), pick = k;
            if (pick < 0) break;
            const int c = ch[pick];
            ch[pick] = bn[c].left;
            ch.push_back(bn[c].right);
        }
        const uint32_t me = static_cast<uint32_t>(out.nodes.size() / 8);
        out.nodes.resize(out.nodes.size() + 8);
        max_depth = std::max(max_depth, depth + 1);
        const int stack_here = stack_above + static_cast<int>(ch.size()) - 1;
        max_stack = std::max(max_stack, stack_here);
        uint32_t links[kWideArity];
        Box boxes[kWideArity];
        for (int k = 0; k < kWideArity; k++) {
            if (k >= static_cast<int>(ch.size())) {
                links[k] = kEmptyLink;
                for (int a = 0; a < 3; a++) boxes[k].lo[a] = boxes[k].hi[a] = 0.f;
                continue;
            }
            const BNode& c = bn[ch[k]];
            boxes[k] = c.box;
            links[k] = c.leaf >= 0 ? leaf_link(c) : emit(ch[k], depth + 1, stack_here);
        }
        float4_t* r = &out.nodes[8 * static_cast<size_t>(me)];
        for (int a = 0; a < 3; a++) {
            r[2 * a] = {boxes[0].lo[a], boxes[1].lo[a], boxes[2].lo[a], boxes[3].lo[a]};
            r[2 * a + 1] = {boxes[0].hi[a], boxes[1].hi[a], boxes[2].hi[a], boxes[3].hi[a]};
        }
        r[6] = {u2f(links[0]), u2f(links[1]), u2f(links[2]), u2f(links[3])};
        r[7] = {0.f, 0.f, 0.f, 0.f};
        return me;
    };
    const uint32_t root = emit(0, 0, 0);
    out.max_stack = max_stack;
    out.depth = max_depth;
    return root;
}

// Node order in memory. The collapse emits nodes depth-first (a node's first
// child follows it; its siblings come after that child's whole subtree).
// BDPT_NODE_ORDER=bfs lays the tree out level by level; =treelet in treelets of
// kTreeletDepth levels (1 + 4 + 16 nodes, contiguous, breadth-first inside), each
// followed by the treelets below it in child order — the order a walk's next few
// levels are read in. Links are renumbered; node 0 stays the root.
constexpr int kTreeletDepth = 3;
void reorder_nodes(WideBvh& out) {
    const char* mode = std::getenv("BDPT_NODE_ORDER");
    if (!mode || std::string(mode) == "dfs") return;
    const bool bfs = std::string(mode) == "bfs";
    const size_t nn = out.nodes.size() / 8;
    if (nn < 2) return;
    auto kids = [&](uint32_t i, uint32_t (&l)[kWideArity]) {
        std::memcpy(l, &out.nodes[8 * static_cast<size_t>(i) + 6], sizeof(l));
    };
    std::vector<uint32_t> order;
    order.reserve(nn);
    if (bfs) {
        order.push_back(0);
        for (size_t h = 0; h < order.size(); h++) {
            uint32_t l[kWideArity];
            kids(order[h], l);
            for (uint32_t c : l)
                if (c != kEmptyLink && !(c & kLeafBit)) order.push_back(c);
        }
    } else {
        std::function<void(uint32_t)> treelet = [&](uint32_t root) {
            std::vector<uint32_t> level{root}, frontier;
            for (int d = 0; d < kTreeletDepth && !level.empty(); d++) {
                std::vector<uint32_t> next;
                for (uint32_t i : level) {
                    order.push_back(i);
                    uint32_t l[kWideArity];
                    kids(i, l);
                    for (uint32_t c : l)
                        if (c != kEmptyLink && !(c & kLeafBit)) (d + 1 < kTreeletDepth ? next : frontier).push_back(c);
                }
                level.swap(next);
            }
            for (uint32_t f : frontier) treelet(f);
        };
        treelet(0);
    }
    std::vector<uint32_t> newid(nn, kEmptyLink);
    for (size_t k = 0; k < order.size(); k++) newid[order[k]] = static_cast<uint32_t>(k);
    std::vector<float4_t> nodes(out.nodes.size());
    for (size_t k = 0; k < order.size(); k++) {
        std::memcpy(&nodes[8 * k], &out.nodes[8 * static_cast<size_t>(order[k])], 8 * sizeof(float4_t));
        uint32_t l[kWideArity];
        std::memcpy(l, &nodes[8 * k + 6], sizeof(l));
        for (uint32_t& c : l)
            if (c != kEmptyLink && !(c & kLeafBit)) c = newid[c];
        std::memcpy(&nodes[8 * k + 6], l, sizeof(l));
    }
    out.nodes.swap(nodes);
}

}  // namespace

bool build_wide_bvh(const std::vector<FlatNode>& flat, WideBvh& out, std::string& err) {
    out = WideBvh();
    if (flat.empty()) {
        err = "empty BVH";
        return false;
    }
    std::vector<Leaf> leaves;
    for (const FlatNode& n : flat) {
        if (n.right_offset != 0) continue;
        Leaf l;
        for (int a = 0; a < 3; a++) {
            l.box.lo[a] = n.bmin[a];
            l.box.hi[a] = n.bmax[a];
            l.c[a] = 0.5f * (n.bmin[a] + n.bmax[a]);
        }
        l.link = make_leaf_link(n.start, n.nprims);
        leaves.push_back(l);
    }
    out.leaves = static_cast<int64_t>(leaves.size());
    if (flat[0].right_offset == 0) {  // the whole scene is one leaf: the reference tests no box
        out.root_link = leaves[0].link;
        return true;
    }
    Builder B(leaves);
    if (const char* e = std::getenv("BDPT_SAH_BINS")) B.bins = std::min(kMaxBins, std::max(2, std::atoi(e)));
    B.build(0, static_cast<int>(leaves.size()), 0);
    if (B.max_depth > kMaxBinaryDepth) {  // degenerate SAH splits: fall back to a balanced tree
        Builder M(leaves);
        M.median_only = true;
        M.build(0, static_cast<int>(leaves.size()), 0);
        B.nodes.swap(M.nodes);
        B.max_depth = M.max_depth;
    }
    out.root_link = collapse(B.nodes, [&](const BNode& c) { return leaves[c.leaf].link; }, out);
    if (out.root_link != 0) {
        err = "wide BVH root must be node 0";
        return false;
    }
    return true;
}

bool build_wide_bvh_tris(const std::vector<FlatNode>& flat, const std::vector<float4_t>& tri,
                         const std::vector<float4_t>& shade, float pad_rel, TriWideBvh& out, std::string& err) {
    out = TriWideBvh();
    const size_t n = tri.size() / 3;
    if (flat.empty() || n == 0) {
        err = "empty BVH";
        return false;
    }
    // reference leaf of every triangle (leaf order) and the leaf boxes
    std::vector<int32_t> leaf_of(n, -1);
    for (const FlatNode& f : flat) {
        if (f.right_offset != 0) continue;
        const int32_t id = static_cast<int32_t>(out.leaf_box.size() / 2);
        for (uint32_t k = 0; k < f.nprims; k++) leaf_of[f.start + k] = id;
        out.leaf_box.push_back({f.bmin[0], f.bmin[1], f.bmin[2], 0.f});
        out.leaf_box.push_back({f.bmax[0], f.bmax[1], f.bmax[2], 0.f});
    }
    if (flat[0].right_offset == 0) {  // the whole scene is one leaf: the reference tests no box
        const float inf = __builtin_inff();
        out.leaf_box[0] = {-inf, -inf, -inf, 0.f};
        out.leaf_box[1] = {inf, inf, inf, 0.f};
    }
    std::vector<Leaf> items(n);
    Box scene;
    scene.clear();
    for (size_t i = 0; i < n; i++) {
        if (leaf_of[i] < 0) {
            err = "triangle outside every BVH leaf";
            return false;
        }
        const float4_t& v0 = tri[3 * i];
        const float4_t& v1 = shade[5 * i + 3];
        const float4_t& v2 = shade[5 * i + 4];
        Box& b = items[i].box;
        b.lo[0] = std::min({v0.x, v1.x, v2.x}), b.hi[0] = std::max({v0.x, v1.x, v2.x});
        b.lo[1] = std::min({v0.y, v1.y, v2.y}), b.hi[1] = std::max({v0.y, v1.y, v2.y});
        b.lo[2] = std::min({v0.z, v1.z, v2.z}), b.hi[2] = std::max({v0.z, v1.z, v2.z});
        scene.grow(b);
        items[i].link = static_cast<uint32_t>(i);
    }
    double diag = 0.0;
    for (int a = 0; a < 3; a++) diag += (double(scene.hi[a]) - scene.lo[a]) * (double(scene.hi[a]) - scene.lo[a]);
    const float pad = static_cast<float>(pad_rel * std::sqrt(diag));
    for (Leaf& it : items)
        for (int a = 0; a < 3; a++) {
            it.c[a] = 0.5f * (it.box.lo[a] + it.box.hi[a]);
            it.box.lo[a] = std::nextafter(it.box.lo[a] - pad, -__builtin_inff());
            it.box.hi[a] = std::nextafter(it.box.hi[a] + pad, __builtin_inff());
        }
    out.pad = pad;
    // BDPT_TRI_LEAF_MAX / BDPT_SAH_NODE_COST override the builder (experiments)
    int leaf_max = kTriLeafMax;
    double node_cost = 1.0;
    if (const char* e = std::getenv("BDPT_TRI_LEAF_MAX")) leaf_max = std::min(7, std::max(1, std::atoi(e)));
    if (const char* e = std::getenv("BDPT_SAH_NODE_COST")) node_cost = std::max(0.0, std::atof(e));
    Builder B(items);
    B.max_leaf = leaf_max;
    B.node_cost = node_cost;
    if (const char* e = std::getenv("BDPT_SAH_BINS")) B.bins = std::min(kMaxBins, std::max(2, std::atoi(e)));
    B.build(0, static_cast<int>(n), 0);
    if (B.max_depth > kMaxBinaryDepth) {
        Builder M(items);
        M.median_only = true;
        M.max_leaf = leaf_max;
        M.node_cost = node_cost;
        M.build(0, static_cast<int>(n), 0);
        B.nodes.swap(M.nodes);
        B.max_depth = M.max_depth;
    }
    // traversal triangles in the new leaf order: v0 | ref index, e1 | ref leaf, e2
    out.tri.resize(3 * n);
    for (size_t k = 0; k < n; k++) {
        const uint32_t i = items[k].link;
        const float4_t a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
        out.tri[3 * k] = {a.x, a.y, a.z, u2f(i)};
        out.tri[3 * k + 1] = {b.x, b.y, b.z, u2f(static_cast<uint32_t>(leaf_of[i]))};
        out.tri[3 * k + 2] = {c.x, c.y, c.z, 0.f};
    }
    int64_t wleaves = 0;
    if (B.nodes[0].leaf >= 0) {  // a single leaf: no node to test
        out.bvh.root_link = make_leaf_link(0, static_cast<uint32_t>(n));
        out.bvh.leaves = 1;
        return true;
    }
    out.bvh.root_link = collapse(B.nodes, [&](const BNode& c) {
        wleaves++;
        return make_leaf_link(static_cast<uint32_t>(c.leaf), static_cast<uint32_t>(c.count));
    }, out.bvh);
    out.bvh.leaves = wleaves;
    reorder_nodes(out.bvh);
    if (out.bvh.root_link != 0) {
        err = "wide BVH root must be node 0";
        return false;
    }
    return true;
}

bool quantize_wide_nodes(const std::vector<float4_t>& wn, std::vector<float4_t>& out) {
    const size_t nn = wn.size() / 8;
    out.assign(4 * nn, float4_t{0.f, 0.f, 0.f, 0.f});
    for (size_t i = 0; i < nn; i++) {
        const float4_t* r = &wn[8 * i];
        uint32_t link[4];
        std::memcpy(link, &r[6], 16);
        float org[3];
        uint32_t ebits = 0, qw[6] = {0, 0, 0, 0, 0, 0};  // lo.x hi.x lo.y hi.y lo.z hi.z, one byte per child
        for (int a = 0; a < 3; a++) {
            const float* lo = &r[2 * a].x;
            const float* hi = &r[2 * a + 1].x;
            float o = __builtin_inff(), top = -__builtin_inff();
            for (int c = 0; c < 4; c++)
                if (link[c] != kEmptyLink) o = std::min(o, lo[c]), top = std::max(top, hi[c]);
            if (o > top) o = top = 0.f;  // no child (not built, kept well-formed)
            if (!std::isfinite(o) || !std::isfinite(top)) return false;
            const double ext = double(top) - double(o);
            int e = kQuantExpMin;
            while (ext > 255.0 * std::ldexp(1.0, e))
                if (++e > kQuantExpMax) return false;
            const double step = std::ldexp(1.0, e);
            for (int c = 0; c < 4; c++) {
                if (link[c] == kEmptyLink) continue;
                const double ql = std::floor((double(lo[c]) - o) / step), qh = std::ceil((double(hi[c]) - o) / step);
                if (ql < 0.0 || qh > 255.0 || ql > qh) return false;  // cannot happen: lo, hi in [o, top]
                qw[2 * a] |= static_cast<uint32_t>(ql) << (8 * c);
                qw[2 * a + 1] |= static_cast<uint32_t>(qh) << (8 * c);
            }
            org[a] = o;
            ebits |= static_cast<uint32_t>(e + 127) << (8 * a);
        }
        float4_t* q = &out[4 * i];
        q[0] = {org[0], org[1], org[2], u2f(ebits)};
        q[1] = {u2f(qw[0]), u2f(qw[1]), u2f(qw[2]), u2f(qw[3])};
        q[2] = {u2f(qw[4]), u2f(qw[5]), 0.f, 0.f};
        q[3] = r[6];
    }
    return true;
}

}  // namespace bdpt
