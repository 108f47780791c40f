// Host model of the traversal work per ray (node visits, leaf visits, triangle
// tests) for the current 4-wide tree over the reference leaves vs a 4-wide
// binned-SAH tree over single triangles (a design probe; not product code).
//   g++ -O2 -std=c++17 -I../include -Icsrc tools/trav_sim.cpp csrc/scene.cpp csrc/wide_bvh.cpp ...
//   trav_sim scene.obj rays.f32 [max_leaf] [pad_rel]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "scene.hpp"
#include "wide_bvh.hpp"

using namespace bdpt;

namespace {
struct V3 {
    float x, y, z;
};
V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct Ray {
    V3 o, d;
    float tmin, tmax;
};

bool tri_test(V3 v0, V3 e1, V3 e2, const Ray& r, float& t) {
    V3 p = cross(r.d, e2);
    float det = dot(e1, p);
    if (std::fabs(det) < 1e-8f) return false;
    float inv = 1.f / det;
    V3 tv = sub(r.o, v0);
    float u = dot(tv, p) * inv;
    if (u < 0.f || u > 1.f) return false;
    V3 q = cross(tv, e1);
    float v = dot(r.d, q) * inv;
    if (v < 0.f || u + v > 1.f) return false;
    t = dot(e2, q) * inv;
    return t >= 0x1.0624dep-10f;
}

bool slab(const float lo[3], const float hi[3], const Ray& r, float& tn, float& tf) {
    float a0 = (lo[0] - r.o.x) / r.d.x, a1 = (hi[0] - r.o.x) / r.d.x;
    float b0 = (lo[1] - r.o.y) / r.d.y, b1 = (hi[1] - r.o.y) / r.d.y;
    float c0 = (lo[2] - r.o.z) / r.d.z, c1 = (hi[2] - r.o.z) / r.d.z;
    tn = std::max(std::max(std::min(a0, a1), std::min(b0, b1)), std::min(c0, c1));
    tf = std::min(std::min(std::max(a0, a1), std::max(b0, b1)), std::max(c0, c1));
    return tn <= tf + 1e-6f * (std::fabs(tn) + std::fabs(tf));
}

struct Box {
    float lo[3], hi[3];
    void clear() {
        for (int a = 0; a < 3; a++) lo[a] = INFINITY, hi[a] = -INFINITY;
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; a++) lo[a] = std::min(lo[a], b.lo[a]), hi[a] = std::max(hi[a], b.hi[a]);
    }
    double area() const {
        double x = std::max(0.0, double(hi[0]) - lo[0]), y = std::max(0.0, double(hi[1]) - lo[1]),
               z = std::max(0.0, double(hi[2]) - lo[2]);
        return 2 * (x * y + y * z + z * x);
    }
};

// 4-wide node (host form): child boxes and links (leaf: first | count << 24 | 1 << 31)
struct WNode {
    Box b[4];
    uint32_t link[4];
    int n;
};
constexpr uint32_t LEAF = 0x80000000u;

struct Tree {
    std::vector<WNode> nodes;
    std::vector<int> tri_order;  // leaf tri slots -> triangle index (leaf order of the layout)
};

// binned SAH over items (boxes + centroids), leaves of <= max_leaf items
struct Item {
    Box box;
    float c[3];
    int id;
};

struct BN {
    Box box;
    int l = -1, r = -1, b = 0, e = 0;
};

void build_sah(std::vector<Item>& it, int max_leaf, double ci, std::vector<BN>& out) {
    std::function<int(int, int)> rec = [&](int b, int e) -> int {
        int id = (int)out.size();
        out.emplace_back();
        Box box;
        box.clear();
        for (int i = b; i < e; i++) box.grow(it[i].box);
        out[id].box = box;
        out[id].b = b, out[id].e = e;
        int n = e - b;
        float cl[3], ch[3];
        for (int a = 0; a < 3; a++) cl[a] = INFINITY, ch[a] = -INFINITY;
        for (int i = b; i < e; i++)
            for (int a = 0; a < 3; a++) cl[a] = std::min(cl[a], it[i].c[a]), ch[a] = std::max(ch[a], it[i].c[a]);
        double best = INFINITY;
        int ba = -1, bb = -1;
        const int K = 32;
        for (int a = 0; a < 3 && n > 1; a++) {
            if (!(ch[a] > cl[a])) continue;
            double sc = K / (double(ch[a]) - cl[a]);
            Box bx[K];
            int cn[K] = {};
            for (int k = 0; k < K; k++) bx[k].clear();
            for (int i = b; i < e; i++) {
                int k = std::min(std::max(int((it[i].c[a] - cl[a]) * sc), 0), K - 1);
                cn[k]++;
                bx[k].grow(it[i].box);
            }
            double ra[K];
            int rc[K];
            Box acc;
            acc.clear();
            int m = 0;
            for (int k = K - 1; k > 0; k--) acc.grow(bx[k]), m += cn[k], ra[k] = acc.area(), rc[k] = m;
            acc.clear();
            m = 0;
            for (int k = 0; k < K - 1; k++) {
                acc.grow(bx[k]);
                m += cn[k];
                if (!m || !rc[k + 1]) continue;
                double cost = acc.area() * m + ra[k + 1] * rc[k + 1];
                if (cost < best) best = cost, ba = a, bb = k;
            }
        }
        double leaf_cost = box.area() * n;
        double split_cost = ci * box.area() + best;
        if (n <= max_leaf && (ba < 0 || leaf_cost <= split_cost)) return id;
        int mid;
        if (ba < 0) {
            mid = (b + e) / 2;
        } else {
            double sc = K / (double(ch[ba]) - cl[ba]);
            float lo = cl[ba];
            auto p = std::partition(it.begin() + b, it.begin() + e, [&](const Item& x) {
                return std::min(std::max(int((x.c[ba] - lo) * sc), 0), K - 1) <= bb;
            });
            mid = int(p - it.begin());
            if (mid == b || mid == e) mid = (b + e) / 2;
        }
        int l = rec(b, mid), r = rec(mid, e);
        out[id].l = l, out[id].r = r;
        return id;
    };
    rec(0, (int)it.size());
}

// collapse binary to 4-wide; leaf payload = items [b, e)
void collapse(const std::vector<BN>& bn, Tree& T, const std::vector<Item>& it, bool item_is_group,
              const std::vector<std::pair<int, int>>& groups) {
    std::function<uint32_t(int)> emit = [&](int id) -> uint32_t {
        std::vector<int> ch = {bn[id].l, bn[id].r};
        while (ch.size() < 4) {
            int pick = -1;
            double ar = -1;
            for (size_t k = 0; k < ch.size(); k++)
                if (bn[ch[k]].l >= 0 && bn[ch[k]].box.area() > ar) ar = bn[ch[k]].box.area(), pick = (int)k;
            if (pick < 0) break;
            int c = ch[pick];
            ch[pick] = bn[c].l;
            ch.push_back(bn[c].r);
        }
        uint32_t me = (uint32_t)T.nodes.size();
        T.nodes.emplace_back();
        WNode w;
        w.n = (int)ch.size();
        for (int k = 0; k < w.n; k++) {
            const BN& c = bn[ch[k]];
            w.b[k] = c.box;
            if (c.l < 0) {
                uint32_t first = (uint32_t)T.tri_order.size();
                for (int i = c.b; i < c.e; i++) {
                    if (item_is_group)
                        for (int t = groups[it[i].id].first; t < groups[it[i].id].second; t++) T.tri_order.push_back(t);
                    else
                        T.tri_order.push_back(it[i].id);
                }
                w.link[k] = LEAF | (uint32_t(T.tri_order.size()) - first) << 24 | first;
            } else {
                w.link[k] = emit(ch[k]);
            }
        }
        T.nodes[me] = w;
        return me;
    };
    if (bn[0].l < 0) {
        std::fprintf(stderr, "single leaf\n");
        exit(1);
    }
    emit(0);
}

struct Stat {
    double nodes = 0, leaves = 0, tris = 0, iters = 0;
};

int trace(const Tree& T, const std::vector<float4_t>& tri, const Ray& r, bool any, Stat& s) {
    struct E {
        uint32_t link;
        float tn;
    };
    E st[256];
    int sp = 0;
    uint32_t link = 0;
    float best = r.tmax;
    int hit = -1;
    auto far = [&]() { float b = any ? r.tmax : best; return b + std::fabs(b) * 1e-3f + 1e-4f; };
    for (;;) {
        s.iters++;
        if (link & LEAF) {
            s.leaves++;
            uint32_t first = link & 0xffffff, cnt = (link >> 24) & 0x7f;
            for (uint32_t k = 0; k < cnt; k++) {
                int t = T.tri_order[first + k];
                s.tris++;
                V3 v0{tri[3 * t].x, tri[3 * t].y, tri[3 * t].z}, e1{tri[3 * t + 1].x, tri[3 * t + 1].y, tri[3 * t + 1].z},
                    e2{tri[3 * t + 2].x, tri[3 * t + 2].y, tri[3 * t + 2].z};
                float th;
                if (tri_test(v0, e1, e2, r, th)) {
                    if (any) {
                        if (th <= r.tmax && th >= r.tmin) return t;
                    } else if (th < best || (th == best && t < hit)) best = th, hit = t;
                }
            }
        } else {
            s.nodes++;
            const WNode& w = T.nodes[link];
            E c[4];
            int n = 0;
            for (int k = 0; k < w.n; k++) {
                float tn, tf;
                if (slab(w.b[k].lo, w.b[k].hi, r, tn, tf) && !(tn > far()) && !(tf < 5e-4f)) c[n++] = {w.link[k], tn};
            }
            std::sort(c, c + n, [](const E& a, const E& b) { return a.tn < b.tn; });
            if (n) {
                for (int k = n - 1; k >= 1; k--) st[sp++] = c[k];
                link = c[0].link;
                continue;
            }
        }
        bool got = false;
        while (sp > 0) {
            E e = st[--sp];
            if (!(e.tn > far())) {
                link = e.link;
                got = true;
                break;
            }
        }
        if (!got) break;
    }
    return any ? -1 : hit;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int max_leaf = argc > 3 ? atoi(argv[3]) : 4;
    const float pad_rel = argc > 4 ? atof(argv[4]) : 1e-4f;
    const double ci = argc > 5 ? atof(argv[5]) : 1.0;
    HostScene hs;
    std::string err;
    if (!load_obj_scene(argv[1], hs, err)) return std::fprintf(stderr, "%s\n", err.c_str()), 1;
    DeviceLayout L;
    if (!build_device_layout(hs, L, err)) return std::fprintf(stderr, "%s\n", err.c_str()), 1;
    FILE* f = fopen(argv[2], "rb");
    std::vector<float> rv;
    float buf[8];
    while (fread(buf, 4, 8, f) == 8) rv.insert(rv.end(), buf, buf + 8);
    fclose(f);
    const size_t nr = rv.size() / 8;
    const int ntri = (int)(L.tri.size() / 3);
    // scene diagonal
    Box sb;
    sb.clear();
    std::vector<Box> tb(ntri);
    for (int t = 0; t < ntri; t++) {
        V3 v0{L.tri[3 * t].x, L.tri[3 * t].y, L.tri[3 * t].z};
        V3 e1{L.tri[3 * t + 1].x, L.tri[3 * t + 1].y, L.tri[3 * t + 1].z}, e2{L.tri[3 * t + 2].x, L.tri[3 * t + 2].y, L.tri[3 * t + 2].z};
        V3 p[3] = {v0, {v0.x + e1.x, v0.y + e1.y, v0.z + e1.z}, {v0.x + e2.x, v0.y + e2.y, v0.z + e2.z}};
        tb[t].clear();
        for (auto& q : p) {
            float a[3] = {q.x, q.y, q.z};
            for (int k = 0; k < 3; k++) tb[t].lo[k] = std::min(tb[t].lo[k], a[k]), tb[t].hi[k] = std::max(tb[t].hi[k], a[k]);
        }
        sb.grow(tb[t]);
    }
    double diag = std::sqrt(std::pow(sb.hi[0] - sb.lo[0], 2) + std::pow(sb.hi[1] - sb.lo[1], 2) + std::pow(sb.hi[2] - sb.lo[2], 2));
    float pad = float(pad_rel * diag);
    // (A) current: the reference leaves as items
    std::vector<std::pair<int, int>> groups;
    std::vector<Item> ga;
    for (const FlatNode& n : hs.nodes)
        if (n.right_offset == 0) {
            Item it;
            for (int a = 0; a < 3; a++) it.box.lo[a] = n.bmin[a], it.box.hi[a] = n.bmax[a], it.c[a] = 0.5f * (n.bmin[a] + n.bmax[a]);
            it.id = (int)groups.size();
            groups.push_back({(int)n.start, (int)(n.start + n.nprims)});
            ga.push_back(it);
        }
    std::vector<BN> bna;
    build_sah(ga, 1, 1.0, bna);
    Tree A;
    collapse(bna, A, ga, true, groups);
    // (B) single triangles, padded boxes
    std::vector<Item> gb(ntri);
    for (int t = 0; t < ntri; t++) {
        gb[t].box = tb[t];
        for (int a = 0; a < 3; a++) gb[t].box.lo[a] -= pad, gb[t].box.hi[a] += pad, gb[t].c[a] = 0.5f * (tb[t].lo[a] + tb[t].hi[a]);
        gb[t].id = t;
    }
    std::vector<BN> bnb;
    build_sah(gb, max_leaf, ci, bnb);
    Tree B;
    collapse(bnb, B, gb, false, groups);
    Stat sa, sbs, sa_any, sb_any;
    size_t mism = 0, nany = 0, nclose = 0;
    for (size_t i = 0; i < nr; i++) {
        const float* q = &rv[8 * i];
        Ray r{{q[0], q[1], q[2]}, {q[3], q[4], q[5]}, q[6], q[7]};
        if (r.d.x == 0 || r.d.y == 0 || r.d.z == 0) continue;
        bool any = r.tmax < 1e30f && r.tmin < 1e-6f;  // shadow segments of the fixture
        if (any) {
            nany++;
            int a = trace(A, L.tri, r, true, sa_any), b = trace(B, L.tri, r, true, sb_any);
            if ((a >= 0) != (b >= 0)) mism++;
        } else {
            nclose++;
            int a = trace(A, L.tri, r, false, sa), b = trace(B, L.tri, r, false, sbs);
            if (a != b) mism++;
        }
    }
    auto pr = [](const char* n, const Stat& s, size_t k) {
        std::printf("%-14s nodes %6.2f leaves %6.2f tris %6.2f iters %6.2f\n", n, s.nodes / k, s.leaves / k, s.tris / k,
                    s.iters / k);
    };
    std::printf("tris %d, A nodes %zu, B nodes %zu (leaf<=%d pad %.2e ci %.2f)\n", ntri, A.nodes.size(), B.nodes.size(),
                max_leaf, pad, ci);
    pr("A closest", sa, nclose);
    pr("B closest", sbs, nclose);
    pr("A any", sa_any, nany);
    pr("B any", sb_any, nany);
    std::printf("mismatches %zu of %zu\n", mism, nclose + nany);
    return 0;
}
