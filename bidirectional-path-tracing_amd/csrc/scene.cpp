// Host-side scene ingest (see scene.hpp). Compiled with -ffp-contract=off:
// every float expression below must round exactly like the reference's.
#include "scene.hpp"
#include "wide_bvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <unordered_map>

namespace bdpt {
namespace {

// ---------------------------------------------------------------- lexing
inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_digit(char c) { return static_cast<unsigned>(c - '0') < 10u; }
inline bool is_newline(char c) { return c == '\r' || c == '\n' || c == '\0'; }

bool read_whole_file(const std::string& path, std::string& buf) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    buf = ss.str();
    return true;
}

// Splits like tinyobj's safeGetline (tiny_obj_loader.h:419-451): a line ends at
// '\n', "\r\n" or a lone '\r'. Calls fn(line) with a NUL-terminated copy.
template <class F>
void for_each_line(const std::string& buf, F&& fn) {
    std::string line;
    size_t i = 0, n = buf.size();
    while (i < n) {
        size_t j = i;
        while (j < n && buf[j] != '\n' && buf[j] != '\r') ++j;
        line.assign(buf, i, j - i);
        if (j < n && buf[j] == '\r' && j + 1 < n && buf[j + 1] == '\n') ++j;
        i = j + 1;
        fn(line);
    }
}

// tinyobj tryParseDouble (tiny_obj_loader.h:525-638): decimal digits are
// accumulated in double through a 10^-k table, exponents via ldexp(m*5^e, e).
bool parse_double(const char* s, const char* end, double* out) {
    if (s >= end) return false;
    double mant = 0.0;
    int expo = 0, read = 0;
    char sign = '+', esign = '+';
    const char* c = s;
    if (*c == '+' || *c == '-') sign = *c++;
    else if (!is_digit(*c)) return false;
    bool more = c != end;
    while (more && is_digit(*c)) {
        mant *= 10;
        mant += static_cast<int>(*c - '0');
        ++c, ++read;
        more = c != end;
    }
    if (read == 0) return false;
    if (more) {
        if (*c == '.') {
            ++c;
            read = 1;
            more = c != end;
            static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (more && is_digit(*c)) {
                mant += static_cast<int>(*c - '0') * (read < 8 ? lut[read] : std::pow(10.0, -read));
                ++read, ++c;
                more = c != end;
            }
        } else if (*c != 'e' && *c != 'E') {
            more = false;  // anything else ends the number
            goto done;
        }
        if (more && (*c == 'e' || *c == 'E')) {
            ++c;
            more = c != end;
            if (more && (*c == '+' || *c == '-')) esign = *c++;
            else if (!is_digit(*c)) return false;
            read = 0;
            more = c != end;
            while (more && is_digit(*c)) {
                expo = expo * 10 + static_cast<int>(*c - '0');
                ++c, ++read;
                more = c != end;
            }
            expo *= (esign == '+' ? 1 : -1);
            if (read == 0) return false;
        }
    }
done:
    *out = (sign == '+' ? 1 : -1) * (expo ? std::ldexp(mant * std::pow(5.0, expo), expo) : mant);
    return true;
}

// parseReal (tiny_obj_loader.h:640-648)
float next_real(const char*& t, double def) {
    t += std::strspn(t, " \t");
    const char* e = t + std::strcspn(t, " \t\r");
    double v = def;
    parse_double(t, e, &v);
    t = e;
    return static_cast<float>(v);
}

int next_int(const char*& t) {
    t += std::strspn(t, " \t");
    int v = std::atoi(t);
    t += std::strcspn(t, " \t\r");
    return v;
}

bool resolve_index(int idx, int n, int* out) {  // fixIndex (tiny_obj_loader.h:459-480)
    if (idx > 0) return *out = idx - 1, true;
    if (idx == 0) return false;
    return *out = n + idx, true;
}

struct Corner {
    int v = -1, vn = -1, vt = -1;
};

// parseTriple (tiny_obj_loader.h:775-827)
bool next_corner(const char*& t, int nv, int nvn, int nvt, Corner* out) {
    Corner c;
    auto skip = [&] { t += std::strcspn(t, "/ \t\r"); };
    if (!resolve_index(std::atoi(t), nv, &c.v)) return false;
    skip();
    if (*t != '/') return *out = c, true;
    ++t;
    if (*t == '/') {
        ++t;
        if (!resolve_index(std::atoi(t), nvn, &c.vn)) return false;
        skip();
        return *out = c, true;
    }
    if (!resolve_index(std::atoi(t), nvt, &c.vt)) return false;
    skip();
    if (*t != '/') return *out = c, true;
    ++t;
    if (!resolve_index(std::atoi(t), nvn, &c.vn)) return false;
    skip();
    return *out = c, true;
}

// ------------------------------------------------------------------ MTL
struct MaterialTable {
    std::vector<Material> list;
    std::unordered_map<std::string, int> by_name;  // first definition wins (std::map::insert)
    void flush(const Material& m) {
        by_name.emplace(m.name, static_cast<int>(list.size()));
        list.push_back(m);
    }
};

// LoadMtl (tiny_obj_loader.h:1273-1657), keys the BDPT path reads.
void parse_mtl(const std::string& text, MaterialTable& tab) {
    Material m;
    for_each_line(text, [&](std::string& line) {
        size_t keep = line.find_last_not_of(" \t");
        line.resize(keep == std::string::npos ? 0 : keep + 1);
        if (line.empty()) return;
        const char* t = line.c_str();
        t += std::strspn(t, " \t");
        if (*t == '\0' || *t == '#') return;
        auto key2 = [&](char a, char b) { return t[0] == a && t[1] == b && is_space(t[2]); };
        if (std::strncmp(t, "newmtl", 6) == 0 && is_space(t[6])) {
            if (!m.name.empty()) tab.flush(m);
            m = Material();
            m.name = t + 7;
        } else if (key2('K', 'd')) {
            t += 2;
            for (float& x : m.Kd) x = next_real(t, 0.0);
        } else if (key2('K', 's')) {
            t += 2;
            for (float& x : m.Ks) x = next_real(t, 0.0);
        } else if (key2('K', 't') || key2('T', 'f')) {
            t += 2;
            for (float& x : m.Tf) x = next_real(t, 0.0);
        } else if (key2('N', 'i')) {
            t += 2;
            m.Ni = next_real(t, 0.0);
        } else if (key2('K', 'e')) {
            t += 2;
            for (float& x : m.Ke) x = next_real(t, 0.0);
        } else if (key2('N', 's')) {
            t += 2;
            m.Ns = next_real(t, 0.0);
        } else if (std::strncmp(t, "illum", 5) == 0 && is_space(t[5])) {
            t += 6;
            m.illum = next_int(t);
        } else if ((std::strncmp(t, "map_Kd", 6) == 0 || std::strncmp(t, "map_Ks", 6) == 0) && is_space(t[6])) {
            m.has_texture = true;
        }
    });
    tab.flush(m);  // the last material is always flushed
}

// ------------------------------------------------------------------ OBJ
struct Face {
    std::vector<Corner> c;
};

// pnpoly (tiny_obj_loader.h:1004-1015) for a triangle.
bool point_in_triangle(const float* vx, const float* vy, float tx, float ty) {
    bool inside = false;
    for (int i = 0, j = 2; i < 3; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i]))
            inside = !inside;
    }
    return inside;
}

struct ObjBuilder {
    std::vector<float> v, vn;
    int nvt = 0;
    std::vector<Face> group;
    struct Tri {
        Corner c[3];
        int mat, shape, prim;
    };
    std::vector<Tri> tris;
    int shapes = 0;            // shapes pushed so far
    size_t shape_begin = 0;    // first triangle of the current shape
    int shape_prims = 0;       // triangles already in the current shape

    void emit(const Corner& a, const Corner& b, const Corner& c, int mat) {
        tris.push_back(Tri{{a, b, c}, mat, shapes, shape_prims++});
    }

    // exportFaceGroupToShape with triangulate = true (tiny_obj_loader.h:1018-1261).
    bool flush_group(int material) {
        if (group.empty()) return false;
        const size_t vs = v.size();
        for (const Face& face : group) {
            size_t np = face.c.size();
            if (np < 3) continue;
            size_t axes[2] = {1, 2};
            for (size_t k = 0; k < np; ++k) {
                size_t a = face.c[k % np].v, b = face.c[(k + 1) % np].v, c = face.c[(k + 2) % np].v;
                if (3 * a + 2 >= vs || 3 * b + 2 >= vs || 3 * c + 2 >= vs) continue;
                float e0x = v[3 * b] - v[3 * a], e0y = v[3 * b + 1] - v[3 * a + 1], e0z = v[3 * b + 2] - v[3 * a + 2];
                float e1x = v[3 * c] - v[3 * b], e1y = v[3 * c + 1] - v[3 * b + 1], e1z = v[3 * c + 2] - v[3 * b + 2];
                float cx = std::fabs(e0y * e1z - e0z * e1y);
                float cy = std::fabs(e0z * e1x - e0x * e1z);
                float cz = std::fabs(e0x * e1y - e0y * e1x);
                const float eps = 1.19209290e-07f;  // numeric_limits<float>::epsilon()
                if (cx > eps || cy > eps || cz > eps) {
                    if (!(cx > cy && cx > cz)) {
                        axes[0] = 0;
                        if (cz > cx && cz > cy) axes[1] = 1;
                    }
                    break;
                }
            }
            auto coord = [&](size_t vi, int ax) { return v[vi * 3 + axes[ax]]; };
            auto in_range = [&](size_t vi) { return vi * 3 + axes[0] < vs && vi * 3 + axes[1] < vs; };
            float area = 0;
            for (size_t k = 0; k < np; ++k) {
                size_t a = face.c[k % np].v, b = face.c[(k + 1) % np].v;
                if (!in_range(a) || !in_range(b)) continue;
                area += (coord(a, 0) * coord(b, 1) - coord(a, 1) * coord(b, 0)) * 0.5f;
            }
            std::vector<Corner> rem = face.c;
            int rounds = 10;
            size_t guess = 0;
            while (rem.size() > 3 && rounds > 0) {
                np = rem.size();
                if (guess >= np) {
                    rounds -= 1;
                    guess -= np;
                }
                Corner ind[3];
                float vx[3], vy[3];
                for (size_t k = 0; k < 3; k++) {
                    ind[k] = rem[(guess + k) % np];
                    size_t vi = ind[k].v;
                    vx[k] = in_range(vi) ? coord(vi, 0) : 0.f;
                    vy[k] = in_range(vi) ? coord(vi, 1) : 0.f;
                }
                float cross = (vx[1] - vx[0]) * (vy[2] - vy[1]) - (vy[1] - vy[0]) * (vx[2] - vx[1]);
                if (cross * area < 0.f) {
                    guess += 1;
                    continue;
                }
                bool overlap = false;
                for (size_t o = 3; o < np && !overlap; ++o) {
                    size_t idx = (guess + o) % np;
                    if (idx >= rem.size()) continue;
                    size_t ov = rem[idx].v;
                    if (!in_range(ov)) continue;
                    overlap = point_in_triangle(vx, vy, coord(ov, 0), coord(ov, 1));
                }
                if (overlap) {
                    guess += 1;
                    continue;
                }
                emit(ind[0], ind[1], ind[2], material);
                rem.erase(rem.begin() + static_cast<long>((guess + 1) % np));
            }
            if (rem.size() == 3) emit(rem[0], rem[1], rem[2], material);
        }
        return true;
    }

    void push_shape() {
        shapes++;
        shape_begin = tris.size();
        shape_prims = 0;
    }
    void drop_shape() {
        tris.resize(shape_begin);
        shape_prims = 0;
    }
};

bool parse_obj(const std::string& path, ObjBuilder& ob, MaterialTable& mats, std::string& err) {
    std::string text;
    if (!read_whole_file(path, text)) {
        err = "cannot open " + path;
        return false;
    }
    std::string base = path.substr(0, path.find_last_of('/') + 1);
    if (base.empty()) base = "./";
    int material = -1;
    bool ok = true;
    for_each_line(text, [&](std::string& line) {
        if (!ok || line.empty()) return;
        const char* t = line.c_str();
        t += std::strspn(t, " \t");
        if (*t == '\0' || *t == '#') return;
        if (t[0] == 'v' && is_space(t[1])) {
            t += 2;
            for (int k = 0; k < 3; k++) ob.v.push_back(next_real(t, 0.0));
        } else if (t[0] == 'v' && t[1] == 'n' && is_space(t[2])) {
            t += 3;
            for (int k = 0; k < 3; k++) ob.vn.push_back(next_real(t, 0.0));
        } else if (t[0] == 'v' && t[1] == 't' && is_space(t[2])) {
            ob.nvt++;
        } else if (t[0] == 'f' && is_space(t[1])) {
            t += 2;
            t += std::strspn(t, " \t");
            Face f;
            while (!is_newline(*t)) {
                Corner c;
                if (!next_corner(t, static_cast<int>(ob.v.size() / 3), static_cast<int>(ob.vn.size() / 3), ob.nvt, &c)) {
                    err = "Failed parse `f' line (e.g. zero value for face index) in " + path;
                    ok = false;
                    return;
                }
                f.c.push_back(c);
                t += std::strspn(t, " \t\r");
            }
            ob.group.push_back(std::move(f));
        } else if (std::strncmp(t, "usemtl", 6) == 0 && is_space(t[6])) {
            auto it = mats.by_name.find(std::string(t + 7));
            int id = it == mats.by_name.end() ? -1 : it->second;
            if (id != material) {
                ob.flush_group(material);
                ob.group.clear();
                material = id;
            }
        } else if (std::strncmp(t, "mtllib", 6) == 0 && is_space(t[6])) {
            std::stringstream ss(std::string(t + 7));
            std::string name, mtl;
            while (std::getline(ss, name, ' ')) {
                if (!name.empty() && read_whole_file(base + name, mtl)) {
                    parse_mtl(mtl, mats);
                    break;
                }
            }
        } else if ((t[0] == 'g' || t[0] == 'o') && is_space(t[1])) {
            bool exported = ob.flush_group(material);
            bool keep = (t[0] == 'g') ? ob.tris.size() > ob.shape_begin : exported;
            if (keep) ob.push_shape();
            else ob.drop_shape();
            ob.group.clear();
        }
    });
    if (!ok) return false;
    bool exported = ob.flush_group(material);
    if (exported || ob.tris.size() > ob.shape_begin) ob.push_shape();
    else ob.drop_shape();
    return true;
}

// ---------------------------------------------------------------- float3
struct F3 {
    float x, y, z;
};
inline F3 operator+(F3 a, F3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline F3 operator-(F3 a, F3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline F3 operator*(F3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline F3 operator/(F3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
inline float dot(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }  // glm: (x + y) + z
inline F3 cross(F3 a, F3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline F3 normalize(F3 v) { return v * (1.f / std::sqrt(dot(v, v))); }
inline float comp(F3 v, int d) { return d == 0 ? v.x : (d == 1 ? v.y : v.z); }
inline F3 load3(const float* p) { return {p[0], p[1], p[2]}; }

// --------------------------------------------------------------- Fast-BVH
struct Box {
    F3 lo, hi;
};
inline float gmin(float a, float b) { return (b < a) ? b : a; }  // glm::min
inline float gmax(float a, float b) { return (a < b) ? b : a; }  // glm::max
inline void grow(Box& b, F3 p) {
    b.lo = {gmin(b.lo.x, p.x), gmin(b.lo.y, p.y), gmin(b.lo.z, p.z)};
    b.hi = {gmax(b.hi.x, p.x), gmax(b.hi.y, p.y), gmax(b.hi.z, p.z)};
}
inline void grow(Box& b, const Box& o) {
    b.lo = {gmin(b.lo.x, o.lo.x), gmin(b.lo.y, o.lo.y), gmin(b.lo.z, o.lo.z)};
    b.hi = {gmax(b.hi.x, o.hi.x), gmax(b.hi.y, o.hi.y), gmax(b.hi.z, o.hi.z)};
}
// BBox::maxDimension (bvh.h:82-87) on extent = max - min.
inline int widest(const Box& b) {
    F3 e = b.hi - b.lo;
    int r = 0;
    if (e.y > e.x) r = 1;
    if (e.z > e.y) r = 2;
    return r;
}

// BVH::build (bvh.h:147-247): midpoint split of the centroid bounds, leaf <= 4,
// in-place partition, median on a bad split, preorder with left child at i+1.
void build_bvh(HostScene& s) {
    const size_t n = s.num_triangles();
    s.order.resize(n);
    std::vector<F3> cen(n);
    std::vector<Box> tb(n);
    for (size_t i = 0; i < n; i++) {
        s.order[i] = static_cast<int32_t>(i);
        F3 a = load3(&s.pos[9 * i]), b = load3(&s.pos[9 * i + 3]), c = load3(&s.pos[9 * i + 6]);
        cen[i] = (a + b + c) / 3.0f;  // getCentroid (accel.h:105)
        tb[i] = Box{a, a};            // getBBox (accel.h:85-88)
        grow(tb[i], b);
        grow(tb[i], c);
    }
    struct Todo {
        uint32_t parent, start, end;
        int depth;
    };
    std::vector<Todo> todo;
    todo.push_back({0xfffffffcu, 0, static_cast<uint32_t>(n), 0});
    s.nodes.clear();
    s.nodes.reserve(2 * n + 1);
    s.max_depth = 0;
    while (!todo.empty()) {
        Todo t = todo.back();
        todo.pop_back();
        FlatNode node;
        node.start = t.start;
        node.nprims = t.end - t.start;
        node.right_offset = 0xffffffffu;
        Box bb = tb[s.order[t.start]];
        Box bc{cen[s.order[t.start]], cen[s.order[t.start]]};
        for (uint32_t p = t.start + 1; p < t.end; ++p) {
            grow(bb, tb[s.order[p]]);
            grow(bc, cen[s.order[p]]);
        }
        node.bmin[0] = bb.lo.x, node.bmin[1] = bb.lo.y, node.bmin[2] = bb.lo.z;
        node.bmax[0] = bb.hi.x, node.bmax[1] = bb.hi.y, node.bmax[2] = bb.hi.z;
        if (node.nprims <= 4) node.right_offset = 0;
        s.max_depth = std::max(s.max_depth, t.depth);
        const uint32_t self = static_cast<uint32_t>(s.nodes.size());
        s.nodes.push_back(node);
        if (t.parent != 0xfffffffcu) {
            FlatNode& p = s.nodes[t.parent];
            p.right_offset--;
            if (p.right_offset == 0xfffffffdu) p.right_offset = self - t.parent;
        }
        if (node.right_offset == 0) continue;
        const int d = widest(bc);
        const float split = .5f * (comp(bc.lo, d) + comp(bc.hi, d));
        uint32_t mid = t.start;
        for (uint32_t i = t.start; i < t.end; ++i)
            if (comp(cen[s.order[i]], d) < split) std::swap(s.order[i], s.order[mid++]);
        if (mid == t.start || mid == t.end) mid = t.start + (t.end - t.start) / 2;
        todo.push_back({self, mid, t.end, t.depth + 1});
        todo.push_back({self, t.start, mid, t.depth + 1});
    }
}

// The BSDF the reference constructs for a material (renderer.cpp:258-271):
// kind and EBSDFType bits by illum, the MTL constants; the mixture / Phong
// constructor constants (scale, specw) are filled by the caller.
BsdfRecord bsdf_record(const Material& m) {
    BsdfRecord b{};
    for (int k = 0; k < 3; k++) {
        b.kd[k] = m.Kd[k], b.ks[k] = m.Ks[k], b.tf[k] = m.Tf[k], b.emission[k] = m.Ke[k];
    }
    b.exponent = m.Ns;
    b.ior = m.Ni;
    b.scale = 1.f;
    switch (m.illum) {
        case 7: b.kind = BSDF_DIFFUSE, b.type = kTypeDiffuseRefl; break;
        case 3: b.kind = BSDF_MIRROR, b.type = kTypeDeltaRefl; break;
        case 6: b.kind = BSDF_GLASS, b.type = kTypeDeltaRefl | kTypeDeltaTrans; break;
        case 5: b.kind = BSDF_NULL, b.type = 0; break;
        default: b.kind = (m.illum == 8) ? BSDF_MIXTURE : BSDF_PHONG, b.type = kTypeGlossyRefl | kTypeDiffuseRefl;
    }
    return b;
}

// Scene::load dereferences the BSDF of every shape's first face
// (renderer.cpp:277-278: bsdf->isEmissive()); a null BSDF there would crash it.
bool check_shape_bsdfs(const HostScene& s, std::string& err) {
    for (size_t sh = 0; sh < s.shape_first.size(); sh++) {
        if (s.shape_count[sh] == 0) continue;
        if (s.bsdfs[s.tri_mat[s.shape_first[sh]]].kind == BSDF_NULL) {
            err = "shape " + std::to_string(sh) + " uses a null BSDF (illum 5) on its first face";
            return false;
        }
    }
    return true;
}

}  // namespace

bool load_obj_scene(const std::string& obj_path, HostScene& s, std::string& err) {
    ObjBuilder ob;
    MaterialTable mats;
    if (!parse_obj(obj_path, ob, mats, err)) return false;
    const size_t n = ob.tris.size();
    s = HostScene();
    s.pos.resize(9 * n);
    s.nrm.resize(9 * n);
    s.tri_shape.resize(n);
    s.tri_prim.resize(n);
    s.tri_mat.resize(n);
    for (size_t i = 0; i < n; i++) {
        const ObjBuilder::Tri& t = ob.tris[i];
        for (int c = 0; c < 3; c++) {
            if (t.c[c].v < 0 || 3 * static_cast<size_t>(t.c[c].v) + 2 >= ob.v.size()) {
                err = "face vertex index out of range";
                return false;
            }
            if (t.c[c].vn < 0 || 3 * static_cast<size_t>(t.c[c].vn) + 2 >= ob.vn.size()) {
                err = "face without a valid normal index (the reference needs per-vertex normals)";
                return false;
            }
            for (int d = 0; d < 3; d++) {
                s.pos[9 * i + 3 * c + d] = ob.v[3 * t.c[c].v + d];
                s.nrm[9 * i + 3 * c + d] = ob.vn[3 * t.c[c].vn + d];
            }
        }
        if (t.mat < 0 || static_cast<size_t>(t.mat) >= mats.list.size()) {
            err = "face without a material (usemtl missing or unknown)";
            return false;
        }
        s.tri_shape[i] = t.shape;
        s.tri_prim[i] = t.prim;
        s.tri_mat[i] = t.mat;
    }
    s.materials = mats.list;
    const int nshapes = ob.shapes;
    s.shape_first.assign(nshapes, 0);
    s.shape_count.assign(nshapes, 0);
    s.shape_emitter.assign(nshapes, -1);
    for (size_t i = n; i-- > 0;) s.shape_first[s.tri_shape[i]] = static_cast<int32_t>(i);
    for (size_t i = 0; i < n; i++) s.shape_count[s.tri_shape[i]]++;

    // BSDFs by illum (renderer.cpp:258-271) with the constructors' constants.
    for (const Material& m : s.materials) {
        if (m.has_texture) {
            err = "material '" + m.name + "' uses a bitmap texture (not supported)";
            return false;
        }
        BsdfRecord b = bsdf_record(m);
        if (b.kind == BSDF_MIXTURE || b.kind == BSDF_PHONG) {
            // mixture.h:39-46 / phong.h:40-47: energy-conserving scale and specular sampling weight.
            F3 mx = load3(b.ks) + load3(b.kd);
            float actualMax = std::max(std::max(mx.x, mx.y), mx.z);
            b.scale = actualMax > 1.0f ? 0.99f * (1.0f / actualMax) : 1.0f;
            const F3 lum{0.212671f, 0.715160f, 0.072169f};
            float dAvg = dot(load3(b.kd) * b.scale, lum);
            float sAvg = dot(load3(b.ks) * b.scale, lum);
            b.specw = sAvg / (dAvg + sAvg);
        }
        s.bsdfs.push_back(b);
    }
    if (!check_shape_bsdfs(s, err)) return false;
    // Emitters: shapes whose first face's BSDF emits (renderer.cpp:279-305).
    for (int sh = 0; sh < nshapes; sh++) {
        const BsdfRecord& b = s.bsdfs[s.tri_mat[s.shape_first[sh]]];
        F3 e = load3(b.emission);
        if (!(dot(e, e) > 0.f)) continue;
        Emitter em;
        em.shape = sh;
        for (int k = 0; k < 3; k++) em.radiance[k] = b.emission[k];
        em.cdf.push_back(0.f);
        for (int f = 0; f < s.shape_count[sh]; f++) {  // getShapeArea (renderer.cpp:317-339)
            const float* p = &s.pos[9 * static_cast<size_t>(s.shape_first[sh] + f)];
            F3 c = cross(load3(p + 3) - load3(p), load3(p + 6) - load3(p));
            em.cdf.push_back(em.cdf.back() + 0.5f * std::sqrt((c.x * c.x + c.y * c.y) + c.z * c.z));
        }
        em.area = em.cdf.back();
        const float sum = em.cdf.back();
        for (float& x : em.cdf) x /= sum;
        s.shape_emitter[sh] = static_cast<int32_t>(s.emitters.size());
        s.emitters.push_back(std::move(em));
    }
    build_bvh(s);
    return true;
}

// ------------------------------------------------------ caller's Scene (desc)
bool load_desc_scene(const bdpt_scene_desc& d, HostScene& s, std::string& err) {
    s = HostScene();
    if (d.triangles <= 0 || !d.positions || !d.normals || !d.tri_shape || !d.tri_prim || !d.tri_mat) {
        err = "scene descriptor: no triangles or a null triangle array";
        return false;
    }
    if (d.shapes <= 0 || d.materials <= 0 || !d.material || d.emitters < 0 || (d.emitters > 0 && !d.emitter) ||
        d.bvh_nodes <= 0 || !d.bvh || !d.bvh_order) {
        err = "scene descriptor: bad shape / material / emitter / BVH table";
        return false;
    }
    const size_t n = static_cast<size_t>(d.triangles);
    if (n >= (1u << 28)) {
        err = "more than 2^28 triangles";
        return false;
    }
    s.pos.assign(d.positions, d.positions + 9 * n);
    s.nrm.assign(d.normals, d.normals + 9 * n);
    s.tri_shape.assign(d.tri_shape, d.tri_shape + n);
    s.tri_prim.assign(d.tri_prim, d.tri_prim + n);
    s.tri_mat.assign(d.tri_mat, d.tri_mat + n);
    // AcceleratorBVH::build (accel.h:115-123) lists the triangles shape by shape,
    // faces in mesh order: primID = face index within its shape.
    s.shape_first.assign(d.shapes, 0);
    s.shape_count.assign(d.shapes, 0);
    s.shape_emitter.assign(d.shapes, -1);
    for (size_t i = 0; i < n; i++) {
        const int32_t sh = s.tri_shape[i];
        if (sh < 0 || sh >= d.shapes || (i > 0 && sh < s.tri_shape[i - 1])) {
            err = "scene descriptor: triangle " + std::to_string(i) + " is not in (shape, face) order";
            return false;
        }
        if (s.shape_count[sh] == 0) s.shape_first[sh] = static_cast<int32_t>(i);
        if (s.tri_prim[i] != s.shape_count[sh]) {
            err = "scene descriptor: triangle " + std::to_string(i) + " has primID " + std::to_string(s.tri_prim[i]) +
                  ", expected its face index " + std::to_string(s.shape_count[sh]);
            return false;
        }
        s.shape_count[sh]++;
        if (s.tri_mat[i] < 0 || s.tri_mat[i] >= d.materials) {
            err = "scene descriptor: triangle " + std::to_string(i) + " has no valid material";
            return false;
        }
    }
    for (int32_t m = 0; m < d.materials; m++) {
        const bdpt_material_desc& md = d.material[m];
        if (md.has_texture) {
            err = "material " + std::to_string(m) + " uses a bitmap texture (not supported)";
            return false;
        }
        Material mt;
        mt.name = "material" + std::to_string(m);
        mt.illum = md.illum;
        for (int k = 0; k < 3; k++) mt.Kd[k] = md.kd[k], mt.Ks[k] = md.ks[k], mt.Ke[k] = md.ke[k], mt.Tf[k] = md.tf[k];
        mt.Ns = md.ns;
        mt.Ni = md.ni;
        s.materials.push_back(mt);
        BsdfRecord b = bsdf_record(mt);
        if (b.kind == BSDF_MIXTURE || b.kind == BSDF_PHONG) {  // the caller's constructed values
            b.scale = md.scale;
            b.specw = md.spec_weight;
        }
        s.bsdfs.push_back(b);
    }
    if (!check_shape_bsdfs(s, err)) return false;
    for (int32_t k = 0; k < d.emitters; k++) {
        const bdpt_emitter_desc& ed = d.emitter[k];
        if (ed.shape < 0 || ed.shape >= d.shapes || s.shape_emitter[ed.shape] >= 0) {
            err = "scene descriptor: emitter " + std::to_string(k) + " names a bad or repeated shape";
            return false;
        }
        if (!ed.cdf || ed.ncdf != s.shape_count[ed.shape] + 1) {
            err = "scene descriptor: emitter " + std::to_string(k) + " needs a CDF of faces + 1 entries";
            return false;
        }
        Emitter em;
        em.shape = ed.shape;
        em.area = ed.area;
        for (int c = 0; c < 3; c++) em.radiance[c] = ed.radiance[c];
        em.cdf.assign(ed.cdf, ed.cdf + ed.ncdf);
        s.shape_emitter[ed.shape] = k;
        s.emitters.push_back(std::move(em));
    }
    // The flattened Fast-BVH (bvh.h:102-105, :147-247): preorder, left child at
    // i + 1, right child at i + rightOffset, leaves (rightOffset 0) covering
    // build_prims[start, start + nPrims). Checked here: the layout, every
    // triangle in exactly one leaf, and every child box inside its parent's box
    // (the nesting the traversal's exactness argument needs).
    const size_t nn = static_cast<size_t>(d.bvh_nodes);
    s.order.assign(d.bvh_order, d.bvh_order + n);
    std::vector<uint8_t> seen(n, 0);
    for (size_t i = 0; i < n; i++) {
        const int32_t t = s.order[i];
        if (t < 0 || static_cast<size_t>(t) >= n || seen[t]) {
            err = "scene descriptor: bvh_order is not a permutation of the triangles";
            return false;
        }
        seen[t] = 1;
    }
    s.nodes.resize(nn);
    for (size_t i = 0; i < nn; i++) {
        const bdpt_bvh_node_desc& b = d.bvh[i];
        FlatNode& f = s.nodes[i];
        for (int a = 0; a < 3; a++) f.bmin[a] = b.bmin[a], f.bmax[a] = b.bmax[a];
        f.start = b.start, f.nprims = b.nprims, f.right_offset = b.right_offset;
    }
    std::fill(seen.begin(), seen.end(), 0);
    std::vector<uint8_t> visited(nn, 0);
    struct Item {
        size_t node;
        int depth;
    };
    std::vector<Item> stack{{0, 0}};
    size_t covered = 0, reached = 0;
    s.max_depth = 0;
    auto inside = [](const FlatNode& c, const FlatNode& p) {
        for (int a = 0; a < 3; a++)
            if (!(c.bmin[a] >= p.bmin[a] && c.bmax[a] <= p.bmax[a])) return false;
        return true;
    };
    while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        if (visited[it.node]) {
            err = "scene descriptor: BVH node reached twice";
            return false;
        }
        visited[it.node] = 1;
        reached++;
        s.max_depth = std::max(s.max_depth, it.depth);
        const FlatNode& f = s.nodes[it.node];
        if (f.right_offset == 0) {
            if (f.nprims == 0 || f.start > n || f.nprims > n - f.start) {
                err = "scene descriptor: BVH leaf " + std::to_string(it.node) + " has a bad triangle range";
                return false;
            }
            for (uint32_t k = 0; k < f.nprims; k++) {
                if (seen[f.start + k]++) {
                    err = "scene descriptor: a triangle is in two BVH leaves";
                    return false;
                }
            }
            covered += f.nprims;
            continue;
        }
        const size_t l = it.node + 1, r = it.node + f.right_offset;
        if (f.right_offset < 2 || r >= nn || l >= nn) {
            err = "scene descriptor: BVH node " + std::to_string(it.node) + " has a bad rightOffset";
            return false;
        }
        if (!inside(s.nodes[l], f) || !inside(s.nodes[r], f)) {
            err = "scene descriptor: BVH node " + std::to_string(it.node) + " has a child box outside its own box";
            return false;
        }
        stack.push_back({r, it.depth + 1});
        stack.push_back({l, it.depth + 1});
    }
    if (covered != n || reached != nn) {
        err = "scene descriptor: the BVH leaves do not cover every triangle once, or nodes are unreachable";
        return false;
    }
    return true;
}

// ------------------------------------------------------------ device layout
bool build_device_layout(const HostScene& s, DeviceLayout& out, std::string& err) {
    const size_t n = s.num_triangles();
    if (n == 0) {
        err = "scene has no triangles";
        return false;
    }
    if (n >= (1u << 28)) {
        err = "more than 2^28 triangles";
        return false;
    }
    auto bits = [](int32_t i) {
        float f;
        std::memcpy(&f, &i, 4);
        return f;
    };
    out = DeviceLayout();
    out.tri.resize(3 * n);
    out.shade.resize(5 * n);
    for (size_t i = 0; i < n; i++) {
        const size_t t = static_cast<size_t>(s.order[i]);
        const int32_t ids[3] = {s.tri_mat[t], s.tri_shape[t], s.tri_prim[t]};
        const float* v = &s.pos[9 * t];
        // v0 and the edges e1 = v1 - v0, e2 = v2 - v0 exactly as rayTriangleIntersect
        // forms them in float (core.h:381-382), so the device test skips 6 subtractions.
        out.tri[3 * i + 0] = {v[0], v[1], v[2], 0.f};
        out.tri[3 * i + 1] = {v[3] - v[0], v[4] - v[1], v[5] - v[2], 0.f};
        out.tri[3 * i + 2] = {v[6] - v[0], v[7] - v[1], v[8] - v[2], 0.f};
        for (int c = 0; c < 3; c++) {
            const float* q = &s.nrm[9 * t + 3 * c];
            out.shade[5 * i + c] = {q[0], q[1], q[2], bits(ids[c])};
        }
        out.shade[5 * i + 3] = {v[3], v[4], v[5], 0.f};
        out.shade[5 * i + 4] = {v[6], v[7], v[8], 0.f};
    }
    // Flat preorder tree -> interior records holding both child boxes.
    std::vector<int32_t> rec(s.nodes.size(), -1);
    int32_t ninterior = 0;
    for (size_t i = 0; i < s.nodes.size(); i++)
        if (s.nodes[i].right_offset != 0) rec[i] = ninterior++;
    auto link_of = [&](size_t i) -> uint32_t {
        const FlatNode& nd = s.nodes[i];
        return nd.right_offset == 0 ? make_leaf_link(nd.start, nd.nprims) : static_cast<uint32_t>(rec[i]);
    };
    out.root_link = link_of(0);
    out.nodes.resize(4 * static_cast<size_t>(ninterior));
    for (size_t i = 0; i < s.nodes.size(); i++) {
        if (rec[i] < 0) continue;
        const FlatNode& a = s.nodes[i + 1];
        const FlatNode& b = s.nodes[i + s.nodes[i].right_offset];
        float4_t* r = &out.nodes[4 * static_cast<size_t>(rec[i])];
        r[0] = {a.bmin[0], a.bmin[1], a.bmin[2], a.bmax[0]};
        r[1] = {a.bmax[1], a.bmax[2], b.bmin[0], b.bmin[1]};
        r[2] = {b.bmin[2], b.bmax[0], b.bmax[1], b.bmax[2]};
        r[3] = {bits(static_cast<int32_t>(link_of(i + 1))), bits(static_cast<int32_t>(link_of(i + s.nodes[i].right_offset))),
                0.f, 0.f};
    }
    // Traversal hierarchy (wide_bvh.hpp): by default a 4-wide SAH tree over single
    // triangles; BDPT_TRAV_TREE=refleaf keeps the reference's leaves as its leaves
    // (the round-1 layout, for comparisons). Both feed the same device code.
    const char* tree_env = std::getenv("BDPT_TRAV_TREE");
    out.tri_tree = !(tree_env && std::string(tree_env) == "refleaf");
    if (out.tri_tree) {
        TriWideBvh tb;
        if (!build_wide_bvh_tris(s.nodes, out.tri, out.shade, kTriBoxPad, tb, err)) return false;
        out.wnodes.swap(tb.bvh.nodes);
        out.wroot_link = tb.bvh.root_link;
        out.wmax_stack = tb.bvh.max_stack;
        out.wdepth = tb.bvh.depth;
        out.wleaves = tb.bvh.leaves;
        out.wtri.swap(tb.tri);
        out.lbox.swap(tb.leaf_box);
        // the padded boxes absorb the compressed records' slab rounding (wide_bvh.hpp)
        out.q_ok = quantize_wide_nodes(out.wnodes, out.qnodes);
        if (!out.q_ok) out.qnodes.clear();
    } else {
        WideBvh wb;
        if (!build_wide_bvh(s.nodes, wb, err)) return false;
        out.wnodes.swap(wb.nodes);
        out.wroot_link = wb.root_link;
        out.wmax_stack = wb.max_stack;
        out.wdepth = wb.depth;
        out.wleaves = wb.leaves;
        out.wtri.resize(3 * n);
        int32_t leaf_id = 0;
        for (const FlatNode& f : s.nodes) {
            if (f.right_offset != 0) continue;
            for (uint32_t k = 0; k < f.nprims; k++) {
                const size_t i = f.start + k;
                out.wtri[3 * i] = {out.tri[3 * i].x, out.tri[3 * i].y, out.tri[3 * i].z, bits(static_cast<int32_t>(i))};
                out.wtri[3 * i + 1] = {out.tri[3 * i + 1].x, out.tri[3 * i + 1].y, out.tri[3 * i + 1].z, bits(leaf_id)};
                out.wtri[3 * i + 2] = out.tri[3 * i + 2];
            }
            out.lbox.push_back({f.bmin[0], f.bmin[1], f.bmin[2], 0.f});
            out.lbox.push_back({f.bmax[0], f.bmax[1], f.bmax[2], 0.f});
            leaf_id++;
        }
        if (s.nodes[0].right_offset == 0) {
            const float inf = __builtin_inff();
            out.lbox[0] = {-inf, -inf, -inf, 0.f};
            out.lbox[1] = {inf, inf, inf, 0.f};
        }
    }
    out.bsdfs = s.bsdfs;
    for (const Emitter& e : s.emitters) {
        EmitterRecord r{};
        r.shape = e.shape;
        r.nfaces = s.shape_count[e.shape];
        r.face_offset = static_cast<int32_t>(out.emit_tri.size() / 5);
        r.cdf_offset = static_cast<int32_t>(out.emit_cdf.size());
        r.area = e.area;
        for (int k = 0; k < 3; k++) r.radiance[k] = e.radiance[k];
        for (int f = 0; f < r.nfaces; f++) {
            const size_t t = static_cast<size_t>(s.shape_first[e.shape] + f);
            const float* p = &s.pos[9 * t];
            const float* q = &s.nrm[9 * t];
            out.emit_tri.push_back({p[0], p[1], p[2], p[3]});
            out.emit_tri.push_back({p[4], p[5], p[6], p[7]});
            out.emit_tri.push_back({p[8], q[0], q[1], q[2]});
            out.emit_tri.push_back({q[3], q[4], q[5], q[6]});
            out.emit_tri.push_back({q[7], q[8], 0.f, 0.f});
        }
        {  // shape center and "radius" (renderer.cpp:295-304, :349-353), float sums in corner order
            float c[3] = {0.f, 0.f, 0.f}, maxx = -__builtin_inff();
            for (int f = 0; f < r.nfaces; f++) {
                const float* p = &s.pos[9 * static_cast<size_t>(s.shape_first[e.shape] + f)];
                for (int k = 0; k < 3; k++) {
                    for (int d = 0; d < 3; d++) c[d] = c[d] + p[3 * k + d];
                    maxx = (maxx < p[3 * k]) ? p[3 * k] : maxx;  // std::max
                }
            }
            const float n = static_cast<float>(3 * r.nfaces);
            for (int d = 0; d < 3; d++) r.center[d] = c[d] / n;
            r.radius = maxx - r.center[0];
        }
        out.emit_cdf.insert(out.emit_cdf.end(), e.cdf.begin(), e.cdf.end());
        out.emitters.push_back(r);
    }
    if (out.emitters.empty()) {
        err = "scene has no emitter (BDPT light subpaths need one)";
        return false;
    }
    out.shape_emitter = s.shape_emitter;
    return true;
}

// ------------------------------------------------------------------ camera
namespace {
struct M4 {
    float m[4][4];  // [col][row]
};
M4 identity() {
    M4 r{};
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
    return r;
}
M4 mul(const M4& a, const M4& b) {  // type_mat4x4.inl:588-606
    M4 r;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 4; i++)
            r.m[c][i] = ((a.m[0][i] * b.m[c][0] + a.m[1][i] * b.m[c][1]) + a.m[2][i] * b.m[c][2]) + a.m[3][i] * b.m[c][3];
    return r;
}
M4 inverse(const M4& M) {  // func_matrix.inl:297-354
    const auto& m = M.m;
    float c00 = m[2][2] * m[3][3] - m[3][2] * m[2][3], c02 = m[1][2] * m[3][3] - m[3][2] * m[1][3],
          c03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float c04 = m[2][1] * m[3][3] - m[3][1] * m[2][3], c06 = m[1][1] * m[3][3] - m[3][1] * m[1][3],
          c07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float c08 = m[2][1] * m[3][2] - m[3][1] * m[2][2], c10 = m[1][1] * m[3][2] - m[3][1] * m[1][2],
          c11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float c12 = m[2][0] * m[3][3] - m[3][0] * m[2][3], c14 = m[1][0] * m[3][3] - m[3][0] * m[1][3],
          c15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float c16 = m[2][0] * m[3][2] - m[3][0] * m[2][2], c18 = m[1][0] * m[3][2] - m[3][0] * m[1][2],
          c19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float c20 = m[2][0] * m[3][1] - m[3][0] * m[2][1], c22 = m[1][0] * m[3][1] - m[3][0] * m[1][1],
          c23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    const float f0[4] = {c00, c00, c02, c03}, f1[4] = {c04, c04, c06, c07}, f2[4] = {c08, c08, c10, c11},
                f3[4] = {c12, c12, c14, c15}, f4[4] = {c16, c16, c18, c19}, f5[4] = {c20, c20, c22, c23};
    const float v0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]}, v1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]},
                v2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]}, v3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    const float sa[4] = {+1, -1, +1, -1}, sb[4] = {-1, +1, -1, +1};
    M4 r;
    for (int i = 0; i < 4; i++) {
        r.m[0][i] = ((v1[i] * f0[i] - v2[i] * f1[i]) + v3[i] * f2[i]) * sa[i];
        r.m[1][i] = ((v0[i] * f0[i] - v2[i] * f3[i]) + v3[i] * f4[i]) * sb[i];
        r.m[2][i] = ((v0[i] * f1[i] - v1[i] * f3[i]) + v3[i] * f5[i]) * sa[i];
        r.m[3][i] = ((v0[i] * f2[i] - v1[i] * f4[i]) + v2[i] * f5[i]) * sb[i];
    }
    const float row0[4] = {r.m[0][0], r.m[1][0], r.m[2][0], r.m[3][0]};
    float d[4];
    for (int i = 0; i < 4; i++) d[i] = m[0][i] * row0[i];
    const float inv_det = 1.f / ((d[0] + d[1]) + (d[2] + d[3]));
    for (auto& col : r.m)
        for (float& x : col) x = x * inv_det;
    return r;
}
void store(const M4& a, float* dst) {
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) dst[4 * c + r] = a.m[c][r];
}
}  // namespace

void camera_constants(const float eye_[3], const float at_[3], const float up_[3], float fov, int width, int height,
                      CameraConstants& out) {
    const F3 eye = load3(eye_), at = load3(at_), up = load3(up_);
    // glm::lookAtRH (gtc/matrix_transform.inl:754-774)
    const F3 f = normalize(at - eye);
    const F3 s = normalize(cross(f, up));
    const F3 u = cross(s, f);
    M4 L = identity();
    L.m[0][0] = s.x, L.m[1][0] = s.y, L.m[2][0] = s.z;
    L.m[0][1] = u.x, L.m[1][1] = u.y, L.m[2][1] = u.z;
    L.m[0][2] = -f.x, L.m[1][2] = -f.y, L.m[2][2] = -f.z;
    L.m[3][0] = -dot(s, eye), L.m[3][1] = -dot(u, eye), L.m[3][2] = dot(f, eye);
    const float deg2rad = 3.14159265358979323846f / 180.f;  // platform.h:50,55
    const float aspect = static_cast<float>(width) / static_cast<float>(height);
    // glm::perspectiveRH_NO (gtc/matrix_transform.inl:343-356), near 1, far 1000
    const float tan_half = std::tan(deg2rad * fov / 2.f);
    M4 P{};
    P.m[0][0] = 1.f / (aspect * tan_half);
    P.m[1][1] = 1.f / tan_half;
    P.m[2][2] = -(1000.f + 1.f) / (1000.f - 1.f);
    P.m[2][3] = -1.f;
    P.m[3][2] = -(2.f * 1000.f * 1.f) / (1000.f - 1.f);
    // scale(I, (W, H, 1)) * scale(I, (0.5, -0.5, 1)) * translate(I, (1, -1, 0))
    const M4 I = identity();
    M4 S1 = I, S2 = I, T = I;
    const float s1[3] = {static_cast<float>(width), static_cast<float>(height), 1.f}, s2[3] = {0.5f, -0.5f, 1.f},
                tr[3] = {1.f, -1.f, 0.f};
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < 4; i++) S1.m[c][i] = I.m[c][i] * s1[c], S2.m[c][i] = I.m[c][i] * s2[c];
    for (int i = 0; i < 4; i++) T.m[3][i] = ((I.m[0][i] * tr[0] + I.m[1][i] * tr[1]) + I.m[2][i] * tr[2]) + I.m[3][i];
    store(L, out.w2c);
    store(inverse(L), out.c2w);
    store(P, out.c2clip);
    store(mul(mul(S1, S2), T), out.ndc2screen);
    out.invW = 1.f / static_cast<float>(width);
    out.invH = 1.f / static_cast<float>(height);
    out.angle = std::tan(deg2rad * fov * 0.5f);
    out.aspect = aspect;
    out.fwd[0] = f.x, out.fwd[1] = f.y, out.fwd[2] = f.z;
    out.vnear = ((1.f / std::tan(deg2rad * fov * 0.5f)) * static_cast<float>(height)) * 0.5f;
}

}  // namespace bdpt
