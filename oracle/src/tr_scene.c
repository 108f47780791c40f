/* TEST INFRASTRUCTURE (oracle): scene ingest restated in C.
 *
 *  - OBJ/MTL parsing + triangulation: tinyobjloader v1.2.0 as vendored by the
 *    reference (externals/tiny_obj_loader.h): tryParseDouble :525-638,
 *    parseTriple :775-827, exportFaceGroupToShape :1018-1261 (ear clipping),
 *    LoadMtl :1273-1657, LoadObj :1756-2116. real_t = float.
 *  - BSDF selection + derived constants: renderer.cpp:258-271,
 *    bsdfs/mixture.h:24-57, bsdfs/glass.h:20-35.
 *  - Emitters + area CDFs: renderer.cpp:279-305, :317-339; math.h:81-112.
 *  - BVH build: externals/bvh.h:147-247 (Fast-BVH, leaf size 4), objects in
 *    (shape, face) order (core/accel.h:115-123).
 *  - Camera constants: renderer.cpp:140-153 with GLM 0.9.9 formulas
 *    (gtc/matrix_transform.inl lookAtRH :754-774, perspectiveRH_NO :343-356,
 *    scale :79-87, translate :11-16; detail/func_matrix.inl compute_inverse
 *    :297-354; detail/type_mat4x4.inl mat*vec :494-540, mat*mat :588-606).
 */
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "tr_internal.h"

static __thread char g_err[512];
const char* tro_last_error(void) { return g_err; }
static void set_err(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

float tr_sqrtf(float x) { return sqrtf(x); }

/* ------------------------------------------------------------ growable arrays */
typedef struct { void* p; size_t n, cap, elt; } vec_t;
static void* vpush(vec_t* v) {
    if (v->n == v->cap) {
        v->cap = v->cap ? v->cap * 2 : 64;
        v->p = realloc(v->p, v->cap * v->elt);
    }
    return (char*)v->p + (v->n++) * v->elt;
}
#define VEC(T) {NULL, 0, 0, sizeof(T)}

static char* read_file(const char* path, size_t* len) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = (char*)malloc((size_t)n + 1);
    if (fread(buf, 1, (size_t)n, f) != (size_t)n) { fclose(f); free(buf); return NULL; }
    buf[n] = 0;
    fclose(f);
    *len = (size_t)n;
    return buf;
}

/* safeGetline (tiny_obj_loader.h:419-451): '\n', '\r\n' and lone '\r' end a line. */
static int next_line(const char* buf, size_t len, size_t* pos, char* out, size_t outcap) {
    if (*pos >= len) return 0;
    size_t o = 0;
    while (*pos < len) {
        char c = buf[(*pos)++];
        if (c == '\n') break;
        if (c == '\r') {
            if (*pos < len && buf[*pos] == '\n') (*pos)++;
            break;
        }
        if (o + 1 < outcap) out[o++] = c;
    }
    out[o] = 0;
    return 1;
}

#define IS_SPACE(x) (((x) == ' ') || ((x) == '\t'))
#define IS_DIGIT(x) ((unsigned)((x) - '0') < 10u)
#define IS_NEW_LINE(x) (((x) == '\r') || ((x) == '\n') || ((x) == '\0'))

/* tryParseDouble (tiny_obj_loader.h:525-638). */
static int try_parse_double(const char* s, const char* s_end, double* result) {
    if (s >= s_end) return 0;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char* curr = s;
    int read = 0;
    int end_not_reached = 0;
    if (*curr == '+' || *curr == '-') {
        sign = *curr;
        curr++;
    } else if (IS_DIGIT(*curr)) {
    } else {
        return 0;
    }
    end_not_reached = (curr != s_end);
    while (end_not_reached && IS_DIGIT(*curr)) {
        mantissa *= 10;
        mantissa += (int)(*curr - 0x30);
        curr++;
        read++;
        end_not_reached = (curr != s_end);
    }
    if (read == 0) return 0;
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            mantissa += (int)(*curr - 0x30) * (read < 8 ? pow_lut[read] : pow(10.0, -read));
            read++;
            curr++;
            end_not_reached = (curr != s_end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = (curr != s_end);
        if (end_not_reached && (*curr == '+' || *curr == '-')) {
            exp_sign = *curr;
            curr++;
        } else if (IS_DIGIT(*curr)) {
        } else {
            return 0;
        }
        read = 0;
        end_not_reached = (curr != s_end);
        while (end_not_reached && IS_DIGIT(*curr)) {
            exponent *= 10;
            exponent += (int)(*curr - 0x30);
            curr++;
            read++;
            end_not_reached = (curr != s_end);
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return 0;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? ldexp(mantissa * pow(5.0, exponent), exponent) : mantissa);
    return 1;
}

/* parseReal (tiny_obj_loader.h:640-648). */
static float parse_real(const char** token, double def) {
    (*token) += strspn(*token, " \t");
    const char* end = (*token) + strcspn(*token, " \t\r");
    double val = def;
    try_parse_double(*token, end, &val);
    *token = end;
    return (float)val;
}

static int parse_int(const char** token) {
    (*token) += strspn(*token, " \t");
    int i = atoi(*token);
    (*token) += strcspn(*token, " \t\r");
    return i;
}

/* fixIndex (tiny_obj_loader.h:459-480). */
static int fix_index(int idx, int n, int* ret) {
    if (idx > 0) { *ret = idx - 1; return 1; }
    if (idx == 0) return 0;
    *ret = n + idx;
    return 1;
}

typedef struct { int v, vn, vt; } vidx_t;

/* parseTriple (tiny_obj_loader.h:775-827). */
static int parse_triple(const char** token, int vsize, int vnsize, int vtsize, vidx_t* ret) {
    vidx_t vi = {-1, -1, -1};
    if (!fix_index(atoi(*token), vsize, &vi.v)) return 0;
    (*token) += strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return 1; }
    (*token)++;
    if ((*token)[0] == '/') {
        (*token)++;
        if (!fix_index(atoi(*token), vnsize, &vi.vn)) return 0;
        (*token) += strcspn(*token, "/ \t\r");
        *ret = vi;
        return 1;
    }
    if (!fix_index(atoi(*token), vtsize, &vi.vt)) return 0;
    (*token) += strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return 1; }
    (*token)++;
    if (!fix_index(atoi(*token), vnsize, &vi.vn)) return 0;
    (*token) += strcspn(*token, "/ \t\r");
    *ret = vi;
    return 1;
}

/* --------------------------------------------------------------------- MTL */
static void init_material(tro_material* m) {
    memset(m, 0, sizeof *m);
    m->Ns = 1.f; /* shininess */
    m->Ni = 1.f; /* ior */
}

typedef struct { char name[128]; int id; } matmap_t;

/* LoadMtl (tiny_obj_loader.h:1273-1657), restricted to the fields the BDPT
 * path reads; any other key only ever writes fields we do not use. */
static void load_mtl(const char* path, vec_t* mats, vec_t* map) {
    size_t len;
    char* buf = read_file(path, &len);
    if (!buf) return;
    tro_material m;
    init_material(&m);
    char line[4096];
    size_t pos = 0;
    while (next_line(buf, len, &pos, line, sizeof line)) {
        size_t L = strlen(line);
        while (L > 0 && (line[L - 1] == ' ' || line[L - 1] == '\t')) line[--L] = 0; /* trailing ws */
        if (L > 0 && line[L - 1] == '\n') line[--L] = 0;
        if (L > 0 && line[L - 1] == '\r') line[--L] = 0;
        if (L == 0) continue;
        const char* t = line + strspn(line, " \t");
        if (t[0] == 0 || t[0] == '#') continue;
        if (!strncmp(t, "newmtl", 6) && IS_SPACE(t[6])) {
            if (m.name[0]) {
                int dup = 0;
                for (size_t i = 0; i < map->n; i++) dup |= !strcmp(((matmap_t*)map->p)[i].name, m.name);
                if (!dup) {
                    matmap_t* e = (matmap_t*)vpush(map);
                    snprintf(e->name, sizeof e->name, "%s", m.name);
                    e->id = (int)mats->n;
                }
                *(tro_material*)vpush(mats) = m;
            }
            init_material(&m);
            snprintf(m.name, sizeof m.name, "%s", t + 7);
            continue;
        }
        if (t[0] == 'K' && t[1] == 'd' && IS_SPACE(t[2])) {
            t += 2;
            for (int i = 0; i < 3; i++) m.Kd[i] = parse_real(&t, 0.0);
            continue;
        }
        if (t[0] == 'K' && t[1] == 's' && IS_SPACE(t[2])) {
            t += 2;
            for (int i = 0; i < 3; i++) m.Ks[i] = parse_real(&t, 0.0);
            continue;
        }
        if ((t[0] == 'K' && t[1] == 't' && IS_SPACE(t[2])) || (t[0] == 'T' && t[1] == 'f' && IS_SPACE(t[2]))) {
            t += 2;
            for (int i = 0; i < 3; i++) m.Tf[i] = parse_real(&t, 0.0);
            continue;
        }
        if (t[0] == 'N' && t[1] == 'i' && IS_SPACE(t[2])) {
            t += 2;
            m.Ni = parse_real(&t, 0.0);
            continue;
        }
        if (t[0] == 'K' && t[1] == 'e' && IS_SPACE(t[2])) {
            t += 2;
            for (int i = 0; i < 3; i++) m.Ke[i] = parse_real(&t, 0.0);
            continue;
        }
        if (t[0] == 'N' && t[1] == 's' && IS_SPACE(t[2])) {
            t += 2;
            m.Ns = parse_real(&t, 0.0);
            continue;
        }
        if (!strncmp(t, "illum", 5) && IS_SPACE(t[5])) {
            t += 6;
            m.illum = parse_int(&t);
            continue;
        }
        if (!strncmp(t, "map_Kd", 6) && IS_SPACE(t[6])) { m.has_diffuse_tex = 1; continue; }
        if (!strncmp(t, "map_Ks", 6) && IS_SPACE(t[6])) { m.has_specular_tex = 1; continue; }
    }
    /* flush last material (unconditionally, :1650-1653) */
    {
        int dup = 0;
        for (size_t i = 0; i < map->n; i++) dup |= !strcmp(((matmap_t*)map->p)[i].name, m.name);
        if (!dup) {
            matmap_t* e = (matmap_t*)vpush(map);
            snprintf(e->name, sizeof e->name, "%s", m.name);
            e->id = (int)mats->n;
        }
        *(tro_material*)vpush(mats) = m;
    }
    free(buf);
}

/* --------------------------------------------------------------------- OBJ */
typedef struct { int v[3], vn[3], mat, shape, prim; } otri_t;
typedef struct { int start, count; int nverts; } oface_t; /* into a flat vidx list */

typedef struct {
    vec_t faces; /* oface_t */
    vec_t fidx;  /* vidx_t  */
} facegroup_t;

/* pnpoly (tiny_obj_loader.h:1004-1015). */
static int pnpoly3(const float* vx, const float* vy, float tx, float ty) {
    int i, j, c = 0;
    for (i = 0, j = 2; i < 3; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    }
    return c;
}

/* exportFaceGroupToShape with triangulate=true (tiny_obj_loader.h:1018-1261).
 * Appends triangles for shape `shape_id` to `tris`; returns 0 if the group is
 * empty (the caller then does not push the shape). */
static int export_face_group(facegroup_t* fg, int material, int shape_id, int* shape_prim, const float* v, size_t vsize,
                             vec_t* tris) {
    if (fg->faces.n == 0) return 0;
    for (size_t fi = 0; fi < fg->faces.n; fi++) {
        oface_t* face = &((oface_t*)fg->faces.p)[fi];
        vidx_t* fv = &((vidx_t*)fg->fidx.p)[face->start];
        size_t npolys = (size_t)face->nverts;
        if (npolys < 3) continue;
        size_t axes[2] = {1, 2};
        for (size_t k = 0; k < npolys; ++k) {
            vidx_t i0 = fv[(k + 0) % npolys], i1 = fv[(k + 1) % npolys], i2 = fv[(k + 2) % npolys];
            size_t vi0 = (size_t)i0.v, vi1 = (size_t)i1.v, vi2 = (size_t)i2.v;
            if (3 * vi0 + 2 >= vsize || 3 * vi1 + 2 >= vsize || 3 * vi2 + 2 >= vsize) continue;
            float v0x = v[vi0 * 3 + 0], v0y = v[vi0 * 3 + 1], v0z = v[vi0 * 3 + 2];
            float v1x = v[vi1 * 3 + 0], v1y = v[vi1 * 3 + 1], v1z = v[vi1 * 3 + 2];
            float v2x = v[vi2 * 3 + 0], v2y = v[vi2 * 3 + 1], v2z = v[vi2 * 3 + 2];
            float e0x = v1x - v0x, e0y = v1y - v0y, e0z = v1z - v0z;
            float e1x = v2x - v1x, e1y = v2y - v1y, e1z = v2z - v1z;
            float cx = fabsf(e0y * e1z - e0z * e1y);
            float cy = fabsf(e0z * e1x - e0x * e1z);
            float cz = fabsf(e0x * e1y - e0y * e1x);
            const float epsilon = 1.19209290e-07f;
            if (cx > epsilon || cy > epsilon || cz > epsilon) {
                if (cx > cy && cx > cz) {
                } else {
                    axes[0] = 0;
                    if (cz > cx && cz > cy) axes[1] = 1;
                }
                break;
            }
        }
        float area = 0;
        for (size_t k = 0; k < npolys; ++k) {
            vidx_t i0 = fv[(k + 0) % npolys], i1 = fv[(k + 1) % npolys];
            size_t vi0 = (size_t)i0.v, vi1 = (size_t)i1.v;
            if (vi0 * 3 + axes[0] >= vsize || vi0 * 3 + axes[1] >= vsize || vi1 * 3 + axes[0] >= vsize ||
                vi1 * 3 + axes[1] >= vsize)
                continue;
            float v0x = v[vi0 * 3 + axes[0]], v0y = v[vi0 * 3 + axes[1]];
            float v1x = v[vi1 * 3 + axes[0]], v1y = v[vi1 * 3 + axes[1]];
            area += (v0x * v1y - v0y * v1x) * 0.5f;
        }
        int maxRounds = 10;
        vidx_t* rem = (vidx_t*)malloc(npolys * sizeof(vidx_t));
        memcpy(rem, fv, npolys * sizeof(vidx_t));
        size_t nrem = npolys;
        size_t guess_vert = 0;
        vidx_t ind[3];
        float vx[3], vy[3];
        while (nrem > 3 && maxRounds > 0) {
            npolys = nrem;
            if (guess_vert >= npolys) {
                maxRounds -= 1;
                guess_vert -= npolys;
            }
            for (size_t k = 0; k < 3; k++) {
                ind[k] = rem[(guess_vert + k) % npolys];
                size_t vi = (size_t)ind[k].v;
                if (vi * 3 + axes[0] >= vsize || vi * 3 + axes[1] >= vsize) {
                    vx[k] = 0.f;
                    vy[k] = 0.f;
                } else {
                    vx[k] = v[vi * 3 + axes[0]];
                    vy[k] = v[vi * 3 + axes[1]];
                }
            }
            float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0];
            float e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
            float cross = e0x * e1y - e0y * e1x;
            if (cross * area < 0.f) {
                guess_vert += 1;
                continue;
            }
            int overlap = 0;
            for (size_t otherVert = 3; otherVert < npolys; ++otherVert) {
                size_t idx = (guess_vert + otherVert) % npolys;
                if (idx >= nrem) continue;
                size_t ovi = (size_t)rem[idx].v;
                if (ovi * 3 + axes[0] >= vsize || ovi * 3 + axes[1] >= vsize) continue;
                float tx = v[ovi * 3 + axes[0]], ty = v[ovi * 3 + axes[1]];
                if (pnpoly3(vx, vy, tx, ty)) {
                    overlap = 1;
                    break;
                }
            }
            if (overlap) {
                guess_vert += 1;
                continue;
            }
            otri_t* t = (otri_t*)vpush(tris);
            for (int k = 0; k < 3; k++) { t->v[k] = ind[k].v; t->vn[k] = ind[k].vn; }
            t->mat = material;
            t->shape = shape_id;
            t->prim = (*shape_prim)++;
            size_t removed = (guess_vert + 1) % npolys;
            while (removed + 1 < npolys) {
                rem[removed] = rem[removed + 1];
                removed += 1;
            }
            nrem--;
        }
        if (nrem == 3) {
            otri_t* t = (otri_t*)vpush(tris);
            for (int k = 0; k < 3; k++) { t->v[k] = rem[k].v; t->vn[k] = rem[k].vn; }
            t->mat = material;
            t->shape = shape_id;
            t->prim = (*shape_prim)++;
        }
        free(rem);
    }
    return 1;
}

/* LoadObj (tiny_obj_loader.h:1756-2116). Shapes are numbered in push order;
 * triangles of a shape that ends up not pushed are dropped (tinyobj quirk). */
static int load_obj(const char* path, vec_t* verts, vec_t* norms, vec_t* tris, vec_t* mats, int* nshapes) {
    size_t len;
    char* buf = read_file(path, &len);
    if (!buf) { set_err("cannot open %s", path); return 0; }
    char basedir[1024];
    snprintf(basedir, sizeof basedir, "%s", path);
    char* slash = strrchr(basedir, '/');
    if (slash) slash[1] = 0; else strcpy(basedir, "./");

    vec_t map = VEC(matmap_t);
    facegroup_t fg = {VEC(oface_t), VEC(vidx_t)};
    int material = -1;
    int shape_id = 0;   /* id the current shape will get if pushed */
    int shape_prim = 0; /* faces already exported into the current shape */
    size_t shape_tri_begin = 0;
    size_t nvt = 0;
    char* line = (char*)malloc(1 << 20);
    size_t pos = 0;
    int ok = 1;
    while (pos < len && next_line(buf, len, &pos, line, 1 << 20)) {
        size_t L = strlen(line);
        if (L > 0 && line[L - 1] == '\n') line[--L] = 0;
        if (L > 0 && line[L - 1] == '\r') line[--L] = 0;
        if (L == 0) continue;
        const char* t = line + strspn(line, " \t");
        if (t[0] == 0 || t[0] == '#') continue;
        if (t[0] == 'v' && IS_SPACE(t[1])) {
            t += 2;
            float* p = (float*)vpush(verts); *p = parse_real(&t, 0.0);
            p = (float*)vpush(verts); *p = parse_real(&t, 0.0);
            p = (float*)vpush(verts); *p = parse_real(&t, 0.0);
            continue;
        }
        if (t[0] == 'v' && t[1] == 'n' && IS_SPACE(t[2])) {
            t += 3;
            for (int i = 0; i < 3; i++) { float* p = (float*)vpush(norms); *p = parse_real(&t, 0.0); }
            continue;
        }
        if (t[0] == 'v' && t[1] == 't' && IS_SPACE(t[2])) {
            nvt += 1;
            continue;
        }
        if (t[0] == 'f' && IS_SPACE(t[1])) {
            t += 2;
            t += strspn(t, " \t");
            oface_t* face = (oface_t*)vpush(&fg.faces);
            face->start = (int)fg.fidx.n;
            face->nverts = 0;
            while (!IS_NEW_LINE(t[0])) {
                vidx_t vi;
                if (!parse_triple(&t, (int)(verts->n / 3), (int)(norms->n / 3), (int)nvt, &vi)) {
                    set_err("Failed parse `f' line in %s", path);
                    ok = 0;
                    goto done;
                }
                *(vidx_t*)vpush(&fg.fidx) = vi;
                ((oface_t*)fg.faces.p)[fg.faces.n - 1].nverts++;
                t += strspn(t, " \t\r");
            }
            continue;
        }
        if (!strncmp(t, "usemtl", 6) && IS_SPACE(t[6])) {
            const char* name = t + 7;
            int nm = -1;
            for (size_t i = 0; i < map.n; i++)
                if (!strcmp(((matmap_t*)map.p)[i].name, name)) nm = ((matmap_t*)map.p)[i].id;
            if (nm != material) {
                export_face_group(&fg, material, shape_id, &shape_prim, (float*)verts->p, verts->n, tris);
                fg.faces.n = fg.fidx.n = 0;
                material = nm;
            }
            continue;
        }
        if (!strncmp(t, "mtllib", 6) && IS_SPACE(t[6])) {
            /* SplitString(token, ' ') then the first readable file wins. */
            char names[4096];
            snprintf(names, sizeof names, "%s", t + 7);
            char* save = NULL;
            char* tok = names;
            /* std::getline-based split keeps empty items; an empty name fails to open. */
            for (;;) {
                char* sp = strchr(tok, ' ');
                if (sp) *sp = 0;
                char full[2048];
                snprintf(full, sizeof full, "%s%s", basedir, tok);
                FILE* f = tok[0] ? fopen(full, "rb") : NULL;
                if (f) {
                    fclose(f);
                    load_mtl(full, mats, &map);
                    break;
                }
                if (!sp) break;
                tok = sp + 1;
            }
            (void)save;
            continue;
        }
        if ((t[0] == 'g' && IS_SPACE(t[1])) || (t[0] == 'o' && IS_SPACE(t[1]))) {
            int ret = export_face_group(&fg, material, shape_id, &shape_prim, (float*)verts->p, verts->n, tris);
            int push = (t[0] == 'g') ? (tris->n > shape_tri_begin) : ret;
            if (push) {
                shape_id++;
                shape_tri_begin = tris->n;
            } else {
                tris->n = shape_tri_begin; /* shape discarded */
            }
            shape_prim = 0;
            fg.faces.n = fg.fidx.n = 0;
            continue;
        }
        /* 't' (tags), 's' (smoothing groups) and unknown commands: ignored. */
    }
    {
        int ret = export_face_group(&fg, material, shape_id, &shape_prim, (float*)verts->p, verts->n, tris);
        if (ret || tris->n > shape_tri_begin) {
            shape_id++;
        } else {
            tris->n = shape_tri_begin;
        }
    }
done:
    *nshapes = shape_id;
    free(line);
    free(buf);
    free(map.p);
    free(fg.faces.p);
    free(fg.fidx.p);
    return ok;
}

/* -------------------------------------------------------------------- BVH */
typedef struct { v3 bmin, bmax, extent; } bbox_t;

/* glm::min / glm::max (detail/func_common.inl:15-28) */
static inline float gmin(float x, float y) { return (y < x) ? y : x; }
static inline float gmax(float x, float y) { return (x < y) ? y : x; }
static inline bbox_t bb_point(v3 p) { bbox_t b = {p, p, vsub(p, p)}; return b; }
static inline void bb_expand_pt(bbox_t* b, v3 p) {
    b->bmin = V3(gmin(b->bmin.x, p.x), gmin(b->bmin.y, p.y), gmin(b->bmin.z, p.z));
    b->bmax = V3(gmax(b->bmax.x, p.x), gmax(b->bmax.y, p.y), gmax(b->bmax.z, p.z));
    b->extent = vsub(b->bmax, b->bmin);
}
static inline void bb_expand_bb(bbox_t* b, const bbox_t* o) {
    b->bmin = V3(gmin(b->bmin.x, o->bmin.x), gmin(b->bmin.y, o->bmin.y), gmin(b->bmin.z, o->bmin.z));
    b->bmax = V3(gmax(b->bmax.x, o->bmax.x), gmax(b->bmax.y, o->bmax.y), gmax(b->bmax.z, o->bmax.z));
    b->extent = vsub(b->bmax, b->bmin);
}
/* BBox::maxDimension (bvh.h:82-87) */
static inline int bb_maxdim(const bbox_t* b) {
    int r = 0;
    if (b->extent.y > b->extent.x) r = 1;
    if (b->extent.z > b->extent.y) r = 2;
    return r;
}
static inline float v3c(v3 v, int d) { return d == 0 ? v.x : d == 1 ? v.y : v.z; }

/* BVHNode::getBBox / getCentroid (accel.h:71-106) */
static bbox_t tri_bbox(const tro_scene* s, int t) {
    const float* p = s->tv + 9 * (size_t)t;
    bbox_t b = bb_point(V3(p[0], p[1], p[2]));
    bb_expand_pt(&b, V3(p[3], p[4], p[5]));
    bb_expand_pt(&b, V3(p[6], p[7], p[8]));
    return b;
}
static v3 tri_centroid(const tro_scene* s, int t) {
    const float* p = s->tv + 9 * (size_t)t;
    v3 c = vadd(vadd(V3(p[0], p[1], p[2]), V3(p[3], p[4], p[5])), V3(p[6], p[7], p[8]));
    return vdivs(c, 3.0f);
}

/* BVH::build (bvh.h:147-247). Centroids/boxes are recomputed from the
 * triangle, as the reference's virtual getters do. */
static void bvh_build(tro_scene* s) {
    int n = s->ntri;
    s->order = (int*)malloc(sizeof(int) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) s->order[i] = i;
    v3* cen = (v3*)malloc(sizeof(v3) * (size_t)(n > 0 ? n : 1));
    bbox_t* tb = (bbox_t*)malloc(sizeof(bbox_t) * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) { cen[i] = tri_centroid(s, i); tb[i] = tri_bbox(s, i); }
    struct { uint32_t parent, start, end, depth; } todo[128];
    int sp = 0;
    todo[sp].start = 0; todo[sp].end = (uint32_t)n; todo[sp].parent = 0xfffffffc; todo[sp].depth = 0;
    sp++;
    vec_t nodes = VEC(tro_node);
    const uint32_t Untouched = 0xffffffff, TouchedTwice = 0xfffffffd;
    uint32_t nNodes = 0;
    s->max_depth = 0;
    while (sp > 0) {
        sp--;
        uint32_t start = todo[sp].start, end = todo[sp].end, parent = todo[sp].parent, depth = todo[sp].depth;
        uint32_t nPrims = end - start;
        nNodes++;
        tro_node node;
        node.start = start;
        node.nprims = nPrims;
        node.right_offset = Untouched;
        bbox_t bb = tb[s->order[start]];
        bbox_t bc = bb_point(cen[s->order[start]]);
        for (uint32_t p = start + 1; p < end; ++p) {
            bb_expand_bb(&bb, &tb[s->order[p]]);
            bb_expand_pt(&bc, cen[s->order[p]]);
        }
        node.bmin[0] = bb.bmin.x; node.bmin[1] = bb.bmin.y; node.bmin[2] = bb.bmin.z;
        node.bmax[0] = bb.bmax.x; node.bmax[1] = bb.bmax.y; node.bmax[2] = bb.bmax.z;
        if (nPrims <= 4) node.right_offset = 0;
        if ((int)depth > s->max_depth) s->max_depth = (int)depth;
        *(tro_node*)vpush(&nodes) = node;
        if (parent != 0xfffffffc) {
            tro_node* pn = &((tro_node*)nodes.p)[parent];
            pn->right_offset--;
            if (pn->right_offset == TouchedTwice) pn->right_offset = nNodes - 1 - parent;
        }
        if (node.right_offset == 0) continue;
        int split_dim = bb_maxdim(&bc);
        float split_coord = .5f * (v3c(bc.bmin, split_dim) + v3c(bc.bmax, split_dim));
        uint32_t mid = start;
        for (uint32_t i = start; i < end; ++i) {
            if (v3c(cen[s->order[i]], split_dim) < split_coord) {
                int tmp = s->order[i]; s->order[i] = s->order[mid]; s->order[mid] = tmp;
                ++mid;
            }
        }
        if (mid == start || mid == end) mid = start + (end - start) / 2;
        todo[sp].start = mid; todo[sp].end = end; todo[sp].parent = nNodes - 1; todo[sp].depth = depth + 1; sp++;
        todo[sp].start = start; todo[sp].end = mid; todo[sp].parent = nNodes - 1; todo[sp].depth = depth + 1; sp++;
    }
    s->nodes = (tro_node*)nodes.p;
    s->nnodes = (int)nNodes;
    free(cen);
    free(tb);
}

/* ------------------------------------------------------------------ scene */
tro_scene* tro_scene_load(const char* obj_path) {
    vec_t verts = VEC(float), norms = VEC(float), tris = VEC(otri_t), mats = VEC(tro_material);
    int nshapes = 0;
    g_err[0] = 0;
    if (!load_obj(obj_path, &verts, &norms, &tris, &mats, &nshapes)) {
        free(verts.p); free(norms.p); free(tris.p); free(mats.p);
        return NULL;
    }
    tro_scene* s = (tro_scene*)calloc(1, sizeof(tro_scene));
    s->ntri = (int)tris.n;
    s->tv = (float*)malloc(sizeof(float) * 9 * (tris.n + 1));
    s->tn = (float*)malloc(sizeof(float) * 9 * (tris.n + 1));
    s->tshape = (int*)malloc(sizeof(int) * (tris.n + 1));
    s->tprim = (int*)malloc(sizeof(int) * (tris.n + 1));
    s->tmat = (int*)malloc(sizeof(int) * (tris.n + 1));
    const float* V = (const float*)verts.p;
    const float* N = (const float*)norms.p;
    int bad = 0;
    for (size_t i = 0; i < tris.n; i++) {
        otri_t* t = &((otri_t*)tris.p)[i];
        for (int c = 0; c < 3; c++) {
            if (t->v[c] < 0 || (size_t)(3 * t->v[c] + 2) >= verts.n) bad = 1;
            if (t->vn[c] < 0 || (size_t)(3 * t->vn[c] + 2) >= norms.n) bad = 2;
            for (int d = 0; d < 3; d++) {
                s->tv[9 * i + 3 * c + d] = bad ? 0.f : V[3 * t->v[c] + d];
                s->tn[9 * i + 3 * c + d] = bad ? 0.f : N[3 * t->vn[c] + d];
            }
        }
        s->tshape[i] = t->shape;
        s->tprim[i] = t->prim;
        s->tmat[i] = t->mat;
        if (t->mat < 0 || (size_t)t->mat >= mats.n) bad = 3;
    }
    s->nmat = (int)mats.n;
    s->mats = (tro_material*)mats.p;
    free(verts.p); free(norms.p); free(tris.p);
    if (bad) {
        set_err(bad == 1 ? "vertex index out of range" : bad == 2 ? "face without a valid normal index"
                                                               : "face without a material");
        tro_scene_free(s);
        return NULL;
    }
    s->nshapes = nshapes;
    s->shape_first = (int*)calloc((size_t)nshapes + 1, sizeof(int));
    s->shape_count = (int*)calloc((size_t)nshapes + 1, sizeof(int));
    s->shape_emitter = (int*)malloc(sizeof(int) * ((size_t)nshapes + 1));
    for (int i = s->ntri - 1; i >= 0; i--) s->shape_first[s->tshape[i]] = i;
    for (int i = 0; i < s->ntri; i++) s->shape_count[s->tshape[i]]++;

    /* BSDFs (renderer.cpp:258-271; constructors in src/bsdfs/*.h). */
    s->bsdf = (tro_bsdf*)calloc((size_t)s->nmat + 1, sizeof(tro_bsdf));
    for (int i = 0; i < s->nmat; i++) {
        const tro_material* m = &s->mats[i];
        tro_bsdf* b = &s->bsdf[i];
        b->emission = V3(m->Ke[0], m->Ke[1], m->Ke[2]);
        b->kd = V3(m->Kd[0], m->Kd[1], m->Kd[2]);
        b->ks = V3(m->Ks[0], m->Ks[1], m->Ks[2]);
        b->tf = V3(m->Tf[0], m->Tf[1], m->Tf[2]);
        b->exponent = m->Ns;
        b->ior = m->Ni;
        b->scale = 1.f;
        if (m->illum == 7) { b->kind = TRB_DIFFUSE; b->type = TRT_DIFFUSE_REFL; }
        else if (m->illum == 3) { b->kind = TRB_MIRROR; b->type = TRT_DELTA_REFL; }
        else if (m->illum == 6) { b->kind = TRB_GLASS; b->type = TRT_DELTA_REFL | TRT_DELTA_TRANS; }
        else if (m->illum == 5) { b->kind = TRB_NULL; b->type = 0; }
        else { b->kind = (m->illum == 8) ? TRB_MIXTURE : TRB_PHONG; b->type = TRT_GLOSSY_REFL | TRT_DIFFUSE_REFL; }
        if (m->has_diffuse_tex || m->has_specular_tex) {
            set_err("material %s uses a bitmap texture (not supported)", m->name);
            tro_scene_free(s);
            return NULL;
        }
        if (b->kind == TRB_MIXTURE || b->kind == TRB_PHONG) {
            /* mixture.h:39-46 / phong.h:39-46 */
            v3 maxValue = vadd(b->ks, b->kd);
            /* std::max(std::max(x, y), z) */
            float actualMax = (maxValue.x < maxValue.y ? maxValue.y : maxValue.x);
            actualMax = (actualMax < maxValue.z ? maxValue.z : actualMax);
            b->scale = actualMax > 1.0f ? 0.99f * (1.0f / actualMax) : 1.0f;
            v3 lum = V3(0.212671f, 0.715160f, 0.072169f);
            float dAvg = vdot(vscale(b->kd, b->scale), lum);
            float sAvg = vdot(vscale(b->ks, b->scale), lum);
            b->specw = sAvg / (dAvg + sAvg);
        }
    }
    /* Emitters (renderer.cpp:279-305; getShapeArea :317-339). */
    s->emit = (tro_emitter*)calloc((size_t)nshapes + 1, sizeof(tro_emitter));
    for (int sh = 0; sh < nshapes; sh++) {
        s->shape_emitter[sh] = -1;
        if (s->shape_count[sh] == 0) continue;
        const tro_bsdf* b = &s->bsdf[s->tmat[s->shape_first[sh]]];
        if (b->kind == TRB_NULL) {
            set_err("shape %d's first face uses a null BSDF (illum 5)", sh);
            tro_scene_free(s);
            return NULL;
        }
        if (vdot(b->emission, b->emission) > 0.f) {
            tro_emitter* e = &s->emit[s->nemit];
            e->shape = sh;
            e->radiance = b->emission;
            e->ncdf = s->shape_count[sh] + 1;
            e->cdf = (float*)malloc(sizeof(float) * (size_t)e->ncdf);
            e->cdf[0] = 0.f;
            for (int f = 0; f < s->shape_count[sh]; f++) {
                const float* p = s->tv + 9 * (size_t)(s->shape_first[sh] + f);
                v3 e1 = vsub(V3(p[3], p[4], p[5]), V3(p[0], p[1], p[2]));
                v3 e2 = vsub(V3(p[6], p[7], p[8]), V3(p[0], p[1], p[2]));
                v3 e3 = vcross(e1, e2);
                e->cdf[f + 1] = e->cdf[f] + 0.5f * sqrtf((e3.x * e3.x + e3.y * e3.y) + e3.z * e3.z);
            }
            e->area = e->cdf[e->ncdf - 1];
            /* shape center and "radius" as the direct integrator reads them (renderer.cpp:295-304, :349-358) */
            v3 c = V3(0.f, 0.f, 0.f);
            float maxx = -INFINITY;
            for (int f = 0; f < s->shape_count[sh]; f++) {
                const float* p = s->tv + 9 * (size_t)(s->shape_first[sh] + f);
                for (int k = 0; k < 3; k++) {
                    c = vadd(c, V3(p[3 * k], p[3 * k + 1], p[3 * k + 2]));
                    maxx = (maxx < p[3 * k]) ? p[3 * k] : maxx; /* std::max */
                }
            }
            e->center = vdivs(c, (float)(3 * s->shape_count[sh]));
            e->radius = maxx - e->center.x;
            float sum = e->cdf[e->ncdf - 1];
            for (int f = 0; f < e->ncdf; f++) e->cdf[f] /= sum;
            s->shape_emitter[sh] = s->nemit;
            s->nemit++;
        }
    }
    bvh_build(s);
    return s;
}

void tro_scene_free(tro_scene* s) {
    if (!s) return;
    free(s->tv); free(s->tn); free(s->tshape); free(s->tprim); free(s->tmat);
    free(s->shape_first); free(s->shape_count); free(s->shape_emitter);
    free(s->mats); free(s->bsdf);
    if (s->emit) for (int i = 0; i < s->nemit; i++) free(s->emit[i].cdf);
    free(s->emit); free(s->order); free(s->nodes);
    free(s);
}

void tro_scene_stats(const tro_scene* s, int64_t out[6]) {
    out[0] = s->ntri; out[1] = s->nnodes; out[2] = s->nshapes; out[3] = s->nmat; out[4] = s->nemit; out[5] = s->max_depth;
}

void tro_scene_dump(const tro_scene* s, float* tf, int32_t* ti, float* nf, uint32_t* nu) {
    for (int i = 0; i < s->ntri; i++) {
        int t = s->order[i];
        memcpy(tf + 18 * (size_t)i, s->tv + 9 * (size_t)t, 9 * sizeof(float));
        memcpy(tf + 18 * (size_t)i + 9, s->tn + 9 * (size_t)t, 9 * sizeof(float));
        ti[3 * i + 0] = s->tshape[t];
        ti[3 * i + 1] = s->tprim[t];
        ti[3 * i + 2] = s->tmat[t];
    }
    for (int i = 0; i < s->nnodes; i++) {
        memcpy(nf + 6 * (size_t)i, s->nodes[i].bmin, 3 * sizeof(float));
        memcpy(nf + 6 * (size_t)i + 3, s->nodes[i].bmax, 3 * sizeof(float));
        nu[3 * i + 0] = s->nodes[i].start;
        nu[3 * i + 1] = s->nodes[i].nprims;
        nu[3 * i + 2] = s->nodes[i].right_offset;
    }
}

/* ----------------------------------------------------------------- camera */
static m4 m4_ident(void) {
    m4 r;
    memset(&r, 0, sizeof r);
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
    return r;
}
/* mat4 * vec4 (type_mat4x4.inl:494-540): (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
v4 tr_m4v4(const m4* m, v4 v) {
    float r[4];
    for (int i = 0; i < 4; i++) {
        float a0 = m->m[0][i] * v.x, a1 = m->m[1][i] * v.y, a2 = m->m[2][i] * v.z, a3 = m->m[3][i] * v.w;
        r[i] = (a0 + a1) + (a2 + a3);
    }
    v4 o = {r[0], r[1], r[2], r[3]};
    return o;
}
/* mat4 * mat4 (type_mat4x4.inl:588-606): ((A0*b0 + A1*b1) + A2*b2) + A3*b3 */
static m4 m4mul(const m4* a, const m4* b) {
    m4 r;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 4; i++)
            r.m[c][i] = ((a->m[0][i] * b->m[c][0] + a->m[1][i] * b->m[c][1]) + a->m[2][i] * b->m[c][2]) +
                        a->m[3][i] * b->m[c][3];
    return r;
}
/* glm::inverse (func_matrix.inl:297-354) */
static m4 m4inverse(const m4* M) {
    float(*m)[4] = (float(*)[4])M->m;
    float Coef00 = m[2][2] * m[3][3] - m[3][2] * m[2][3];
    float Coef02 = m[1][2] * m[3][3] - m[3][2] * m[1][3];
    float Coef03 = m[1][2] * m[2][3] - m[2][2] * m[1][3];
    float Coef04 = m[2][1] * m[3][3] - m[3][1] * m[2][3];
    float Coef06 = m[1][1] * m[3][3] - m[3][1] * m[1][3];
    float Coef07 = m[1][1] * m[2][3] - m[2][1] * m[1][3];
    float Coef08 = m[2][1] * m[3][2] - m[3][1] * m[2][2];
    float Coef10 = m[1][1] * m[3][2] - m[3][1] * m[1][2];
    float Coef11 = m[1][1] * m[2][2] - m[2][1] * m[1][2];
    float Coef12 = m[2][0] * m[3][3] - m[3][0] * m[2][3];
    float Coef14 = m[1][0] * m[3][3] - m[3][0] * m[1][3];
    float Coef15 = m[1][0] * m[2][3] - m[2][0] * m[1][3];
    float Coef16 = m[2][0] * m[3][2] - m[3][0] * m[2][2];
    float Coef18 = m[1][0] * m[3][2] - m[3][0] * m[1][2];
    float Coef19 = m[1][0] * m[2][2] - m[2][0] * m[1][2];
    float Coef20 = m[2][0] * m[3][1] - m[3][0] * m[2][1];
    float Coef22 = m[1][0] * m[3][1] - m[3][0] * m[1][1];
    float Coef23 = m[1][0] * m[2][1] - m[2][0] * m[1][1];
    float Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
    float Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
    float Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
    float Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
    float Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
    float Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
    float Vec0[4] = {m[1][0], m[0][0], m[0][0], m[0][0]};
    float Vec1[4] = {m[1][1], m[0][1], m[0][1], m[0][1]};
    float Vec2[4] = {m[1][2], m[0][2], m[0][2], m[0][2]};
    float Vec3[4] = {m[1][3], m[0][3], m[0][3], m[0][3]};
    float Inv[4][4];
    for (int i = 0; i < 4; i++) {
        Inv[0][i] = (Vec1[i] * Fac0[i] - Vec2[i] * Fac1[i]) + Vec3[i] * Fac2[i];
        Inv[1][i] = (Vec0[i] * Fac0[i] - Vec2[i] * Fac3[i]) + Vec3[i] * Fac4[i];
        Inv[2][i] = (Vec0[i] * Fac1[i] - Vec1[i] * Fac3[i]) + Vec3[i] * Fac5[i];
        Inv[3][i] = (Vec0[i] * Fac2[i] - Vec1[i] * Fac4[i]) + Vec2[i] * Fac5[i];
    }
    const float SignA[4] = {+1, -1, +1, -1}, SignB[4] = {-1, +1, -1, +1};
    m4 r;
    for (int i = 0; i < 4; i++) {
        r.m[0][i] = Inv[0][i] * SignA[i];
        r.m[1][i] = Inv[1][i] * SignB[i];
        r.m[2][i] = Inv[2][i] * SignA[i];
        r.m[3][i] = Inv[3][i] * SignB[i];
    }
    float Row0[4] = {r.m[0][0], r.m[1][0], r.m[2][0], r.m[3][0]};
    float Dot0[4];
    for (int i = 0; i < 4; i++) Dot0[i] = m[0][i] * Row0[i];
    float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    float OneOverDeterminant = 1.f / Dot1;
    for (int c = 0; c < 4; c++)
        for (int i = 0; i < 4; i++) r.m[c][i] = r.m[c][i] * OneOverDeterminant;
    return r;
}

void tr_camera_mats(const tro_params* p, m4* w2c, m4* c2w, m4* c2clip, m4* ndc2screen, float* angle, float* aspect,
                    v3* fwd, float* vnear) {
    v3 eye = V3(p->eye[0], p->eye[1], p->eye[2]);
    v3 at = V3(p->at[0], p->at[1], p->at[2]);
    v3 up = V3(p->up[0], p->up[1], p->up[2]);
    /* lookAtRH (gtc/matrix_transform.inl:754-774) */
    v3 f = vnormalize(vsub(at, eye));
    v3 s = vnormalize(vcross(f, up));
    v3 u = vcross(s, f);
    m4 L = m4_ident();
    L.m[0][0] = s.x; L.m[1][0] = s.y; L.m[2][0] = s.z;
    L.m[0][1] = u.x; L.m[1][1] = u.y; L.m[2][1] = u.z;
    L.m[0][2] = -f.x; L.m[1][2] = -f.y; L.m[2][2] = -f.z;
    L.m[3][0] = -vdot(s, eye);
    L.m[3][1] = -vdot(u, eye);
    L.m[3][2] = vdot(f, eye);
    *w2c = L;
    *c2w = m4inverse(&L);
    const float deg2rad = TR_PI / 180.f;
    *angle = tanf(deg2rad * p->fov * 0.5f);
    *aspect = (float)p->width / (float)p->height;
    /* perspectiveRH_NO (gtc/matrix_transform.inl:343-356), near 1, far 1000 */
    float fovy = deg2rad * p->fov;
    float zNear = 1.f, zFar = 1000.f;
    float tanHalfFovy = tanf(fovy / 2.f);
    m4 P;
    memset(&P, 0, sizeof P);
    P.m[0][0] = 1.f / (*aspect * tanHalfFovy);
    P.m[1][1] = 1.f / tanHalfFovy;
    P.m[2][2] = -(zFar + zNear) / (zFar - zNear);
    P.m[2][3] = -1.f;
    P.m[3][2] = -(2.f * zFar * zNear) / (zFar - zNear);
    *c2clip = P;
    /* scale(I,(W,H,1)) * scale(I,(0.5,-0.5,1)) * translate(I,(1,-1,0)) */
    m4 I = m4_ident();
    m4 S1 = I, S2 = I, T = I;
    float sv1[3] = {(float)p->width, (float)p->height, 1.f}, sv2[3] = {0.5f, -0.5f, 1.f}, tv[3] = {1.f, -1.f, 0.f};
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < 4; i++) { S1.m[c][i] = I.m[c][i] * sv1[c]; S2.m[c][i] = I.m[c][i] * sv2[c]; }
    for (int i = 0; i < 4; i++)
        T.m[3][i] = ((I.m[0][i] * tv[0] + I.m[1][i] * tv[1]) + I.m[2][i] * tv[2]) + I.m[3][i];
    m4 S12 = m4mul(&S1, &S2);
    *ndc2screen = m4mul(&S12, &T);
    *fwd = f; /* glm::normalize(at - o): same expression as lookAt's f */
    *vnear = ((1.f / tanf(deg2rad * p->fov * 0.5f)) * (float)p->height) * 0.5f;
}

void tro_camera(const tro_params* p, float out[72]) {
    m4 a, b, c, d;
    float angle, aspect, vnear;
    v3 fwd;
    tr_camera_mats(p, &a, &b, &c, &d, &angle, &aspect, &fwd, &vnear);
    const m4* ms[4] = {&a, &b, &c, &d};
    int k = 0;
    for (int i = 0; i < 4; i++)
        for (int col = 0; col < 4; col++)
            for (int r = 0; r < 4; r++) out[k++] = ms[i]->m[col][r];
    out[k++] = 1.f / (float)p->width;
    out[k++] = 1.f / (float)p->height;
    out[k++] = angle;
    out[k++] = aspect;
    out[k++] = fwd.x; out[k++] = fwd.y; out[k++] = fwd.z;
    out[k++] = vnear;
}
