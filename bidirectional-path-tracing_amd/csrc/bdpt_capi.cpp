// C-ABI implementation (include/bdpt_amd.h): scene ingest, device context,
// frame and single-sample renders. Host code only; kernels live in
// bdpt_kernels.hip (the BDPT megakernel), sample_state.hip (single-sample
// kernels), pt_kernels.hip (path / direct) and kat_kernels.hip (per-function). No CPU fallback exists: every render runs the HIP kernels.
#include "../../include/bdpt_amd.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "bdpt_device.hpp"
#include "scene.hpp"

namespace bdpt {
hipError_t launch_frame(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                        uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                        hipStream_t stream, void* dparams);
size_t frame_params_bytes();
// sample_state.hip: the single-sample kernels (the caller's std::mt19937 state at sc.mt_ring)
hipError_t launch_sample(const dev::DevScene& sc, const dev::DevFrame& fr, float* splats, float* lvbuf, uint2* gstack,
                         const dev::Ray& ray, float* out, hipStream_t stream);
hipError_t launch_pt_sample(const dev::DevScene& sc, const dev::DevFrame& fr, const int32_t settings[8],
                            float4* levels, uint32_t* ring, uint2* gstack, const dev::Ray& ray, float* out,
                            unsigned long long* counters, hipStream_t stream, void* dparams);
// kat_kernels.hip: per-function entry points
hipError_t launch_bsdf_kat(const dev::DevScene& sc, int mode, int64_t n, const int32_t* mat, const float* wo,
                           const float* x, float* out, hipStream_t st);
hipError_t launch_fresnel_kat(int64_t n, const float* in, float* out, hipStream_t st);
hipError_t launch_triangle_kat(int64_t n, const float* rays, const float* verts, float* out, hipStream_t st);
hipError_t launch_intersect_kat(const dev::DevScene& sc, int64_t n, int occlusion, const float* rays, const float* nrm,
                                const int32_t* otri, uint2* gstack, uint32_t nslots, float* out, hipStream_t st);
hipError_t launch_splat_kat(const dev::DevFrame& fr, int64_t n, const float* p, int32_t* xy, hipStream_t st);
int frame_kernel_lds_stack();
int frame_kernel_blocks_per_cu(size_t dyn_lds);
// bdpt_kernels_deep.hip: the same megakernel for rrDepth > 28
hipError_t launch_frame_deep(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf,
                             uint2* gstack, uint32_t nslots, unsigned long long* work, unsigned long long* counters,
                             int grid, hipStream_t stream, void* dparams);
int frame_kernel_blocks_per_cu_deep(size_t dyn_lds);
// bdpt_kernels_hbm.hip: the same megakernel with the BSDF records in HBM
hipError_t launch_frame_hbm(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                            uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                            hipStream_t stream, void* dparams);
int frame_kernel_blocks_per_cu_hbm(size_t dyn_lds);
// bdpt_kernels_rr.hip: the same megakernel with Russian roulette (NO_RR = 0)
hipError_t launch_frame_rr(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                           uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                           hipStream_t stream, void* dparams);
int frame_kernel_blocks_per_cu_rr(size_t dyn_lds);
// its continuation pass: one wave per sample parked past park_depth bounces (bdpt_kernels.hip, park_lane)
hipError_t launch_chain_rr(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                           uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                           hipStream_t stream, void* dparams);
// bdpt_kernels_rrc.hip: the Russian-roulette megakernel for scenes with glass (lone trapped chains inline)
hipError_t launch_frame_rrc(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                            uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                            hipStream_t stream, void* dparams);
int frame_kernel_blocks_per_cu_rrc(size_t dyn_lds);
hipError_t launch_chain_rrc(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf, uint2* gstack,
                            uint32_t nslots, unsigned long long* work, unsigned long long* counters, int grid,
                            hipStream_t stream, void* dparams);
// bdpt_kernels_split.hip: the same megakernel for short subpaths (no ST_DEFER step)
hipError_t launch_frame_split(const dev::DevScene& sc, const dev::DevFrame& fr, float* fb, float* lvbuf,
                              uint2* gstack, uint32_t nslots, unsigned long long* work, unsigned long long* counters,
                              int grid, hipStream_t stream, void* dparams);
int frame_kernel_blocks_per_cu_split(size_t dyn_lds);
size_t pt_params_bytes();
int pt_blocks_per_cu(size_t dyn_lds);
hipError_t launch_pt(const dev::DevScene& sc, const dev::DevFrame& fr, const int32_t settings[8], float* fb,
                     float4* levels, uint32_t* ring, uint2* gstack, uint32_t nslots, unsigned long long* work,
                     unsigned long long* counters, int grid, hipStream_t stream, void* dparams);
int frame_kernel_block();
int light_vertex_fields();
hipError_t launch_math_check(int32_t fn, const float* x, const float* y, float* out, int64_t n, hipStream_t st);
}  // namespace bdpt

using namespace bdpt;

namespace {
thread_local std::string g_error;

int fail(int code, const std::string& msg) {
    g_error = msg;
    return code;
}

// Debugging knobs that change what a render computes (BDPT_SAMPLE_RANGE: a part
// of the frame; BDPT_GRAZE_CODES=0: the plain near-cull rule, not exact on smooth
// meshes) are read only when BDPT_DEBUG_KNOBS=1 is set too (tools/rr_find.py, A/B
// sweeps); set without it they are ignored with one warning on stderr.
const char* debug_knob(const char* name) {
    const char* v = std::getenv(name);
    if (!v) return nullptr;
    const char* on = std::getenv("BDPT_DEBUG_KNOBS");
    if (on && *on == '1') return v;
    static bool warned = false;
    if (!warned) {
        warned = true;
        std::fprintf(stderr, "bdpt_amd: %s is a debugging knob, ignored without BDPT_DEBUG_KNOBS=1\n", name);
    }
    return nullptr;
}

#define HIP_TRY(expr)                                                                               \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return fail(BDPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

constexpr int kCounterWords = BDPT_NUM_COUNTERS + 3 + 4;  // sums, the counting pass's 3 maxima (Counts::m), the task histogram (Counts::q)
constexpr uint32_t kTaskCap = 256;  // shadow-ray tasks per wave ring (a power of two; DevFrame::tasks)
constexpr int kLazyRrDepth = 28;  // lazy MT19937 covers 10 + 8 * 27 = 226 < 227 draws
// Short subpaths run the BDPT_SPLIT_CONTINUE build (bdpt_kernels_split.hip): the
// ST_DEFER step it removes is one loop slot of the ~(rrDepth + 1)^2 / 2 a sample
// takes, while its separate light / eye continuation bodies cost every shading
// step (measured, DESIGN.md §5: Caustic rrDepth 2 / 3 / 4 / 8: +11.4 / +1.1 / -1.5 / -3.7 %,
// HardLight rrDepth 2 / 3 / 4 / 5: +12.5 / +4.4 / +1.2 / -0.2 %).
// BDPT_SPLIT_MAX_RR overrides the threshold (0: never).
constexpr int kSplitMaxRrDepth = 3;
constexpr int64_t kDeepSceneTris = 262144;  // scenes from this many triangles shade at 36 ready lanes (their walks are longer)
static bool use_split_build(int rr_depth) {
    const char* e = std::getenv("BDPT_SPLIT_MAX_RR");  // read per render (tests force either build)
    return rr_depth <= (e ? std::atoi(e) : kSplitMaxRrDepth);
}
// Russian-roulette continuation pass (bdpt_kernels.hip, park_lane), opt-in: a
// light or eye walk deeper than BDPT_PARK_DEPTH bounces (default 0: off) leaves
// the megakernel for the chain kernel (one wave per sample), which walks its
// delta chain with the whole wave; BDPT_PARK_ROUNDS (default 4) chain + resume
// rounds follow the frame (the last resume keeps every walk in the megakernel).
// Measured slower than walking a lone trapped lane with its own wave inside the
// megakernel (BDPT_COOP_ALONE, the default): Caustic 512^2 x 256 68.6 s vs 45.3 s —
// each round waits for its longest chain, so two long chains of different
// samples that park in different rounds run one after the other.
static int park_depth_setting() {
    const char* e = std::getenv("BDPT_PARK_DEPTH");
    return e ? std::atoi(e) : 0;
}
static int park_rounds_setting() {
    const char* e = std::getenv("BDPT_PARK_ROUNDS");
    return e ? std::max(1, std::atoi(e)) : 4;
}
// One wave per parked walk (grid-stride beyond): a frame parks ~2 400 walks of
// ~180 k bounces on average (Caustic 512^2 x 256), which run side by side.
constexpr int kChainGrid = 8192;
constexpr int kMaxRrDepth = 1024;  // beyond 28 the megakernel continues MT19937 from an HBM ring
// Russian roulette (NO_RR = 0): subpaths are unbounded in the reference (a light
// subpath trapped by total internal reflection in the Caustic sphere was measured
// at 67 714 bounces). Here the light-vertex store of a lane slot holds
// max(kRrLightVerts, rrDepth - 1) vertices (64 B each; the shipped scenes store at
// most 36), and a walk past kRrDepthGuard bounces is a hang guard; a sample that
// meets either is counted (bdpt_stats.capped_samples) and the host render fails
// rather than return a different image.
constexpr int kRrLightVerts = 255;
// A Caustic light subpath trapped in the glass sphere by total internal reflection
// runs for millions of bounces (the oracle over a 512^2 x 256 frame: 2.7 M light /
// 2.1 M eye bounces in one sample); the guard sits an order of magnitude above.
constexpr int kRrDepthGuard = 1 << 25;
}  // namespace

// Error reporting shared with the other C-ABI translation units (exr_io.cpp, toml_config.cpp).
int bdpt::set_error(int code, const std::string& msg) { return fail(code, msg); }

// The state of std::mt19937(seed) after `draws` outputs, as libstdc++'s
// operator<< writes it: _M_x[0..623], then _M_p.
static void mt19937_state(uint32_t seed, int64_t draws, uint32_t st[BDPT_MT19937_WORDS]) {
    std::mt19937 g(seed);
    g.discard(static_cast<unsigned long long>(draws));
    std::ostringstream os;
    os << g;
    std::istringstream is(os.str());
    for (int i = 0; i < BDPT_MT19937_WORDS; i++) {
        unsigned long long v = 0;
        is >> v;
        st[i] = static_cast<uint32_t>(v);
    }
}

struct bdpt_scene {
    HostScene host;
    DeviceLayout layout;
};

struct bdpt_ctx {
    const char* last_kernel = "";  // the frame kernel build the last render launched (bdpt_last_kernel)
    int device = 0;
    int cus = 0;
    int grid = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // scene arrays
    std::vector<void*> allocs;
    dev::DevScene sc{};
    int max_depth = 0;
    bool tri_tree = false;              // traversal boxes padded (wide_bvh.hpp kTriBoxPad)
    int64_t wnode_bytes = 0;            // the 4-wide node array (BDPT_SLAB_SIGN: 32-bit offsets into it)
    double box_lo[3] = {}, box_hi[3] = {};  // scene bounds (the reference BVH's root box)
    int64_t scene_bytes = 0;
    int64_t ntri = 0;  // triangles (shade records)
    uint32_t lds_words_base = 0;  // dynamic LDS words without the emitter faces / CDFs
    // work buffers
    unsigned long long* work = nullptr;      // work counter
    unsigned long long* counters = nullptr;  // kCounters
    float* lv = nullptr;
    size_t lv_floats = 0;
    uint2* gstack = nullptr;  // traversal-stack overflow beyond the LDS part
    uint32_t nslots = 0;
    float* tmp_fb = nullptr;
    size_t tmp_fb_floats = 0;
    float* sample_out = nullptr;
    void* dparams = nullptr;  // kernel parameter block (filled in stream order per launch)
    // path tracer (pt_kernels.hip): level stacks, generator rings, parameter block
    int pt_grid = 0;
    uint32_t pt_nslots = 0;
    float4* pt_levels = nullptr;
    size_t pt_levels_f4 = 0;
    uint32_t* pt_ring = nullptr;
    uint32_t* mt_ring = nullptr;  // BDPT megakernel: MT19937 continuation past 227 draws (rrDepth > 28, RR)
    uint32_t* park = nullptr;     // Russian roulette: continuation records + parked-slot list (DevFrame::park)
    float4* tasks = nullptr;      // per-wave shadow-ray task rings (DevFrame::tasks; read by BDPT_HELP builds)
    uint32_t task_cap = 0;        // their capacity (tasks per wave, a power of two)
    bool has_glass = false;       // a GlassBSDF material: Russian-roulette renders run bdpt_kernels_rrc.hip
    int32_t* row_order = nullptr;  // bdpt_set_row_order (device copy; DevFrame::row_order)
    int32_t row_order_n = 0;       // its row count (0: top to bottom)
    unsigned long long* row_cost = nullptr;  // counting renders: queries per local row (DevFrame::row_cost)
    int32_t row_cost_cap = 0, row_cost_n = 0;  // its capacity; the rows of the last counting render
    unsigned long long work_init = 0;  // BDPT_SAMPLE_RANGE's first sample (host copy for the async upload)
    uint32_t* capped = nullptr;   // samples that met the Russian-roulette bounds, per call
    unsigned long long* diag = nullptr;  // the BDPT frame kernel's timeline (dev::kDiag*)
    bool diag_pending = false;    // the last call was a BDPT frame render (diag is its)
    int wall_khz = 100000;        // s_memrealtime rate
    void* pt_dparams = nullptr;
    // single-sample calls: the caller's std::mt19937 state and the splat list
    uint32_t* mt_state = nullptr;  // BDPT_MT19937_WORDS
    float* splat_list = nullptr;   // header (count, capacity) + capacity (pixel, r, g, b) records
    int32_t splat_cap = 0;
    // cross-stream ordering of the context's buffers: the last call's stream and
    // an event recorded on it after that call's work
    hipEvent_t last_use = nullptr;
    hipStream_t last_stream = nullptr;
    bool used = false;
    // stats of the last render
    bool pending_timing = false;
    bdpt_stats stats{};
};

// Calls on one context are ordered even when they use different streams: a
// call first makes its stream wait for the previous call's work (an event
// recorded at that call's end), since all calls share the context's buffers.
static int begin_use(bdpt_ctx* c, hipStream_t st) {
    if (c->used && c->last_stream != st) HIP_TRY(hipStreamWaitEvent(st, c->last_use, 0));
    return BDPT_OK;
}
static int end_use(bdpt_ctx* c, hipStream_t st) {
    HIP_TRY(hipEventRecord(c->last_use, st));
    c->last_stream = st;
    c->used = true;
    return BDPT_OK;
}

// The BSDF records as the kernels read them. A MixtureBSDF with Ks == 0, scale
// == 1 and a finite exponent >= 0 (so specw == 0) returns DiffuseBSDF's values
// bit for bit (mixture.h:59-151 against diffuse.h:35-61): eval adds
// (0 * (n + 2)) * INV_TWOPI * powf(c, n) = +0 (c in [0, 1], so powf is
// finite) to Kd * INV_PI and multiplies by 1; pdf is pdfPhong * 0 + pdfDiffuse
// * 1 with a finite pdfPhong; sample takes the diffuse branch (u.x < 0 never
// holds) with (u.x - 0) / (1 - 0) == u.x. The kernels run it as diffuse, so a
// wave whose lanes shade both kinds runs one branch instead of two.
// BDPT_KEEP_MIXTURE=1 keeps the record as loaded (the A/B of DESIGN.md).
static std::vector<BsdfRecord> device_bsdfs(const std::vector<BsdfRecord>& in) {
    std::vector<BsdfRecord> out = in;
    const char* keep = std::getenv("BDPT_KEEP_MIXTURE");
    if (keep && *keep == '1') return out;
    for (BsdfRecord& b : out) {
        const bool ks0 = b.ks[0] == 0.f && b.ks[1] == 0.f && b.ks[2] == 0.f;
        if (b.kind == BSDF_MIXTURE && ks0 && b.scale == 1.f && b.specw == 0.f && std::isfinite(b.exponent) &&
            b.exponent >= 0.f)
            b.kind = BSDF_DIFFUSE;  // type keeps the reference's flags (only its delta bits are read)
    }
    return out;
}

// Near-cull exemption margin of a triangle (cull_near_for, bdpt_path.hpp; DESIGN.md
// §2 item 5). The frames exempt a query that leaves a surface at |cos| < kGrazeCos
// to the triangle's GEOMETRIC plane; at run time they only have the interpolated
// shading normal n_s. Every n_s of the triangle is a normalized positive
// combination of its corner normals, so it lies in their cone: if each corner
// normal is within angle th of sgn * n_g (one side of the plane), |n_s - sgn * n_g|
// <= 2 sin(th / 2) and |dot(d, n_g)| < kGrazeCos implies |dot(d, n_s)| < kGrazeCos +
// 2 sin(th / 2). The code is that margin in units of 1/64, rounded up (with 1e-5 for
// the float normalization of n_s); 0 for flat triangles (corner normals parallel to
// n_g: n_s is then n_g's own direction), 255 (always exempt) for corner normals on
// both sides of the plane, zero normals or degenerate triangles.
static uint32_t graze_code(const float* v0, const float* v1, const float* v2, const float* const n[3]) {
    double e1[3], e2[3];
    for (int a = 0; a < 3; a++) e1[a] = double(v1[a]) - v0[a], e2[a] = double(v2[a]) - v0[a];
    double g[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
    const double gl = std::sqrt(g[0] * g[0] + g[1] * g[1] + g[2] * g[2]);
    if (!(gl > 0.0) || !std::isfinite(gl)) return 255u;
    double worst = 0.0;  // max over corners of 2 sin(th / 2) = |n_k - sgn n_g|
    int sgn = 0;
    for (int k = 0; k < 3; k++) {
        const double nl = std::sqrt(double(n[k][0]) * n[k][0] + double(n[k][1]) * n[k][1] + double(n[k][2]) * n[k][2]);
        if (!(nl > 0.0) || !std::isfinite(nl)) return 255u;
        const double c = (n[k][0] * g[0] + n[k][1] * g[1] + n[k][2] * g[2]) / (nl * gl);
        const int s = c > 0.0 ? 1 : c < 0.0 ? -1 : 0;
        if (s == 0 || (sgn != 0 && s != sgn)) return 255u;
        sgn = s;
        worst = std::max(worst, std::sqrt(std::max(0.0, 2.0 - 2.0 * std::fabs(c))));
    }
    if (worst < 1e-9) return 0u;
    const double code = std::ceil((worst + 1e-5) * 64.0);
    return code >= 255.0 ? 255u : static_cast<uint32_t>(code);
}

// The shading records as uploaded (bdpt_types.h kShadeStride): the host five
// (n0, mat) (n1, shape) (n2, prim) (v1) (v2), + (v0) in the wide layout, with the
// triangle's graze code in bits 24..31 of the shape word (shape ids < 2^24).
static std::vector<float4_t> device_shade(const DeviceLayout& L) {
    const char* gz = debug_knob("BDPT_GRAZE_CODES");  // "0": every code 0 (the plain |cos| < 0.02 test; A/B only)
    const bool codes = !(gz && *gz == '0');
    const size_t ntri = L.shade.size() / 5;
    std::vector<float4_t> out(kShadeStride * ntri, float4_t{0.f, 0.f, 0.f, 0.f});
    for (size_t i = 0; i < ntri; i++) {
        for (int q = 0; q < 5; q++) out[kShadeStride * i + q] = L.shade[5 * i + q];
        if (kShadeStride > kShadeV0) out[kShadeStride * i + kShadeV0] = L.tri[3 * i];
        const float4_t* s = &L.shade[5 * i];
        const float v0[3] = {L.tri[3 * i].x, L.tri[3 * i].y, L.tri[3 * i].z};
        const float v1[3] = {s[3].x, s[3].y, s[3].z}, v2[3] = {s[4].x, s[4].y, s[4].z};
        const float n0[3] = {s[0].x, s[0].y, s[0].z}, n1[3] = {s[1].x, s[1].y, s[1].z}, n2[3] = {s[2].x, s[2].y, s[2].z};
        const float* const n[3] = {n0, n1, n2};
        uint32_t shape;
        std::memcpy(&shape, &s[1].w, 4);
        if (codes) shape |= graze_code(v0, v1, v2, n) << 24;
        std::memcpy(&out[kShadeStride * i + 1].w, &shape, 4);
    }
    return out;
}

// The emitter faces as uploaded: 5 float4 per face (v0 v1 v2 n0 n1 n2, 18 floats)
// with the face's graze code in the first free word (the first light ray leaves it).
static std::vector<float4_t> device_emit_tri(const DeviceLayout& L) {
    std::vector<float4_t> out = L.emit_tri;
    for (size_t f = 0; f + 5 <= out.size(); f += 5) {
        float w[20];
        std::memcpy(w, &out[f], sizeof(w));
        const float* const n[3] = {w + 9, w + 12, w + 15};
        const uint32_t code = graze_code(w, w + 3, w + 6, n);
        std::memcpy(&out[f + 4].z, &code, 4);
    }
    return out;
}

extern "C" {

const char* bdpt_last_error(void) { return g_error.c_str(); }
const char* bdpt_version(void) { return "bdpt_amd 0.1 (gfx950 megakernel v0)"; }

int bdpt_scene_load_obj(const char* obj_path, bdpt_scene** out) {
    if (!obj_path || !out) return fail(BDPT_ERR_INVALID, "null argument");
    auto s = std::make_unique<bdpt_scene>();
    std::string err;
    if (!load_obj_scene(obj_path, s->host, err)) return fail(BDPT_ERR_IO, err);
    if (!build_device_layout(s->host, s->layout, err)) return fail(BDPT_ERR_INVALID, err);
    *out = s.release();
    return BDPT_OK;
}

int bdpt_scene_create(const bdpt_scene_desc* desc, bdpt_scene** out) {
    if (!desc || !out) return fail(BDPT_ERR_INVALID, "null argument");
    auto s = std::make_unique<bdpt_scene>();
    std::string err;
    if (!load_desc_scene(*desc, s->host, err)) return fail(BDPT_ERR_INVALID, err);
    if (!build_device_layout(s->host, s->layout, err)) return fail(BDPT_ERR_INVALID, err);
    *out = s.release();
    return BDPT_OK;
}

int bdpt_scene_export_layout(const bdpt_scene* s, int32_t array, void* dst, int64_t* bytes) {
    if (!s || !bytes) return fail(BDPT_ERR_INVALID, "null argument");
    const DeviceLayout& L = s->layout;
    const uint32_t roots[4] = {L.root_link, L.wroot_link, static_cast<uint32_t>(L.wmax_stack),
                               static_cast<uint32_t>(L.wdepth)};
    const void* src = nullptr;
    size_t n = 0;
    std::vector<float4_t> tmp4;
    std::vector<BsdfRecord> tmpb;
    switch (array) {
        case 0: src = L.tri.data(), n = L.tri.size() * 16; break;
        case 1: tmp4 = device_shade(L), src = tmp4.data(), n = tmp4.size() * 16; break;
        case 2: src = L.nodes.data(), n = L.nodes.size() * 16; break;
        case 3: src = L.wnodes.data(), n = L.wnodes.size() * 16; break;
        case 4: src = L.wtri.data(), n = L.wtri.size() * 16; break;
        case 5: src = L.lbox.data(), n = L.lbox.size() * 16; break;
        case 6: tmpb = device_bsdfs(L.bsdfs), src = tmpb.data(), n = tmpb.size() * sizeof(BsdfRecord); break;
        case 7: src = L.emitters.data(), n = L.emitters.size() * sizeof(EmitterRecord); break;
        case 8: tmp4 = device_emit_tri(L), src = tmp4.data(), n = tmp4.size() * 16; break;
        case 9: src = L.emit_cdf.data(), n = L.emit_cdf.size() * 4; break;
        case 10: src = L.shape_emitter.data(), n = L.shape_emitter.size() * 4; break;
        case 11: src = roots, n = sizeof(roots); break;
        case 12: src = L.bsdfs.data(), n = L.bsdfs.size() * sizeof(BsdfRecord); break;
        default: return fail(BDPT_ERR_INVALID, "unknown layout array");
    }
    if (dst) {
        if (*bytes < static_cast<int64_t>(n)) return fail(BDPT_ERR_INVALID, "destination too small");
        if (n) std::memcpy(dst, src, n);
    }
    *bytes = static_cast<int64_t>(n);
    return BDPT_OK;
}

int bdpt_scene_free(bdpt_scene* scene) {
    delete scene;
    return BDPT_OK;
}

int bdpt_scene_get_info(const bdpt_scene* s, bdpt_scene_info* out) {
    if (!s || !out) return fail(BDPT_ERR_INVALID, "null argument");
    out->triangles = static_cast<int64_t>(s->host.num_triangles());
    out->bvh_nodes = static_cast<int64_t>(s->host.nodes.size());
    out->shapes = static_cast<int64_t>(s->host.shape_first.size());
    out->materials = static_cast<int64_t>(s->host.materials.size());
    out->emitters = static_cast<int64_t>(s->host.emitters.size());
    out->bvh_max_depth = s->host.max_depth;
    const DeviceLayout& L = s->layout;
    int64_t leaves = 0;
    for (const FlatNode& n : s->host.nodes) leaves += (n.right_offset == 0);
    out->bvh_leaves = leaves;
    out->wide_nodes = static_cast<int64_t>(L.wnodes.size() / 8);
    out->wide_depth = L.wdepth;
    out->wide_max_stack = L.wmax_stack;
    out->wide_leaves = L.wleaves;
    out->triangle_tree = L.tri_tree ? 1 : 0;
    out->device_bytes = static_cast<int64_t>((L.tri.size() + L.shade.size() + L.nodes.size() + L.wnodes.size() +
                                              L.wtri.size() + L.lbox.size() + L.emit_tri.size()) * 16 +
                                             L.bsdfs.size() * sizeof(BsdfRecord) +
                                             L.emitters.size() * sizeof(EmitterRecord) + L.emit_cdf.size() * 4 +
                                             L.shape_emitter.size() * 4);
    return BDPT_OK;
}

int bdpt_scene_export(const bdpt_scene* s, float* tri_f32, int32_t* tri_i32, float* node_f32, uint32_t* node_u32) {
    if (!s) return fail(BDPT_ERR_INVALID, "null scene");
    const HostScene& h = s->host;
    for (size_t i = 0; i < h.num_triangles(); i++) {
        const size_t t = static_cast<size_t>(h.order[i]);
        if (tri_f32) {
            std::memcpy(tri_f32 + 18 * i, &h.pos[9 * t], 9 * sizeof(float));
            std::memcpy(tri_f32 + 18 * i + 9, &h.nrm[9 * t], 9 * sizeof(float));
        }
        if (tri_i32) {
            tri_i32[3 * i] = h.tri_shape[t];
            tri_i32[3 * i + 1] = h.tri_prim[t];
            tri_i32[3 * i + 2] = h.tri_mat[t];
        }
    }
    for (size_t i = 0; i < h.nodes.size(); i++) {
        if (node_f32) {
            std::memcpy(node_f32 + 6 * i, h.nodes[i].bmin, 3 * sizeof(float));
            std::memcpy(node_f32 + 6 * i + 3, h.nodes[i].bmax, 3 * sizeof(float));
        }
        if (node_u32) {
            node_u32[3 * i] = h.nodes[i].start;
            node_u32[3 * i + 1] = h.nodes[i].nprims;
            node_u32[3 * i + 2] = h.nodes[i].right_offset;
        }
    }
    return BDPT_OK;
}

int bdpt_scene_export_traversal(const bdpt_scene* s, float* wnodes, float* wtri, float* lbox, uint32_t* root_link) {
    if (!s) return fail(BDPT_ERR_INVALID, "null scene");
    const DeviceLayout& L = s->layout;
    if (wnodes) std::memcpy(wnodes, L.wnodes.data(), L.wnodes.size() * sizeof(float4_t));
    if (wtri) std::memcpy(wtri, L.wtri.data(), L.wtri.size() * sizeof(float4_t));
    if (lbox) std::memcpy(lbox, L.lbox.data(), L.lbox.size() * sizeof(float4_t));
    if (root_link) *root_link = L.wroot_link;
    return BDPT_OK;
}

int bdpt_camera_constants(const bdpt_camera* cam, int32_t width, int32_t height, float out[72]) {
    if (!cam || !out || width <= 0 || height <= 0) return fail(BDPT_ERR_INVALID, "bad camera arguments");
    CameraConstants c;
    camera_constants(cam->eye, cam->at, cam->up, cam->fov, width, height, c);
    std::memcpy(out, &c, sizeof(c));
    return BDPT_OK;
}

int bdpt_device_count(int32_t* count) {
    if (!count) return fail(BDPT_ERR_INVALID, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *count = n;
    return BDPT_OK;
}

static int upload(bdpt_ctx* c, const void* src, size_t bytes, void** dst) {
    if (bytes == 0) bytes = 16;
    HIP_TRY(hipMalloc(dst, bytes));
    c->allocs.push_back(*dst);
    if (src) HIP_TRY(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    c->scene_bytes += static_cast<int64_t>(bytes);
    return BDPT_OK;
}

int bdpt_ctx_destroy(bdpt_ctx* c) {
    if (!c) return BDPT_OK;
    (void)hipSetDevice(c->device);
    // Teardown is best effort: errors here cannot be acted on by the caller.
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (void* p : c->allocs) (void)hipFree(p);
    for (void* p : {static_cast<void*>(c->work), static_cast<void*>(c->counters), static_cast<void*>(c->lv),
                    static_cast<void*>(c->gstack), static_cast<void*>(c->tmp_fb), static_cast<void*>(c->sample_out), c->dparams,
                    static_cast<void*>(c->pt_levels), static_cast<void*>(c->pt_ring), c->pt_dparams,
                    static_cast<void*>(c->mt_ring), static_cast<void*>(c->mt_state), static_cast<void*>(c->capped),
                    static_cast<void*>(c->diag),
                    static_cast<void*>(c->splat_list), static_cast<void*>(c->park), static_cast<void*>(c->tasks),
                    static_cast<void*>(c->row_order), static_cast<void*>(c->row_cost)})
        if (p) (void)hipFree(p);
    if (c->last_use) (void)hipEventDestroy(c->last_use);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return BDPT_OK;
}

int bdpt_ctx_create(const bdpt_scene* s, int32_t hip_device, bdpt_ctx** out) {
    if (!s || !out) return fail(BDPT_ERR_INVALID, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(BDPT_ERR_NO_DEVICE, "no HIP device available");
    if (hip_device < 0 || hip_device >= n) return fail(BDPT_ERR_INVALID, "hip_device out of range");
    auto c = std::make_unique<bdpt_ctx>();
    c->device = hip_device;
    HIP_TRY(hipSetDevice(hip_device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, hip_device));
    c->cus = prop.multiProcessorCount;
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&c->ev0));
    HIP_TRY(hipEventCreate(&c->ev1));
    HIP_TRY(hipEventCreateWithFlags(&c->last_use, hipEventDisableTiming));
    const DeviceLayout& L = s->layout;
    void* p;
    int rc;
    if ((rc = upload(c.get(), L.tri.data(), L.tri.size() * 16, &p))) return rc;
    c->sc.tri = static_cast<const float4*>(p);
    if (s->host.shape_first.size() >= (size_t(1) << 24))
        return fail(BDPT_ERR_UNSUPPORTED, "more than 2^24 shapes (the shading record packs the shape id in 24 bits)");
    c->ntri = static_cast<int64_t>(L.shade.size() / 5);
    {  // the device shade records (bdpt_types.h kShadeStride): the host five + v0, one line each
        const std::vector<float4_t> dev_shade = device_shade(L);
        if ((rc = upload(c.get(), dev_shade.data(), dev_shade.size() * 16, &p))) return rc;
    }
    c->sc.shade = static_cast<const float4*>(p);
    if ((rc = upload(c.get(), L.nodes.data(), L.nodes.size() * 16, &p))) return rc;
    c->sc.nodes = static_cast<const float4*>(p);
    if ((rc = upload(c.get(), L.wnodes.data(), L.wnodes.size() * 16, &p))) return rc;
    c->sc.wnodes = static_cast<const float4*>(p);
    c->sc.wroot_link = L.wroot_link;
    c->sc.qnodes = nullptr;
    c->sc.q_ok = 0u;
    if (L.q_ok) {
        if ((rc = upload(c.get(), L.qnodes.data(), L.qnodes.size() * 16, &p))) return rc;
        c->sc.qnodes = static_cast<const float4*>(p);
        c->sc.q_ok = 1u;
    }
    if ((rc = upload(c.get(), L.wtri.data(), L.wtri.size() * 16, &p))) return rc;
    c->sc.wtri = static_cast<const float4*>(p);
    if ((rc = upload(c.get(), L.lbox.data(), L.lbox.size() * 16, &p))) return rc;
    c->sc.lbox = static_cast<const float4*>(p);
    {
        const std::vector<BsdfRecord> dev_bsdfs = device_bsdfs(L.bsdfs);
        if ((rc = upload(c.get(), dev_bsdfs.data(), dev_bsdfs.size() * sizeof(BsdfRecord), &p))) return rc;
        for (const BsdfRecord& b : dev_bsdfs) c->has_glass = c->has_glass || b.kind == BSDF_GLASS;
    }
    c->sc.bsdf = static_cast<const BsdfRecord*>(p);
    if ((rc = upload(c.get(), L.emitters.data(), L.emitters.size() * sizeof(EmitterRecord), &p))) return rc;
    c->sc.emit = static_cast<const EmitterRecord*>(p);
    {
        const std::vector<float4_t> dev_etri = device_emit_tri(L);
        if ((rc = upload(c.get(), dev_etri.data(), dev_etri.size() * 16, &p))) return rc;
    }
    c->sc.emit_tri = static_cast<const float4*>(p);
    if ((rc = upload(c.get(), L.emit_cdf.data(), L.emit_cdf.size() * 4, &p))) return rc;
    c->sc.emit_cdf = static_cast<const float*>(p);
    if ((rc = upload(c.get(), L.shape_emitter.data(), L.shape_emitter.size() * 4, &p))) return rc;
    c->sc.shape_emitter = static_cast<const int32_t*>(p);
    c->sc.root_link = L.root_link;
    c->sc.node_slack = 1u;  // per render: node_slack_needed
    c->tri_tree = L.tri_tree;
    c->wnode_bytes = static_cast<int64_t>(L.wnodes.size()) * 16;
    for (int a = 0; a < 3; a++) c->box_lo[a] = s->host.nodes[0].bmin[a], c->box_hi[a] = s->host.nodes[0].bmax[a];
    {  // the region whose queries the culled, padded traversal tree serves (DevScene::near_lo/hi)
        double diag2 = 0.0;
        for (int a = 0; a < 3; a++) diag2 += (c->box_hi[a] - c->box_lo[a]) * (c->box_hi[a] - c->box_lo[a]);
        const double grow = 100.0 * std::sqrt(diag2);
        for (int a = 0; a < 3; a++) {
            const double lo = c->box_lo[a] - grow, hi = c->box_hi[a] + grow;
            c->sc.near_lo[a] = std::isfinite(lo) ? static_cast<float>(lo) : -__builtin_inff();
            c->sc.near_hi[a] = std::isfinite(hi) ? static_cast<float>(hi) : __builtin_inff();
        }
    }
    c->sc.mt_ring = nullptr;
    c->sc.mt_ring_stride = 0;
    c->sc.nemit = static_cast<int32_t>(L.emitters.size());
    c->sc.inv_nemit = 1.f / static_cast<float>(c->sc.nemit);  // the device's 1.f / nemit, bit for bit
    c->sc.nbsdf = static_cast<int32_t>(L.bsdfs.size());
    c->sc.nshapes = static_cast<int32_t>(L.shape_emitter.size());
    {  // LDS table layout (bdpt_device.hpp scene_tables_to_lds), 16-byte aligned parts
        auto up4 = [](uint32_t w) { return (w + 3u) & ~3u; };
        constexpr uint32_t kBudget = 24u * 1024u;
        const uint32_t nb = static_cast<uint32_t>(L.bsdfs.size() * sizeof(BsdfRecord) / 4);
        const uint32_t ne = static_cast<uint32_t>(L.emitters.size() * sizeof(EmitterRecord) / 4);
        // BSDF records in LDS unless they do not fit with the emitter records (then
        // the frame renders run bdpt_kernels_hbm.hip); BDPT_BSDF_IN_HBM=1 forces
        // HBM (tests of that build on small scenes).
        const char* force = std::getenv("BDPT_BSDF_IN_HBM");
        const bool hbm = (force && *force == '1') || (up4(up4(dev::kLdsHdr + nb) + ne) * 4u > kBudget);
        c->sc.lds_bsdf_off = hbm ? dev::kNoLds : dev::kLdsHdr;
        c->sc.lds_emit_off = hbm ? dev::kLdsHdr : up4(dev::kLdsHdr + nb);
        c->sc.lds_shape_off = up4(c->sc.lds_emit_off + ne);
        c->sc.lds_words = up4(c->sc.lds_shape_off + static_cast<uint32_t>(L.shape_emitter.size()));
        if (c->sc.lds_words * 4u > kBudget) {  // many shapes: their emitter map stays in HBM
            c->sc.lds_words = c->sc.lds_shape_off;
            c->sc.lds_shape_off = dev::kNoLds;
        }
        if (c->sc.lds_words * 4u > kBudget)
            return fail(BDPT_ERR_UNSUPPORTED, "emitter records exceed the 24 KiB LDS budget");
        // Emitter faces + CDFs join the LDS tables when that costs no resident block.
        c->sc.lds_etri_off = c->sc.lds_ecdf_off = dev::kNoLds;
        c->sc.n_etri = static_cast<int32_t>(L.emit_tri.size() / 5);
        c->sc.n_ecdf = static_cast<int32_t>(L.emit_cdf.size());
        c->lds_words_base = c->sc.lds_words;
        const uint32_t etri = c->sc.lds_words, ecdf = up4(etri + 20u * static_cast<uint32_t>(c->sc.n_etri));
        const uint32_t with = up4(ecdf + static_cast<uint32_t>(c->sc.n_ecdf));
        auto blocks = [&](uint32_t words) {
            const size_t bytes = 4 * static_cast<size_t>(words);
            return hbm ? frame_kernel_blocks_per_cu_hbm(bytes) : frame_kernel_blocks_per_cu(bytes);
        };
        if (with * 4u <= kBudget && blocks(with) >= blocks(c->sc.lds_words)) {
            c->sc.lds_etri_off = etri;
            c->sc.lds_ecdf_off = ecdf;
            c->sc.lds_words = with;
        }
    }
    c->max_depth = s->host.max_depth;
    HIP_TRY(hipMalloc(&c->work, sizeof(unsigned long long)));
    HIP_TRY(hipMalloc(&c->counters, sizeof(unsigned long long) * kCounterWords));
    HIP_TRY(hipMalloc(&c->diag, sizeof(unsigned long long) * dev::kDiagWords));
    {
        int khz = 0;
        if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device) == hipSuccess && khz > 0)
            c->wall_khz = khz;
    }
    HIP_TRY(hipMalloc(&c->sample_out, 16 * sizeof(float)));
    HIP_TRY(hipMalloc(&c->capped, sizeof(uint32_t)));
    HIP_TRY(hipMemset(c->capped, 0, sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&c->dparams, frame_params_bytes()));
    // Persistent grid: exactly the resident blocks (no co-residency is assumed:
    // the work queue has no inter-block waits, extra blocks would just queue).
    const size_t dyn = 4 * static_cast<size_t>(c->sc.lds_words);
    c->grid = c->cus * (c->sc.lds_bsdf_off == dev::kNoLds ? frame_kernel_blocks_per_cu_hbm(dyn)
                                                          : frame_kernel_blocks_per_cu(dyn));
    c->nslots = static_cast<uint32_t>(c->grid * frame_kernel_block());
    // Traversal stack: worst case of either tree (binary: depth + 1 pending
    // right children; 4-wide: the host-computed bound), the part beyond the
    // kernel's LDS entries in HBM.
    const int depth = std::max(s->host.max_depth + 2, L.wmax_stack + 1);
    const int lds_entries = frame_kernel_lds_stack();
    c->sc.gdepth = static_cast<uint32_t>(std::max(1, depth - lds_entries));  // per slot (DevScene::gdepth)
    const size_t spill_mega = static_cast<size_t>(c->sc.gdepth) * c->nslots;
    HIP_TRY(hipMalloc(&c->gstack, sizeof(uint2) * std::max<size_t>(1, spill_mega)));
    // shadow-ray task rings, one per wave of the persistent grid (4096 waves x 256 x 48 B = 50 MB on
    // 256 CUs); only builds with BDPT_HELP read them
    c->task_cap = kTaskCap;
    if (const char* e = std::getenv("BDPT_TASK_CAP")) {  // (sweeps) a power of two in [64, 4096]
        const int v = std::atoi(e);
        if (v >= 64 && v <= 4096 && (v & (v - 1)) == 0) c->task_cap = static_cast<uint32_t>(v);
    }
    HIP_TRY(hipMalloc(&c->tasks, sizeof(float4) * 3 * c->task_cap * (c->nslots / 64)));
    *out = c.release();
    return BDPT_OK;
}

static int check_params(const bdpt_frame_params* p) {
    if (!p) return fail(BDPT_ERR_INVALID, "null params");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return fail(BDPT_ERR_INVALID, "width/height/spp must be > 0");
    if (static_cast<int64_t>(p->width) * p->height >= (1ll << 31))
        return fail(BDPT_ERR_INVALID, "image too large (W*H must fit int32, as in the reference)");
    if (p->rr_depth < 1 || p->rr_depth > kMaxRrDepth)
        return fail(BDPT_ERR_UNSUPPORTED, "rr_depth must be in [1, 1024]");
    if (p->flags & ~(BDPT_FLAG_COUNT | BDPT_FLAG_FULL_TRAVERSAL))
        return fail(BDPT_ERR_UNSUPPORTED, "unknown flag (bit 2, the round-1 wavefront schedule, was removed)");
    if (p->strategy < 0 || p->strategy > 2) return fail(BDPT_ERR_INVALID, "unknown strategy");
    if (p->row_stride < 1 || p->row_offset < 0) return fail(BDPT_ERR_INVALID, "bad row shard");
    if (p->russian_roulette != BDPT_RR_NONE && p->russian_roulette != BDPT_RR_LUMINANCE)
        return fail(BDPT_ERR_INVALID, "unknown russian_roulette mode");
    return BDPT_OK;
}

constexpr int kExpressDepth = 512;  // Russian roulette: express mode past this many bounces
static dev::DevFrame make_frame(const bdpt_frame_params* p) {
    dev::DevFrame fr{};
    camera_constants(p->camera.eye, p->camera.at, p->camera.up, p->camera.fov, p->width, p->height, fr.cam);
    for (int i = 0; i < 3; i++) fr.cam_o[i] = p->camera.eye[i];
    fr.W = p->width, fr.H = p->height, fr.spp = p->spp, fr.rr_depth = p->rr_depth, fr.strategy = p->strategy;
    fr.seed_base = p->seed_base;
    fr.row_offset = p->row_offset, fr.row_stride = p->row_stride;
    fr.nrows = p->row_offset >= p->height ? 0 : (p->height - p->row_offset + p->row_stride - 1) / p->row_stride;
    fr.flags = p->flags;
    fr.total_samples = static_cast<uint64_t>(fr.nrows) * static_cast<uint64_t>(p->width) * p->spp;
    fr.rr_mode = p->russian_roulette == BDPT_RR_LUMINANCE ? 1 : 0;
    fr.depth_cap = fr.rr_mode ? kRrDepthGuard : p->rr_depth;
    fr.lv_max = fr.rr_mode ? std::max(kRrLightVerts, p->rr_depth - 1) : std::max(p->rr_depth - 1, 1);
    fr.inv_spp = 1.f / static_cast<float>(fr.spp);  // IEEE divisions: the bits of the device's rcp_cr
    fr.inv_pixels = 1.f / static_cast<float>(fr.W * fr.H);
    fr.capped = nullptr;  // the context's word, set by the caller
    fr.diag = nullptr;    // the context's timeline, set by bdpt_render
    // Russian-roulette schedule (bdpt_kernels.hip express mode): BDPT_EXPRESS_DEPTH and
    // BDPT_COOP_GROUPS=0 override the build's depth and grouped walks (tests reach the
    // grouped and turn-taking walks on small frames this way; the results are the same)
    fr.express_depth = kExpressDepth;
    if (const char* e = std::getenv("BDPT_EXPRESS_DEPTH")) fr.express_depth = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("BDPT_COOP_GROUPS")) fr.sched_flags |= *e == '0' ? dev::kSchedNoCoopGroups : 0u;
    return fr;
}

static int ensure_lv(bdpt_ctx* c, int lv_max, uint32_t nslots) {
    const size_t need = static_cast<size_t>(std::max(lv_max, 1)) * light_vertex_fields() * nslots;
    if (need > c->lv_floats) {
        if (c->lv) HIP_TRY(hipFree(c->lv));
        c->lv = nullptr;
        HIP_TRY(hipMalloc(&c->lv, need * sizeof(float)));
        c->lv_floats = need;
    }
    return BDPT_OK;
}

// Interior boxes of the triangle traversal tree are padded by kTriBoxPad x the
// scene diagonal (wide_bvh.hpp), so a ray that hits a triangle passes through
// every box above it over a t-interval of at least 2 pad; slab_fast's rounding
// (RN(1/d), three roundings per plane: < 3.6e-7 (|tn| + |tf|)) can only close
// that interval for boxes more than ~280 diagonals away along the ray. Every
// query of a BDPT frame starts inside the scene box or at the camera, so when
// the camera is within 100 diagonals of the scene the plain tn <= tf test is
// conservative and the ambiguity slack is skipped. Other rays
// (bdpt_intersect's, the refleaf tree's unpadded boxes) keep it.
//
// BDPT_SLAB_FMA builds test those boxes by one fma per plane (slab_fma), whose
// error also grows with the origin's distance from 0 (2^-24 |o_i| per plane in
// scene units): they skip the slack only while the origins and the scene box
// also lie within kFmaCoordDiags diagonals of 0, where the per-plane error,
// 2^-23 · 101 + 2^-24 · 300 < 3e-5 diagonals, stays below slab_fast's own bound
// at 100 diagonals (3.6e-7 · 202 = 7.3e-5) and far inside the padding.
constexpr double kFmaCoordDiags = 300.0;
static uint32_t node_slack_needed(const bdpt_ctx* c, const float* const* origins, int n) {
    if (!c->tri_tree) return 1u;
    double diag2 = 0.0;
    for (int a = 0; a < 3; a++) diag2 += (c->box_hi[a] - c->box_lo[a]) * (c->box_hi[a] - c->box_lo[a]);
    if (!(diag2 > 0.0) || !std::isfinite(diag2)) return 1u;
    // BDPT_SLAB_SIGN builds address the node planes by 32-bit offsets (load_wnode_nf)
    if (BDPT_SLAB_SIGN && c->wnode_bytes >= (int64_t{1} << 32)) return 1u;
    constexpr bool kFmaPlanes = BDPT_SLAB_FMA != 0 || BDPT_SLAB_SIGN != 0;
    const double coord_max = kFmaPlanes ? kFmaCoordDiags * std::sqrt(diag2) : HUGE_VAL;
    for (int a = 0; a < 3; a++)
        if (!(std::fabs(c->box_lo[a]) <= coord_max && std::fabs(c->box_hi[a]) <= coord_max)) return 1u;
    for (int k = 0; k < n; k++) {
        double far2 = 0.0;  // squared distance to the farthest corner of the scene box
        for (int a = 0; a < 3; a++) {
            const double o = origins[k][a];
            const double d = std::max(std::fabs(o - c->box_lo[a]), std::fabs(o - c->box_hi[a]));
            far2 += d * d;
            if (!(std::fabs(o) <= coord_max)) return 1u;
        }
        if (!std::isfinite(far2) || far2 > 1.0e4 * diag2) return 1u;
    }
    return 0u;
}

int bdpt_render(bdpt_ctx* c, const bdpt_frame_params* p, float* fb, void* hip_stream) {
    if (!c || !fb) return fail(BDPT_ERR_INVALID, "null argument");
    int rc = check_params(p);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    dev::DevFrame fr = make_frame(p);
    fr.capped = c->capped;
    fr.tasks = c->tasks;
    fr.task_cap = c->task_cap;
    if (c->row_order_n) {
        if (c->row_order_n != fr.nrows)
            return fail(BDPT_ERR_INVALID, "the row order set by bdpt_set_row_order has " + std::to_string(c->row_order_n) +
                                              " rows, the shard " + std::to_string(fr.nrows));
        fr.row_order = c->row_order;
    }
    const bool hbm = c->sc.lds_bsdf_off == dev::kNoLds;
    const bool rr = fr.rr_mode != 0;
    const float* eye[1] = {p->camera.eye};
    if (hbm && (p->rr_depth > kLazyRrDepth || rr))
        return fail(BDPT_ERR_UNSUPPORTED, "rr_depth > 28 or Russian roulette with BSDF records in HBM (too many "
                                          "materials for the LDS table) is not built");
    if ((rc = ensure_lv(c, fr.lv_max, c->nslots))) return rc;
    // Shading threshold of the frame kernels: a scene whose tree is deep (from
    // kDeepSceneTris triangles: longer walks) shades at 36 ready lanes, others at 44
    // (round 5, r5m / r5ag: synth1m 1024^2x64 191.8 vs 188.5 Msamples/s at 40 / 44,
    // then 205.6 / 205.1 / 205.2 at 36 vs 203.8 / 203.3 / 204.6 at 40; Caustic and
    // HardLight 0.3-0.8 % slower below 44). BDPT_SHADE_READY overrides it (sweeps).
    fr.shade_ready = c->ntri >= kDeepSceneTris ? 36 : 44;
    if (const char* e = std::getenv("BDPT_SHADE_READY")) fr.shade_ready = std::max(1, std::min(64, std::atoi(e)));
    dev::DevScene sc = c->sc;
    sc.node_slack = node_slack_needed(c, eye, 1);
    if (p->rr_depth > kLazyRrDepth || rr) {  // draws past 226: the lanes' MT19937 rings
        if (!c->mt_ring) HIP_TRY(hipMalloc(&c->mt_ring, sizeof(uint32_t) * kMtRingSlotWords * static_cast<size_t>(c->nslots)));
        sc.mt_ring = c->mt_ring;
        sc.mt_ring_stride = 1;  // slot-major blocks of kMtRingSlotWords words (DevScene::mt_ring)
    }
    if ((rc = begin_use(c, st))) return rc;
    HIP_TRY(hipMemsetAsync(c->work, 0, sizeof(unsigned long long), st));
    // BDPT_SAMPLE_RANGE="lo,hi" (debugging aid, tools/rr_find.py): only the shard's
    // samples [lo, hi) — the work counter starts at lo and the frame ends at hi
    uint64_t range_lo = 0;  // samples [range_lo, total_samples) are rendered
    if (const char* sr = debug_knob("BDPT_SAMPLE_RANGE")) {
        unsigned long long lo = 0, hi = 0;
        if (std::sscanf(sr, "%llu,%llu", &lo, &hi) == 2 && lo <= hi) {
            fr.total_samples = std::min<uint64_t>(fr.total_samples, hi);
            c->work_init = std::min<unsigned long long>(lo, fr.total_samples);
            range_lo = c->work_init;
            HIP_TRY(hipMemcpyAsync(c->work, &c->work_init, sizeof(unsigned long long), hipMemcpyHostToDevice, st));
        }
    }
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kCounterWords, st));
    if ((p->flags & BDPT_FLAG_COUNT) && fr.nrows > 0) {  // queries per local row (bdpt_get_row_costs)
        if (c->row_cost_cap < fr.nrows) {
            HIP_TRY(hipStreamSynchronize(st));
            if (c->row_cost) HIP_TRY(hipFree(c->row_cost));
            c->row_cost = nullptr;
            c->row_cost_cap = 0;
            HIP_TRY(hipMalloc(&c->row_cost, sizeof(unsigned long long) * fr.nrows));
            c->row_cost_cap = fr.nrows;
        }
        HIP_TRY(hipMemsetAsync(c->row_cost, 0, sizeof(unsigned long long) * fr.nrows, st));
        fr.row_cost = c->row_cost;
        c->row_cost_n = fr.nrows;
    }
    HIP_TRY(hipMemsetAsync(c->capped, 0, sizeof(uint32_t), st));
    HIP_TRY(hipMemsetAsync(c->diag, 0, sizeof(unsigned long long) * dev::kDiagWords, st));
    HIP_TRY(hipMemsetAsync(c->diag + dev::kDiagStart, 0xff, sizeof(unsigned long long), st));
    fr.diag = c->diag;
    HIP_TRY(hipEventRecord(c->ev0, st));
    int64_t launches = 0;
    if (fr.total_samples > 0) {
        if (rr) {  // never more resident blocks than the slots allocated
            // scenes with a dielectric can trap a subpath in a chain of delta bounces: the
            // build that runs a lone chain inline (bdpt_kernels_rrc.hip); BDPT_RR_CHAIN=0/1 forces
            const char* ce = std::getenv("BDPT_RR_CHAIN");
            const bool chain = ce ? *ce == '1' : c->has_glass;
            auto launch_rr = chain ? launch_frame_rrc : launch_frame_rr;
            auto launch_chain_k = chain ? launch_chain_rrc : launch_chain_rr;
            const int grid = std::min(c->grid, c->cus * (chain ? frame_kernel_blocks_per_cu_rrc : frame_kernel_blocks_per_cu_rr)(
                                                           4 * static_cast<size_t>(c->sc.lds_words)));
            const int park_depth = park_depth_setting();
            const bool park = park_depth > 0 && !(p->flags & BDPT_FLAG_COUNT);
            if (park) {
                const size_t words = static_cast<size_t>(c->nslots) * (kParkSlotWords + 1) + 1;
                if (!c->park) HIP_TRY(hipMalloc(&c->park, words * sizeof(uint32_t)));
                HIP_TRY(hipMemsetAsync(c->park, 0, words * sizeof(uint32_t), st));
                fr.park = c->park;
                fr.park_depth = park_depth;
                fr.park_flags = dev::kParkOn;
            }
            HIP_TRY(launch_rr(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, grid, st, c->dparams));
            const int rounds = park ? park_rounds_setting() : 0;
            uint32_t* const list = c->park + static_cast<size_t>(c->nslots) * kParkSlotWords;
            for (int k = 0; k < rounds; k++) {
                HIP_TRY(launch_chain_k(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, kChainGrid, st,
                                       c->dparams));
                HIP_TRY(hipMemsetAsync(list, 0, sizeof(uint32_t), st));  // the resume launch parks anew
                dev::DevFrame fres = fr;
                fres.park_flags = dev::kParkResume | (k + 1 < rounds ? dev::kParkOn : 0u);
                HIP_TRY(launch_rr(sc, fres, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, grid, st, c->dparams));
            }
            launches += 2 * rounds;
            c->last_kernel = chain ? "bdpt_frame_kernel_rrc" : "bdpt_frame_kernel_rr";
        } else if (p->rr_depth > kLazyRrDepth) {  // never more resident blocks than the slots allocated
            const int grid = std::min(c->grid, c->cus * frame_kernel_blocks_per_cu_deep(
                                                           4 * static_cast<size_t>(c->sc.lds_words)));
            HIP_TRY(launch_frame_deep(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, grid, st,
                                      c->dparams));
            c->last_kernel = "bdpt_frame_kernel_deep";
        } else if (hbm) {
            HIP_TRY(launch_frame_hbm(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, c->grid, st,
                                     c->dparams));
            c->last_kernel = "bdpt_frame_kernel_hbm";
        } else if (use_split_build(p->rr_depth)) {  // never more resident blocks than the slots allocated
            const int grid = std::min(c->grid, c->cus * frame_kernel_blocks_per_cu_split(
                                                           4 * static_cast<size_t>(c->sc.lds_words)));
            HIP_TRY(launch_frame_split(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, grid, st,
                                       c->dparams));
            c->last_kernel = "bdpt_frame_kernel_split";
        } else {
            HIP_TRY(launch_frame(sc, fr, fb, c->lv, c->gstack, c->nslots, c->work, c->counters, c->grid, st,
                                 c->dparams));
            c->last_kernel = "bdpt_frame_kernel";
        }
        launches += 1;
    }
    HIP_TRY(hipEventRecord(c->ev1, st));
    if ((rc = end_use(c, st))) return rc;
    c->pending_timing = true;
    c->diag_pending = true;
    c->stats = bdpt_stats{};
    c->stats.samples = static_cast<int64_t>(fr.total_samples - range_lo);
    c->stats.launches = launches;
    return BDPT_OK;
}

static int ensure_tmp_fb(bdpt_ctx* c, size_t floats);

// PathTracerIntegrator (path.h) on the same substrate: pt_kernels.hip.
constexpr int kPtMaxLevels = 512;  // recursion levels per lane under Russian roulette (P(> 512) ~ 0.95^507)

// The path / direct frame kernels read the BSDF records from the LDS table only.
static int pt_frame_tables(const bdpt_ctx* c) {
    if (c->sc.lds_bsdf_off == dev::kNoLds)
        return fail(BDPT_ERR_UNSUPPORTED, "the path / direct frame renders need the BSDF records in the LDS table "
                                          "(too many materials; bdpt_render and the single-sample calls take them)");
    return BDPT_OK;
}

static int ensure_pt(bdpt_ctx* c, int levels) {
    if (!c->pt_dparams) {
        HIP_TRY(hipMalloc(&c->pt_dparams, pt_params_bytes()));
        // Up to 4 resident 256-lane blocks per CU (4 waves/SIMD at 128 VGPRs;
        // measured 70 -> 119 Msamples/s from 2), within the BDPT grid (the
        // traversal-stack overflow buffer is sized for that many slots).
        // BDPT_PT_BLOCKS overrides the cap (experiments). Level stacks: 512 x 80 B
        // per slot, ~10.7 GB at 256 CUs x 1024 slots under Russian roulette.
        const char* cap_env = std::getenv("BDPT_PT_BLOCKS");
        const int cap = cap_env ? std::max(1, std::atoi(cap_env)) : 4;
        c->pt_grid = std::min(c->grid, c->cus * std::min(cap, pt_blocks_per_cu(4 * static_cast<size_t>(c->sc.lds_words))));
        c->pt_nslots = static_cast<uint32_t>(c->pt_grid) * 256u;
        HIP_TRY(hipMalloc(&c->pt_ring, sizeof(uint32_t) * 624 * static_cast<size_t>(c->pt_nslots)));
    }
    const size_t need = static_cast<size_t>(levels) * 5 * c->pt_nslots;
    if (need > c->pt_levels_f4) {
        if (c->pt_levels) HIP_TRY(hipFree(c->pt_levels));
        c->pt_levels = nullptr;
        HIP_TRY(hipMalloc(&c->pt_levels, need * sizeof(float4)));
        c->pt_levels_f4 = need;
    }
    return BDPT_OK;
}

// The path tracer's and direct integrator's scene: its queries start inside the
// scene box or at the camera, as the BDPT frame's do, so the same per-render
// choice of interior-box test applies (node_slack_needed).
#ifndef BDPT_PT_SLACK_FREE
#define BDPT_PT_SLACK_FREE 1  // 0: the path tracer keeps the slack test everywhere (A/B only)
#endif
static dev::DevScene pt_scene(const bdpt_ctx* c, const bdpt_frame_params* p) {
    dev::DevScene sc = c->sc;
    const float* eye[1] = {p->camera.eye};
    sc.node_slack = BDPT_PT_SLACK_FREE ? node_slack_needed(c, eye, 1) : 1u;
    return sc;
}

int bdpt_render_path(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_path_params* path, float* fb,
                     void* hip_stream) {
    if (!c || !fb || !path) return fail(BDPT_ERR_INVALID, "null argument");
    if (!p) return fail(BDPT_ERR_INVALID, "null params");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return fail(BDPT_ERR_INVALID, "width/height/spp must be > 0");
    if (static_cast<int64_t>(p->width) * p->height >= (1ll << 31))
        return fail(BDPT_ERR_INVALID, "image too large (W*H must fit int32, as in the reference)");
    if (p->row_stride < 1 || p->row_offset < 0) return fail(BDPT_ERR_INVALID, "bad row shard");
    if (path->emitter_samples < 0 || path->bsdf_samples < 0) return fail(BDPT_ERR_INVALID, "negative sample counts");
    // the recursion depth the settings allow: maxDepth levels, or Russian roulette
    const bool rr = path->is_explicit && path->max_depth == -1;
    const int levels = rr ? kPtMaxLevels : std::max(path->max_depth, 0) + 2;
    if (levels > kPtMaxLevels) return fail(BDPT_ERR_UNSUPPORTED, "maxDepth > 510 is not supported");
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = pt_frame_tables(c)) || (rc = ensure_pt(c, levels))) return rc;
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    const dev::DevFrame fr = make_frame(p);
    int32_t settings[8] = {path->is_explicit ? 1 : 0, path->max_depth, path->rr_depth, 0, path->emitter_samples,
                           path->bsdf_samples, levels, 0};
    std::memcpy(&settings[3], &path->rr_prob, 4);
    if ((rc = begin_use(c, st))) return rc;
    HIP_TRY(hipMemsetAsync(c->work, 0, sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kCounterWords, st));
    HIP_TRY(hipEventRecord(c->ev0, st));
    if (fr.total_samples > 0)
        HIP_TRY(launch_pt(pt_scene(c, p), fr, settings, fb, c->pt_levels, c->pt_ring, c->gstack, c->pt_nslots, c->work,
                          c->counters, c->pt_grid, st, c->pt_dparams));
    HIP_TRY(hipEventRecord(c->ev1, st));
    if ((rc = end_use(c, st))) return rc;
    c->pending_timing = true;
    c->diag_pending = false;
    c->stats = bdpt_stats{};
    c->stats.samples = static_cast<int64_t>(fr.total_samples);
    c->stats.launches = fr.total_samples > 0 ? 1 : 0;
    return BDPT_OK;
}

int bdpt_render_path_host(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_path_params* path, float* fb_host) {
    if (!c || !fb_host || !p) return fail(BDPT_ERR_INVALID, "null argument");
    if (p->width <= 0 || p->height <= 0) return fail(BDPT_ERR_INVALID, "width/height must be > 0");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = static_cast<size_t>(p->width) * p->height * 3;
    int rc;
    if ((rc = ensure_tmp_fb(c, n))) return rc;
    HIP_TRY(hipMemcpyAsync(c->tmp_fb, fb_host, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if ((rc = bdpt_render_path(c, p, path, c->tmp_fb, c->stream))) return rc;
    HIP_TRY(hipMemcpyAsync(fb_host, c->tmp_fb, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    bdpt_stats st;
    if ((rc = bdpt_get_stats(c, &st))) return rc;
    if (st.counters[1] != 0)
        return fail(BDPT_ERR_UNSUPPORTED, std::to_string(st.counters[1]) + " samples outgrew the path tracer's level stack");
    return BDPT_OK;
}

// DirectIntegrator (direct.h) on the path tracer's kernel: one level, no recursion.
int bdpt_render_direct(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_direct_params* d, float* fb,
                       void* hip_stream) {
    if (!c || !fb || !d) return fail(BDPT_ERR_INVALID, "null argument");
    if (!p) return fail(BDPT_ERR_INVALID, "null params");
    if (p->width <= 0 || p->height <= 0 || p->spp <= 0) return fail(BDPT_ERR_INVALID, "width/height/spp must be > 0");
    if (static_cast<int64_t>(p->width) * p->height >= (1ll << 31))
        return fail(BDPT_ERR_INVALID, "image too large (W*H must fit int32, as in the reference)");
    if (p->row_stride < 1 || p->row_offset < 0) return fail(BDPT_ERR_INVALID, "bad row shard");
    if (d->sampling_strategy < BDPT_DIRECT_AREA || d->sampling_strategy > BDPT_DIRECT_MIS)
        return fail(BDPT_ERR_INVALID, "Error: wrong strategy");  // direct.h:460
    if (d->emitter_samples < 0 || d->bsdf_samples < 0) return fail(BDPT_ERR_INVALID, "negative sample counts");
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = pt_frame_tables(c)) || (rc = ensure_pt(c, 1))) return rc;
    hipStream_t st = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->stream;
    const dev::DevFrame fr = make_frame(p);
    const int32_t settings[8] = {1, -1, 0, 0, d->emitter_samples, d->bsdf_samples, 1, d->sampling_strategy};
    if ((rc = begin_use(c, st))) return rc;
    HIP_TRY(hipMemsetAsync(c->work, 0, sizeof(unsigned long long), st));
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kCounterWords, st));
    HIP_TRY(hipEventRecord(c->ev0, st));
    if (fr.total_samples > 0)
        HIP_TRY(launch_pt(pt_scene(c, p), fr, settings, fb, c->pt_levels, c->pt_ring, c->gstack, c->pt_nslots, c->work,
                          c->counters, c->pt_grid, st, c->pt_dparams));
    HIP_TRY(hipEventRecord(c->ev1, st));
    if ((rc = end_use(c, st))) return rc;
    c->pending_timing = true;
    c->diag_pending = false;
    c->stats = bdpt_stats{};
    c->stats.samples = static_cast<int64_t>(fr.total_samples);
    c->stats.launches = fr.total_samples > 0 ? 1 : 0;
    return BDPT_OK;
}

int bdpt_render_direct_host(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_direct_params* d, float* fb_host) {
    if (!c || !fb_host || !p) return fail(BDPT_ERR_INVALID, "null argument");
    if (p->width <= 0 || p->height <= 0) return fail(BDPT_ERR_INVALID, "width/height must be > 0");
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = static_cast<size_t>(p->width) * p->height * 3;
    int rc;
    if ((rc = ensure_tmp_fb(c, n))) return rc;
    HIP_TRY(hipMemcpyAsync(c->tmp_fb, fb_host, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if ((rc = bdpt_render_direct(c, p, d, c->tmp_fb, c->stream))) return rc;
    HIP_TRY(hipMemcpyAsync(fb_host, c->tmp_fb, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

static int ensure_sample_buffers(bdpt_ctx* c, int32_t splat_cap) {
    if (!c->mt_state) HIP_TRY(hipMalloc(&c->mt_state, sizeof(uint32_t) * BDPT_MT19937_WORDS));
    if (splat_cap > c->splat_cap) {
        if (c->splat_list) HIP_TRY(hipFree(c->splat_list));
        c->splat_list = nullptr;
        HIP_TRY(hipMalloc(&c->splat_list, sizeof(float) * 4 * (static_cast<size_t>(splat_cap) + 1)));
        c->splat_cap = splat_cap;
    }
    return BDPT_OK;
}

static int check_mt_state(const uint32_t* state) {
    if (!state) return fail(BDPT_ERR_INVALID, "null sampler state");
    if (state[BDPT_MT19937_WORDS - 1] > 624u) return fail(BDPT_ERR_INVALID, "sampler state position _M_p > 624");
    return BDPT_OK;
}

// One PathTracerIntegrator / DirectIntegrator::render(ray, sampler) call with the
// caller's std::mt19937 state (settings: the launch_pt block; levels: level-stack
// depth it needs).
static int render_pt_sample(bdpt_ctx* c, const bdpt_frame_params* p, const int32_t settings[8], int levels,
                            const float ray[8], uint32_t* state, float Li[3], uint32_t* taken = nullptr) {
    if (!c || !p || !ray || !Li) return fail(BDPT_ERR_INVALID, "null argument");
    int rc;
    if ((rc = check_mt_state(state))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    if ((rc = ensure_pt(c, levels))) return rc;
    if ((rc = ensure_sample_buffers(c, 1))) return rc;
    if ((rc = begin_use(c, c->stream))) return rc;
    const dev::DevFrame fr = make_frame(p);
    const dev::Ray r{dev::f3{ray[0], ray[1], ray[2]}, dev::f3{ray[3], ray[4], ray[5]}, ray[6], ray[7]};
    dev::DevScene sc = c->sc;
    sc.mt_ring = c->mt_state;  // the sample kernel's generator state (mt_state_u32)
    HIP_TRY(hipMemcpyAsync(c->mt_state, state, sizeof(uint32_t) * BDPT_MT19937_WORDS, hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * kCounterWords, c->stream));
    HIP_TRY(launch_pt_sample(sc, fr, settings, c->pt_levels, c->pt_ring, c->gstack, r, c->sample_out, c->counters,
                             c->stream, c->pt_dparams));
    float out[4];
    unsigned long long ctr[2];
    HIP_TRY(hipMemcpyAsync(out, c->sample_out, sizeof(out), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(ctr, c->counters, sizeof(ctr), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(state, c->mt_state, sizeof(uint32_t) * BDPT_MT19937_WORDS, hipMemcpyDeviceToHost,
                           c->stream));
    if ((rc = end_use(c, c->stream))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (ctr[1] != 0) return fail(BDPT_ERR_UNSUPPORTED, "the sample outgrew the path tracer's level stack");
    Li[0] = out[0], Li[1] = out[1], Li[2] = out[2];
    if (taken) std::memcpy(taken, &out[3], 4);
    return BDPT_OK;
}

static int path_sample_settings(const bdpt_path_params* path, int32_t settings[8], int& levels) {
    if (!path) return fail(BDPT_ERR_INVALID, "null argument");
    if (path->emitter_samples < 0 || path->bsdf_samples < 0) return fail(BDPT_ERR_INVALID, "negative sample counts");
    const bool rr = path->is_explicit && path->max_depth == -1;
    levels = rr ? kPtMaxLevels : std::max(path->max_depth, 0) + 2;
    if (levels > kPtMaxLevels) return fail(BDPT_ERR_UNSUPPORTED, "maxDepth > 510 is not supported");
    const int32_t s[8] = {path->is_explicit ? 1 : 0, path->max_depth, path->rr_depth, 0, path->emitter_samples,
                          path->bsdf_samples, levels, 0};
    std::memcpy(settings, s, sizeof(s));
    std::memcpy(&settings[3], &path->rr_prob, 4);
    return BDPT_OK;
}

static int direct_sample_settings(const bdpt_direct_params* d, int32_t settings[8]) {
    if (!d) return fail(BDPT_ERR_INVALID, "null argument");
    if (d->sampling_strategy < BDPT_DIRECT_AREA || d->sampling_strategy > BDPT_DIRECT_MIS)
        return fail(BDPT_ERR_INVALID, "Error: wrong strategy");  // direct.h:460
    if (d->emitter_samples < 0 || d->bsdf_samples < 0) return fail(BDPT_ERR_INVALID, "negative sample counts");
    const int32_t s[8] = {1, -1, 0, 0, d->emitter_samples, d->bsdf_samples, 1, d->sampling_strategy};
    std::memcpy(settings, s, sizeof(s));
    return BDPT_OK;
}

int bdpt_render_path_sample_mt(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_path_params* path,
                               const float ray[8], uint32_t state[BDPT_MT19937_WORDS], float Li[3]) {
    int32_t settings[8];
    int levels = 0, rc;
    if ((rc = path_sample_settings(path, settings, levels))) return rc;
    return render_pt_sample(c, p, settings, levels, ray, state, Li);
}

int bdpt_render_direct_sample_mt(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_direct_params* d,
                                 const float ray[8], uint32_t state[BDPT_MT19937_WORDS], float Li[3]) {
    int32_t settings[8];
    int rc;
    if ((rc = direct_sample_settings(d, settings))) return rc;
    return render_pt_sample(c, p, settings, 1, ray, state, Li);
}

// (seed, draws) sampler: std::mt19937(seed) advanced by *draws outputs.
static int pt_sample_seeded(bdpt_ctx* c, const bdpt_frame_params* p, const int32_t settings[8], int levels,
                            const float ray[8], uint32_t seed, int32_t* draws, float Li[3]) {
    if (!draws) return fail(BDPT_ERR_INVALID, "null argument");
    if (*draws < 0) return fail(BDPT_ERR_INVALID, "negative draw count");
    uint32_t st[BDPT_MT19937_WORDS], used = 0;
    mt19937_state(seed, *draws, st);
    int rc;
    if ((rc = render_pt_sample(c, p, settings, levels, ray, st, Li, &used))) return rc;
    *draws += static_cast<int32_t>(used);
    return BDPT_OK;
}

int bdpt_render_path_sample(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_path_params* path,
                            const float ray[8], uint32_t seed, int32_t* draws, float Li[3]) {
    int32_t settings[8];
    int levels = 0, rc;
    if ((rc = path_sample_settings(path, settings, levels))) return rc;
    return pt_sample_seeded(c, p, settings, levels, ray, seed, draws, Li);
}

int bdpt_render_direct_sample(bdpt_ctx* c, const bdpt_frame_params* p, const bdpt_direct_params* d,
                              const float ray[8], uint32_t seed, int32_t* draws, float Li[3]) {
    int32_t settings[8];
    int rc;
    if ((rc = direct_sample_settings(d, settings))) return rc;
    return pt_sample_seeded(c, p, settings, 1, ray, seed, draws, Li);
}

int bdpt_debug_math(int32_t device, int32_t fn, const float* x, const float* y, float* out, int64_t n) {
    if (!x || !out || n < 0 || (fn == 2 && !y) || fn < 0 || fn > 4) return fail(BDPT_ERR_INVALID, "bad argument");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(BDPT_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(BDPT_ERR_INVALID, "bad device");
    HIP_TRY(hipSetDevice(device));
    if (n == 0) return BDPT_OK;
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    const size_t bytes = sizeof(float) * static_cast<size_t>(n);
    hipError_t e = hipMalloc(&dx, bytes);
    if (e == hipSuccess) e = hipMalloc(&dy, bytes);
    if (e == hipSuccess) e = hipMalloc(&dout, bytes);
    if (e == hipSuccess) e = hipMemcpy(dx, x, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(dy, y ? y : x, bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch_math_check(fn, dx, dy, dout, n, nullptr);
    if (e == hipSuccess) e = hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost);
    for (float* p : {dx, dy, dout})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return fail(BDPT_ERR_HIP, std::string("bdpt_debug_math: ") + hipGetErrorString(e));
    return BDPT_OK;
}

const char* bdpt_last_kernel(const bdpt_ctx* c) { return c ? c->last_kernel : ""; }

int bdpt_set_row_order(bdpt_ctx* c, const int32_t* order, int32_t n) {
    if (!c || n < 0 || (n > 0 && !order)) return fail(BDPT_ERR_INVALID, "bdpt_set_row_order: bad argument");
    std::vector<char> seen(static_cast<size_t>(n), 0);
    for (int32_t i = 0; i < n; i++) {
        if (order[i] < 0 || order[i] >= n || seen[static_cast<size_t>(order[i])])
            return fail(BDPT_ERR_INVALID, "bdpt_set_row_order: not a permutation of 0..n-1");
        seen[static_cast<size_t>(order[i])] = 1;
    }
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());  // a render in flight may read the previous order
    if (c->row_order) HIP_TRY(hipFree(c->row_order));
    c->row_order = nullptr;
    c->row_order_n = 0;
    if (n == 0) return BDPT_OK;
    HIP_TRY(hipMalloc(&c->row_order, sizeof(int32_t) * static_cast<size_t>(n)));
    HIP_TRY(hipMemcpy(c->row_order, order, sizeof(int32_t) * static_cast<size_t>(n), hipMemcpyHostToDevice));
    c->row_order_n = n;
    return BDPT_OK;
}

int bdpt_get_row_costs(bdpt_ctx* c, int64_t* costs, int32_t n) {
    if (!c || !costs) return fail(BDPT_ERR_INVALID, "null argument");
    if (!c->row_cost || n != c->row_cost_n)
        return fail(BDPT_ERR_INVALID, "bdpt_get_row_costs: no counting render of a " + std::to_string(n) + "-row shard");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    std::vector<unsigned long long> h(static_cast<size_t>(n));
    HIP_TRY(hipMemcpy(h.data(), c->row_cost, sizeof(unsigned long long) * static_cast<size_t>(n), hipMemcpyDeviceToHost));
    for (int32_t i = 0; i < n; i++) costs[i] = static_cast<int64_t>(h[static_cast<size_t>(i)]);
    return BDPT_OK;
}

int bdpt_get_stats(bdpt_ctx* c, bdpt_stats* out) {
    if (!c || !out) return fail(BDPT_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    if (c->pending_timing) {
        HIP_TRY(hipEventSynchronize(c->ev1));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        c->stats.kernel_ms = ms;
        unsigned long long host[BDPT_NUM_COUNTERS];
        HIP_TRY(hipMemcpy(host, c->counters, sizeof(host), hipMemcpyDeviceToHost));
        for (int i = 0; i < BDPT_NUM_COUNTERS; i++) c->stats.counters[i] = static_cast<int64_t>(host[i]);
        uint32_t capped = 0;
        HIP_TRY(hipMemcpy(&capped, c->capped, sizeof(capped), hipMemcpyDeviceToHost));
        c->stats.capped_samples = capped;
        unsigned long long mx[3];
        HIP_TRY(hipMemcpy(mx, c->counters + BDPT_NUM_COUNTERS, sizeof(mx), hipMemcpyDeviceToHost));
        c->stats.max_light_depth = static_cast<int64_t>(mx[0]);
        c->stats.max_eye_depth = static_cast<int64_t>(mx[1]);
        c->stats.max_queries = static_cast<int64_t>(mx[2]);
        unsigned long long sq[4];
        HIP_TRY(hipMemcpy(sq, c->counters + BDPT_NUM_COUNTERS + 3, sizeof(sq), hipMemcpyDeviceToHost));
        for (int i = 0; i < 4; i++) c->stats.sched[i] = static_cast<int64_t>(sq[i]);
        if (c->diag_pending) {
            unsigned long long d[dev::kDiagWords];
            HIP_TRY(hipMemcpy(d, c->diag, sizeof(d), hipMemcpyDeviceToHost));
            const double tick_ms = 1.0 / c->wall_khz;
            if (d[dev::kDiagStart] != ~0ull && d[dev::kDiagEnd] >= d[dev::kDiagStart])
                c->stats.span_ms = static_cast<double>(d[dev::kDiagEnd] - d[dev::kDiagStart]) * tick_ms;
            if (d[dev::kDiagLastClaim] && d[dev::kDiagEnd] >= d[dev::kDiagLastClaim])
                c->stats.tail_ms = static_cast<double>(d[dev::kDiagEnd] - d[dev::kDiagLastClaim]) * tick_ms;
            c->stats.schedule_errors = static_cast<int64_t>(d[dev::kDiagErrors]);
            c->stats.parked_samples = static_cast<int64_t>(d[dev::kDiagParked]);
            c->stats.rr_long_walks_max = static_cast<int64_t>(d[dev::kDiagLongMax]);
            for (int k = 0; k < 3; k++) c->stats.rr_express_iters[k] = static_cast<int64_t>(d[dev::kDiagExpress1 + k]);
        }
        c->pending_timing = false;
    }
    *out = c->stats;
    return BDPT_OK;
}

int bdpt_synchronize(bdpt_ctx* c) {
    if (!c) return fail(BDPT_ERR_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    return BDPT_OK;
}

static int ensure_tmp_fb(bdpt_ctx* c, size_t floats) {
    if (floats > c->tmp_fb_floats) {
        if (c->tmp_fb) HIP_TRY(hipFree(c->tmp_fb));
        c->tmp_fb = nullptr;
        HIP_TRY(hipMalloc(&c->tmp_fb, floats * sizeof(float)));
        c->tmp_fb_floats = floats;
    }
    return BDPT_OK;
}

int bdpt_render_host(bdpt_ctx* c, const bdpt_frame_params* p, float* fb_host) {
    if (!c || !fb_host) return fail(BDPT_ERR_INVALID, "null argument");
    int rc = check_params(p);
    if (rc) return rc;
    HIP_TRY(hipSetDevice(c->device));
    const size_t n = static_cast<size_t>(p->width) * p->height * 3;
    if ((rc = ensure_tmp_fb(c, n))) return rc;
    HIP_TRY(hipMemcpyAsync(c->tmp_fb, fb_host, n * sizeof(float), hipMemcpyHostToDevice, c->stream));
    if ((rc = bdpt_render(c, p, c->tmp_fb, c->stream))) return rc;
    HIP_TRY(hipMemcpyAsync(fb_host, c->tmp_fb, n * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    {
        bdpt_stats st;
        if ((rc = bdpt_get_stats(c, &st))) return rc;
        if (st.schedule_errors)
            return fail(BDPT_ERR_HIP, std::to_string(st.schedule_errors) +
                                          " schedule errors (MT19937 draws past the generated ring, or a continuation walk "
                                          "out of stack)");
        if (p->russian_roulette && st.capped_samples)
            return fail(BDPT_ERR_UNSUPPORTED, std::to_string(st.capped_samples) +
                                                  " samples met the Russian-roulette bounds (light-vertex store / "
                                                  "bounce guard); the image is not the reference's");
    }
    return BDPT_OK;
}

static int render_bdpt_sample(bdpt_ctx* c, const bdpt_frame_params* p, const float ray[8], uint32_t* state,
                              float Li[3], bdpt_splat* splats, int32_t capacity, int32_t* nsplats, uint32_t* taken) {
    if (!c || !ray || !Li || !nsplats || (capacity > 0 && !splats) || capacity < 0)
        return fail(BDPT_ERR_INVALID, "null argument");
    int rc = check_params(p);
    if (rc) return rc;
    if ((rc = check_mt_state(state))) return rc;
    HIP_TRY(hipSetDevice(c->device));
    // the sample kernel's one lane uses lane slot 0 of the light-vertex store
    if ((rc = ensure_lv(c, make_frame(p).lv_max, 1))) return rc;
    // a sample splats at most once per light vertex: rr_depth bounds the list
    // without Russian roulette; with it the list grows on demand (below)
    if ((rc = ensure_sample_buffers(c, std::max(p->rr_depth, 1)))) return rc;
    dev::DevFrame fr = make_frame(p);
    fr.capped = c->capped;
    dev::DevScene sc = c->sc;
    sc.mt_ring = c->mt_state;  // the sample kernel's generator state (mt_state_u32)
    const float* origins[2] = {p->camera.eye, ray};  // camera connections start at the eye, the walk at ray.o
    sc.node_slack = node_slack_needed(c, origins, 2);
    const dev::Ray r{dev::f3{ray[0], ray[1], ray[2]}, dev::f3{ray[3], ray[4], ray[5]}, ray[6], ray[7]};
    uint32_t st_out[BDPT_MT19937_WORDS];
    std::vector<float> list;
    float out[4];
    uint32_t n = 0;
    for (int attempt = 0;; attempt++) {
        if ((rc = begin_use(c, c->stream))) return rc;
        const uint32_t hdr[4] = {0u, static_cast<uint32_t>(c->splat_cap), 0u, 0u};
        HIP_TRY(hipMemcpyAsync(c->mt_state, state, sizeof(uint32_t) * BDPT_MT19937_WORDS, hipMemcpyHostToDevice,
                               c->stream));
        HIP_TRY(hipMemcpyAsync(c->splat_list, hdr, sizeof(hdr), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemsetAsync(c->capped, 0, sizeof(uint32_t), c->stream));
        HIP_TRY(launch_sample(sc, fr, c->splat_list, c->lv, c->gstack, r, c->sample_out, c->stream));
        list.assign(4 * (static_cast<size_t>(c->splat_cap) + 1), 0.f);
        HIP_TRY(hipMemcpyAsync(out, c->sample_out, sizeof(out), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipMemcpyAsync(list.data(), c->splat_list, list.size() * sizeof(float), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipMemcpyAsync(st_out, c->mt_state, sizeof(st_out), hipMemcpyDeviceToHost, c->stream));
        uint32_t capped = 0;
        HIP_TRY(hipMemcpyAsync(&capped, c->capped, sizeof(capped), hipMemcpyDeviceToHost, c->stream));
        if ((rc = end_use(c, c->stream))) return rc;
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (capped)
            return fail(BDPT_ERR_UNSUPPORTED, "the sample met the Russian-roulette bounds (light-vertex store / "
                                              "bounce guard)");
        std::memcpy(&n, &list[0], 4);
        if (n <= static_cast<uint32_t>(c->splat_cap)) break;
        // more splats than the device list holds (the kernel counts them all):
        // grow it and run the sample again from the caller's unchanged state
        if (attempt > 0) return fail(BDPT_ERR_HIP, "splat list overflow");
        if ((rc = ensure_sample_buffers(c, static_cast<int32_t>(n)))) return rc;
    }
    *nsplats = static_cast<int32_t>(n);
    if (static_cast<int32_t>(n) > capacity)  // the caller's state is left as it was
        return fail(BDPT_ERR_INVALID, "splat capacity too small (" + std::to_string(n) + " splats)");
    for (uint32_t k = 0; k < n; k++) {
        const float* e = &list[4 + 4 * static_cast<size_t>(k)];
        std::memcpy(&splats[k].pixel, &e[0], 4);
        splats[k].rgb[0] = e[1], splats[k].rgb[1] = e[2], splats[k].rgb[2] = e[3];
    }
    std::memcpy(state, st_out, sizeof(st_out));
    Li[0] = out[0], Li[1] = out[1], Li[2] = out[2];
    if (taken) std::memcpy(taken, &out[3], 4);
    return BDPT_OK;
}

int bdpt_sampler_state(uint32_t seed, int64_t draws, uint32_t state[BDPT_MT19937_WORDS]) {
    if (!state || draws < 0) return fail(BDPT_ERR_INVALID, "bad argument");
    mt19937_state(seed, draws, state);
    return BDPT_OK;
}

int bdpt_render_sample_mt(bdpt_ctx* c, const bdpt_frame_params* p, const float ray[8],
                          uint32_t state[BDPT_MT19937_WORDS], float Li[3], bdpt_splat* splats, int32_t capacity,
                          int32_t* nsplats) {
    return render_bdpt_sample(c, p, ray, state, Li, splats, capacity, nsplats, nullptr);
}

int bdpt_render_sample(bdpt_ctx* c, const bdpt_frame_params* p, const float ray[8], uint32_t seed,
                       int32_t* draws, float Li[3], float* fb_host) {
    if (!c || !p || !draws || !fb_host) return fail(BDPT_ERR_INVALID, "null argument");
    if (*draws < 0) return fail(BDPT_ERR_INVALID, "negative draw count");
    uint32_t st[BDPT_MT19937_WORDS], used = 0;
    mt19937_state(seed, *draws, st);
    std::vector<bdpt_splat> sp(static_cast<size_t>(std::max(p->rr_depth, 1)));
    int32_t n = 0;
    int rc = render_bdpt_sample(c, p, ray, st, Li, sp.data(), static_cast<int32_t>(sp.size()), &n, &used);
    if (rc == BDPT_ERR_INVALID && n > static_cast<int32_t>(sp.size())) {  // Russian roulette: a longer list
        sp.resize(static_cast<size_t>(n));
        rc = render_bdpt_sample(c, p, ray, st, Li, sp.data(), n, &n, &used);
    }
    if (rc) return rc;
    for (int32_t k = 0; k < n; k++) {  // rgb[pixel] += radiance * misWeight, in the sample's order
        float* px = fb_host + 3 * static_cast<size_t>(sp[k].pixel);
        px[0] += sp[k].rgb[0], px[1] += sp[k].rgb[1], px[2] += sp[k].rgb[2];
    }
    *draws += static_cast<int32_t>(used);
    return BDPT_OK;
}

static int ensure_kat(bdpt_ctx* c, size_t bytes, void** buf) {
    HIP_TRY(hipMalloc(buf, std::max<size_t>(bytes, 16)));
    return BDPT_OK;
}

// Host arrays in, device run, host arrays out (the per-function entry points).
struct KatBuffers {
    std::vector<void*> p;
    ~KatBuffers() {
        for (void* q : p) (void)hipFree(q);
    }
};

static int kat_in(bdpt_ctx* c, KatBuffers& kb, const void* src, size_t bytes, void** dst) {
    int rc;
    if ((rc = ensure_kat(c, bytes, dst))) return rc;
    kb.p.push_back(*dst);
    if (src && bytes) HIP_TRY(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, c->stream));
    return BDPT_OK;
}

static int bsdf_kat(bdpt_ctx* c, int mode, int64_t n, const int32_t* mat, const float* wo, const float* x,
                    float* out, int out_per) {
    if (!c || n < 0 || (n > 0 && (!mat || !wo || !x || !out))) return fail(BDPT_ERR_INVALID, "bad argument");
    for (int64_t i = 0; i < n; i++)
        if (mat[i] < 0 || mat[i] >= c->sc.nbsdf) return fail(BDPT_ERR_INVALID, "material index out of range");
    if (n == 0) return BDPT_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = begin_use(c, c->stream))) return rc;
    KatBuffers kb;
    void *dm, *dwo, *dx, *dout;
    const size_t N = static_cast<size_t>(n);
    if ((rc = kat_in(c, kb, mat, 4 * N, &dm)) || (rc = kat_in(c, kb, wo, 12 * N, &dwo)) ||
        (rc = kat_in(c, kb, x, (mode == 2 ? 8 : 12) * N, &dx)) || (rc = kat_in(c, kb, nullptr, 4 * out_per * N, &dout)))
        return rc;
    HIP_TRY(launch_bsdf_kat(c->sc, mode, n, static_cast<const int32_t*>(dm), static_cast<const float*>(dwo),
                            static_cast<const float*>(dx), static_cast<float*>(dout), c->stream));
    HIP_TRY(hipMemcpyAsync(out, dout, 4 * out_per * N, hipMemcpyDeviceToHost, c->stream));
    if ((rc = end_use(c, c->stream))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_bsdf_eval(bdpt_ctx* c, int64_t n, const int32_t* mat, const float* wo, const float* wi, float* f) {
    return bsdf_kat(c, 0, n, mat, wo, wi, f, 3);
}

int bdpt_bsdf_pdf(bdpt_ctx* c, int64_t n, const int32_t* mat, const float* wo, const float* wi, float* pdf) {
    return bsdf_kat(c, 1, n, mat, wo, wi, pdf, 1);
}

int bdpt_bsdf_sample(bdpt_ctx* c, int64_t n, const int32_t* mat, const float* wo, const float* u, float* f,
                     float* wi, float* pdf) {
    if (n > 0 && (!f || !wi || !pdf)) return fail(BDPT_ERR_INVALID, "null output");
    std::vector<float> o(7 * static_cast<size_t>(std::max<int64_t>(n, 0)));
    int rc = bsdf_kat(c, 2, n, mat, wo, u, o.data(), 7);
    if (rc) return rc;
    for (int64_t i = 0; i < n; i++) {
        const float* r = &o[7 * static_cast<size_t>(i)];
        f[3 * i] = r[0], f[3 * i + 1] = r[1], f[3 * i + 2] = r[2];
        wi[3 * i] = r[3], wi[3 * i + 1] = r[4], wi[3 * i + 2] = r[5];
        pdf[i] = r[6];
    }
    return BDPT_OK;
}

int bdpt_bsdf_type(const bdpt_scene* s, int32_t mat, uint32_t* type, int32_t* kind) {
    if (!s || !type || !kind) return fail(BDPT_ERR_INVALID, "null argument");
    if (mat < 0 || mat >= static_cast<int32_t>(s->layout.bsdfs.size()))
        return fail(BDPT_ERR_INVALID, "material index out of range");
    *type = s->layout.bsdfs[static_cast<size_t>(mat)].type;
    *kind = s->layout.bsdfs[static_cast<size_t>(mat)].kind;
    return BDPT_OK;
}

int bdpt_intersect(bdpt_ctx* c, int64_t n, const float* rays, int32_t occlusion, bdpt_hit* out) {
    return bdpt_intersect_from(c, n, rays, nullptr, nullptr, occlusion, out);
}

int bdpt_intersect_from(bdpt_ctx* c, int64_t n, const float* rays, const float* origin_normals,
                        const int32_t* origin_tris, int32_t occlusion, bdpt_hit* out) {
    static_assert(sizeof(bdpt_hit) == 20 * 4, "bdpt_hit is the kernel's 20-word record");
    if (!c || n < 0 || (n > 0 && (!rays || !out))) return fail(BDPT_ERR_INVALID, "bad argument");
    if (n == 0) return BDPT_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = begin_use(c, c->stream))) return rc;
    KatBuffers kb;
    void *dr, *dout, *dn = nullptr, *dt = nullptr;
    const size_t N = static_cast<size_t>(n);
    if (origin_tris)
        for (size_t i = 0; i < N; i++)
            if (origin_tris[i] < -1 || origin_tris[i] >= c->ntri) return fail(BDPT_ERR_INVALID, "origin_tris out of range");
    if ((rc = kat_in(c, kb, rays, 32 * N, &dr)) || (rc = kat_in(c, kb, nullptr, 80 * N, &dout))) return rc;
    if (origin_normals && (rc = kat_in(c, kb, origin_normals, 12 * N, &dn))) return rc;
    if (origin_normals && origin_tris && (rc = kat_in(c, kb, origin_tris, 4 * N, &dt))) return rc;
    // The interior-box test the frame kernels would use for these origins: without
    // the ambiguity slack when every origin lies within 100 scene diagonals (as
    // for a frame whose camera does, node_slack_needed), with it otherwise.
    std::vector<const float*> origins(N);
    for (size_t i = 0; i < N; i++) origins[i] = rays + 8 * i;
    dev::DevScene sc = c->sc;
    sc.node_slack = node_slack_needed(c, origins.data(), static_cast<int>(std::min<size_t>(N, 0x7fffffff)));
    // the traversal-stack overflow columns serve c->nslots rays at a time
    for (int64_t b = 0; b < n; b += c->nslots) {
        const int64_t m = std::min<int64_t>(c->nslots, n - b);
        HIP_TRY(launch_intersect_kat(sc, m, occlusion ? 1 : 0, static_cast<const float*>(dr) + 8 * b,
                                     dn ? static_cast<const float*>(dn) + 3 * b : nullptr,
                                     dt ? static_cast<const int32_t*>(dt) + b : nullptr, c->gstack, c->nslots,
                                     static_cast<float*>(dout) + 20 * b, c->stream));
    }
    HIP_TRY(hipMemcpyAsync(out, dout, 80 * N, hipMemcpyDeviceToHost, c->stream));
    if ((rc = end_use(c, c->stream))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

int bdpt_splat_to_image_plane(bdpt_ctx* c, const bdpt_frame_params* p, int64_t n, const float* pts, int32_t* xy) {
    if (!c || !p || n < 0 || (n > 0 && (!pts || !xy))) return fail(BDPT_ERR_INVALID, "bad argument");
    if (p->width <= 0 || p->height <= 0) return fail(BDPT_ERR_INVALID, "width/height must be > 0");
    if (n == 0) return BDPT_OK;
    HIP_TRY(hipSetDevice(c->device));
    int rc;
    if ((rc = begin_use(c, c->stream))) return rc;
    KatBuffers kb;
    void *dp, *dxy;
    const size_t N = static_cast<size_t>(n);
    if ((rc = kat_in(c, kb, pts, 12 * N, &dp)) || (rc = kat_in(c, kb, nullptr, 8 * N, &dxy))) return rc;
    HIP_TRY(launch_splat_kat(make_frame(p), n, static_cast<const float*>(dp), static_cast<int32_t*>(dxy), c->stream));
    HIP_TRY(hipMemcpyAsync(xy, dxy, 8 * N, hipMemcpyDeviceToHost, c->stream));
    if ((rc = end_use(c, c->stream))) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return BDPT_OK;
}

// Device-only diagnostics without a scene (synchronous, default stream).
static int device_kat(int32_t device, size_t in_bytes, const float* in, size_t in2_bytes, const float* in2,
                      size_t out_bytes, float* out,
                      hipError_t (*launch)(const float*, const float*, float*)) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return fail(BDPT_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= count) return fail(BDPT_ERR_INVALID, "bad device");
    HIP_TRY(hipSetDevice(device));
    float *a = nullptr, *b = nullptr, *o = nullptr;
    hipError_t e = hipMalloc(&a, std::max<size_t>(in_bytes, 16));
    if (e == hipSuccess) e = hipMalloc(&b, std::max<size_t>(in2_bytes, 16));
    if (e == hipSuccess) e = hipMalloc(&o, std::max<size_t>(out_bytes, 16));
    if (e == hipSuccess) e = hipMemcpy(a, in, in_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess && in2) e = hipMemcpy(b, in2, in2_bytes, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = launch(a, b, o);
    if (e == hipSuccess) e = hipMemcpy(out, o, out_bytes, hipMemcpyDeviceToHost);
    for (float* q : {a, b, o})
        if (q) (void)hipFree(q);
    if (e != hipSuccess) return fail(BDPT_ERR_HIP, std::string("device diagnostic: ") + hipGetErrorString(e));
    return BDPT_OK;
}

static thread_local int64_t g_kat_n = 0;

int bdpt_debug_fresnel(int32_t device, int64_t n, const float* in, float* out) {
    if (n < 0 || (n > 0 && (!in || !out))) return fail(BDPT_ERR_INVALID, "bad argument");
    if (n == 0) return BDPT_OK;
    g_kat_n = n;
    const size_t N = static_cast<size_t>(n);
    return device_kat(device, 16 * N, in, 0, nullptr, 4 * N, out, [](const float* a, const float*, float* o) {
        return launch_fresnel_kat(g_kat_n, a, o, nullptr);
    });
}

int bdpt_debug_triangle(int32_t device, int64_t n, const float* rays, const float* verts, float* out) {
    if (n < 0 || (n > 0 && (!rays || !verts || !out))) return fail(BDPT_ERR_INVALID, "bad argument");
    if (n == 0) return BDPT_OK;
    g_kat_n = n;
    const size_t N = static_cast<size_t>(n);
    return device_kat(device, 32 * N, rays, 36 * N, verts, 16 * N, out, [](const float* a, const float* b, float* o) {
        return launch_triangle_kat(g_kat_n, a, b, o, nullptr);
    });
}

}  // extern "C"
