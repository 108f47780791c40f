// Deterministic driver around the UNMODIFIED reference BDPT integrator.
//
// TEST INFRASTRUCTURE ONLY. This file is compiled together with the reference's
// own sources under /root/reference (see oracle/ref/Makefile); the resulting
// binary oracle/_ref/ref_bdpt is used to (a) generate the golden fixtures under
// tests/golden/ and (b) time the reference CPU path as bench.py's cpu_baseline.
// It is never linked into, or called by, the product library.
//
// What it restates: the offline branch of Renderer::render
// (reference src/core/renderer.cpp:130-214) with ONE change that the survey's
// parity convention requires: instead of one Sampler shared
// racily by all threads (renderer.cpp:155, :159), every (pixel p, sample k)
// gets its own Sampler((int)(260450963u + p*spp + k)). BDPTIntegrator::render
// (src/integrators/bdpt.h:219) and everything below it are the reference's code,
// unchanged.
//
// Modes:
//   ref_bdpt render <scene.toml> W H SPP [--rr D] [--threads T]
//                   [--row-stride S --row-offset O] [--out fb.f32]
//   ref_bdpt sample <scene.toml> W H SPP P K      (one sample: Li + splat list)
//   ref_bdpt dump   <scene.toml> W H OUTDIR       (scene / BVH / camera dump)
//   ref_bdpt exr    <fb.f32> W H <out.exr>        (the reference's saveEXR, utils.h:95-156)
//   ref_bdpt toml   <scene.toml>                  (the reference's loadTOML, main.cpp:22-116, as JSON)
//   ref_bdpt kat    <scene.toml> W H KIND in.f32 out.f32   (per-function known answers, cmdKat)
//   ref_bdpt sample_state <scene.toml> W H SPP RR in.f32 out.f32 -   (render(ray, sampler) from a
//                                                  given std::mt19937 state, cmdSampleState)

#define main tinyrender_reference_main
#include "main.cpp"   // reference src/main.cpp: loadTOML, g_FrameBufferLocks, tinyobj/tinyexr impl
#undef main

#include <integrators/bdpt.h>
#include <integrators/path.h>
// direct.h defines two non-inline free functions that renderer.cpp (which
// includes it for its factory) also defines: renamed here so the driver can
// instantiate DirectIntegrator without a duplicate symbol. Same code.
#define quadratic tr_driver_quadratic
#define raySphereIntersect tr_driver_raySphereIntersect
#include <integrators/direct.h>
#undef quadratic
#undef raySphereIntersect
#include <bsdfs/mixture.h>
#include <bsdfs/glass.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

using namespace TinyRender;

namespace {

struct Cam {
    glm::mat4 worldToCamera, cameraToWorld, cameraToClip, NDCToScreen;
    float invWidth, invHeight, angle, aspectRatio;
};

// renderer.cpp:140-153, verbatim semantics.
Cam makeCam(const Config& cfg, int W, int H) {
    Cam c;
    const float near = 1.f, far = 1000.f;
    c.worldToCamera = glm::lookAt(cfg.camera.o, cfg.camera.at, cfg.camera.up);
    c.cameraToWorld = glm::inverse(c.worldToCamera);
    c.invWidth = 1.f / W;
    c.invHeight = 1.f / H;
    c.angle = std::tanf(deg2rad * cfg.camera.fov * 0.5f);
    c.aspectRatio = (float)W / H;
    c.cameraToClip = glm::perspective(deg2rad * cfg.camera.fov, c.aspectRatio, near, far);
    c.NDCToScreen = glm::scale(glm::mat4(1.f), v3f(W, H, 1.0f)) * glm::scale(glm::mat4(1.f), v3f(0.5f, -0.5f, 1.f)) *
                    glm::translate(glm::mat4(1.f), v3f(1.f, -1.f, 0.f));
    return c;
}

// One camera sample exactly as renderer.cpp:165-195 builds it.
Ray cameraRay(const Config& cfg, const Cam& c, int W, int spp, int pixel, Sampler& sampler) {
    const float near = 1.f, far = 1000.f;
    int j = pixel % W;
    int i = pixel / W;
    float y = (1.f - ((float)i + 0.5f) * c.invHeight) * 2.f - 1.f;
    float x = (((float)j + 0.5f) * c.invWidth) * 2.f - 1.f;
    v4f imagePlanePoint;
    if (spp == 1) {
        imagePlanePoint = v4f(x * c.angle * c.aspectRatio, y * c.angle, -near, 0);
    } else {
        p2f randomSample = sampler.next2D();
        randomSample -= 0.5f;
        randomSample.x = randomSample.x * c.invWidth;
        randomSample.y = randomSample.y * c.invHeight;
        imagePlanePoint = v4f((x + randomSample.x) * c.angle * c.aspectRatio, (y + randomSample.y) * c.angle, -near, 0);
    }
    v3f rayDir = c.cameraToWorld * imagePlanePoint;
    rayDir = glm::normalize(rayDir);
    return Ray(cfg.camera.o, rayDir, near, far);
}

inline int seedFor(int pixel, int spp, int k) {
    return (int)(260450963u + (unsigned)pixel * (unsigned)spp + (unsigned)k);
}

struct Setup {
    Config cfg;
    std::unique_ptr<Scene> scene;
    std::unique_ptr<Integrator> integ;  // BDPTIntegrator, or PathTracerIntegrator for TOML type "path"
    int rrDepth = 0;
};

void setup(Setup& s, const std::string& toml, int W, int H, int spp, int rr) {
    std::cout.setstate(std::ios::failbit);  // silence the reference's progress prints
    loadTOML(s.cfg, toml);
    s.cfg.width = W;
    s.cfg.height = H;
    s.cfg.spp = spp;
    if (rr > 0) s.cfg.integratorSettings.pt.rrDepth = rr;
    s.scene.reset(new Scene(s.cfg));
    if (!s.scene->load(false)) { std::cout.clear(); fprintf(stderr, "scene load failed\n"); exit(2); }
    // the offline integrator the TOML names: "bdpt" (the hot path) or "path"
    // (PathTracerIntegrator, src/integrators/path.h, with its TOML settings)
    if (s.cfg.integrator == EPathTracerIntegrator) s.integ.reset(new PathTracerIntegrator(*s.scene));
    else if (s.cfg.integrator == EDirectIntegrator) s.integ.reset(new DirectIntegrator(*s.scene));
    else s.integ.reset(new BDPTIntegrator(*s.scene));
    s.rrDepth = s.cfg.integratorSettings.pt.rrDepth;
    s.integ->init();
    std::cout.clear();
    g_FrameBufferLocks.reset(new std::mutex[(size_t)W * H]);
}

int cmdRender(int argc, char** argv) {
    std::string toml = argv[2];
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]);
    int rr = 0, threads = 1, rowStride = 1, rowOffset = 0;
    std::string out;
    for (int a = 6; a < argc; a++) {
        std::string k = argv[a];
        if (k == "--rr") rr = atoi(argv[++a]);
        else if (k == "--threads") threads = atoi(argv[++a]);
        else if (k == "--row-stride") rowStride = atoi(argv[++a]);
        else if (k == "--row-offset") rowOffset = atoi(argv[++a]);
        else if (k == "--out") out = argv[++a];
        else { fprintf(stderr, "unknown arg %s\n", k.c_str()); return 2; }
    }
    Setup s;
    setup(s, toml, W, H, spp, rr);
    Cam cam = makeCam(s.cfg, W, H);
    std::vector<int> rows;
    for (int r = rowOffset; r < H; r += rowStride) rows.push_back(r);
    std::atomic<size_t> next(0);
    auto worker = [&]() {
        for (;;) {
            size_t ri = next.fetch_add(1);
            if (ri >= rows.size()) break;
            int row = rows[ri];
            for (int j = 0; j < W; j++) {
                int pixel = row * W + j;
                v3f averageRadiance(0.f);
                for (int k = 0; k < spp; k++) {
                    Sampler sampler(seedFor(pixel, spp, k));
                    Ray ray = cameraRay(s.cfg, cam, W, spp, pixel, sampler);
                    averageRadiance += s.integ->render(ray, sampler);
                }
                std::mutex& lock = g_FrameBufferLocks[pixel];
                lock.lock();
                s.integ->rgb->data[pixel] += averageRadiance * (1.f / spp);
                lock.unlock();
            }
        }
    };
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    double samples = (double)rows.size() * W * spp;
    if (!out.empty()) {
        FILE* f = fopen(out.c_str(), "wb");
        fwrite(&s.integ->rgb->data[0], sizeof(float), (size_t)W * H * 3, f);
        fclose(f);
    }
    printf("{\"samples\": %.0f, \"seconds\": %.6f, \"msamples_per_s\": %.6f, \"threads\": %d, \"rr_depth\": %d}\n",
           samples, sec, samples / sec * 1e-6, threads, s.rrDepth);
    return 0;
}

int cmdSample(int argc, char** argv) {
    if (argc < 8) return 2;
    std::string toml = argv[2];
    int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]), P = atoi(argv[6]), K = atoi(argv[7]);
    Setup s;
    setup(s, toml, W, H, spp, argc > 8 ? atoi(argv[8]) : 0);
    Cam cam = makeCam(s.cfg, W, H);
    Sampler sampler(seedFor(P, spp, K));
    Ray ray = cameraRay(s.cfg, cam, W, spp, P, sampler);
    v3f Li = s.integ->render(ray, sampler);
    printf("ray %a %a %a | %a %a %a\n", ray.o.x, ray.o.y, ray.o.z, ray.d.x, ray.d.y, ray.d.z);
    printf("Li %a %a %a\n", Li.x, Li.y, Li.z);
    for (int p = 0; p < W * H; p++) {
        v3f v = s.integ->rgb->data[p];
        if (v.x != 0.f || v.y != 0.f || v.z != 0.f) printf("splat %d %a %a %a\n", p, v.x, v.y, v.z);
    }
    return 0;
}

void writeBin(const std::string& path, const void* data, size_t bytes) {
    FILE* f = fopen(path.c_str(), "wb");
    fwrite(data, 1, bytes, f);
    fclose(f);
}

int cmdDump(int argc, char** argv) {
    std::string toml = argv[2];
    int W = atoi(argv[3]), H = atoi(argv[4]);
    std::string dir = argv[5];
    Setup s;
    setup(s, toml, W, H, 1, 0);
    const Scene& sc = *s.scene;
    const WorldData& wd = sc.worldData;

    // Triangles in BVH leaf order (AcceleratorBVH::objects is reordered in place
    // by BVH::build, so it IS the build_prims order the flat tree indexes).
    std::vector<float> tf;
    std::vector<int> ti;
    for (Object* o : sc.bvh->objects) {
        auto* n = (AcceleratorBVH::BVHNode*)o;
        const tinyobj::mesh_t& m = wd.shapes[n->shapeID].mesh;
        for (int c = 0; c < 3; c++) {
            const tinyobj::index_t& ix = m.indices[n->faceID + c];
            for (int d = 0; d < 3; d++) tf.push_back(wd.attrib.vertices[3 * ix.vertex_index + d]);
        }
        for (int c = 0; c < 3; c++) {
            const tinyobj::index_t& ix = m.indices[n->faceID + c];
            for (int d = 0; d < 3; d++) tf.push_back(wd.attrib.normals[3 * ix.normal_index + d]);
        }
        ti.push_back((int)n->shapeID);
        ti.push_back((int)(n->faceID / 3));
        ti.push_back(m.material_ids[n->faceID / 3]);
    }
    writeBin(dir + "/tri_f32.bin", tf.data(), tf.size() * 4);
    writeBin(dir + "/tri_i32.bin", ti.data(), ti.size() * 4);

    // Flat BVH nodes in preorder: count by walking from the root.
    const BVHFlatNode* ft = sc.bvh->bvh->flatTree;
    std::vector<uint32_t> stack{0};
    uint32_t maxIdx = 0;
    while (!stack.empty()) {
        uint32_t ni = stack.back();
        stack.pop_back();
        if (ni > maxIdx) maxIdx = ni;
        if (ft[ni].rightOffset != 0) {
            stack.push_back(ni + 1);
            stack.push_back(ni + ft[ni].rightOffset);
        }
    }
    std::vector<float> nb;
    std::vector<uint32_t> ni3;
    for (uint32_t i = 0; i <= maxIdx; i++) {
        const BBox& b = ft[i].bbox;
        float v[6] = {b.min.x, b.min.y, b.min.z, b.max.x, b.max.y, b.max.z};
        nb.insert(nb.end(), v, v + 6);
        ni3.push_back(ft[i].start);
        ni3.push_back(ft[i].nPrims);
        ni3.push_back(ft[i].rightOffset);
    }
    writeBin(dir + "/node_f32.bin", nb.data(), nb.size() * 4);
    writeBin(dir + "/node_u32.bin", ni3.data(), ni3.size() * 4);

    // Camera constants (renderer.cpp:140-153; bdpt.h:49-54, :485-489).
    Cam cam = makeCam(s.cfg, W, H);
    std::vector<float> cf;
    for (const glm::mat4* m : {&cam.worldToCamera, &cam.cameraToWorld, &cam.cameraToClip, &cam.NDCToScreen})
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) cf.push_back((*m)[c][r]);
    v3f fwd = glm::normalize(s.cfg.camera.at - s.cfg.camera.o);
    float vnear = (1.f / std::tanf(deg2rad * s.cfg.camera.fov * 0.5f)) * H * 0.5f;
    float extra[] = {cam.invWidth, cam.invHeight, cam.angle, cam.aspectRatio, fwd.x, fwd.y, fwd.z, vnear};
    cf.insert(cf.end(), extra, extra + 8);
    writeBin(dir + "/camera_f32.bin", cf.data(), cf.size() * 4);

    // Materials: parsed MTL values plus the BSDF constructors' derived constants.
    FILE* f = fopen((dir + "/materials.txt").c_str(), "w");
    for (size_t i = 0; i < wd.materials.size(); i++) {
        const tinyobj::material_t& m = wd.materials[i];
        float scale = 1.f, specW = 0.f;
        if (auto* mx = dynamic_cast<const MixtureBSDF*>(sc.bsdfs[i].get())) { scale = mx->scale; specW = mx->specularSamplingWeight; }
        fprintf(f, "%zu %d %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %a %s\n", i, m.illum,
                m.diffuse[0], m.diffuse[1], m.diffuse[2], m.specular[0], m.specular[1], m.specular[2],
                m.emission[0], m.emission[1], m.emission[2], m.transmittance[0], m.transmittance[1], m.transmittance[2],
                m.shininess, m.ior, scale, specW, 0.f, 0.f, 0.f, 0.f, m.name.c_str());
    }
    fclose(f);
    f = fopen((dir + "/emitters.txt").c_str(), "w");
    for (const Emitter& e : sc.emitters) {
        fprintf(f, "%zu %a %a %a %a %zu", e.shapeID, e.area, e.radiance.x, e.radiance.y, e.radiance.z,
                e.faceAreaDistribution.cdf.size());
        for (float c : e.faceAreaDistribution.cdf) fprintf(f, " %a", c);
        fprintf(f, "\n");
    }
    fclose(f);
    f = fopen((dir + "/shapes.txt").c_str(), "w");
    for (size_t i = 0; i < wd.shapes.size(); i++)
        fprintf(f, "%zu %zu %s\n", i, wd.shapes[i].mesh.indices.size() / 3, wd.shapes[i].name.c_str());
    fclose(f);
    printf("{\"triangles\": %zu, \"nodes\": %u, \"shapes\": %zu, \"materials\": %zu, \"emitters\": %zu}\n",
           sc.bvh->objects.size(), maxIdx + 1, wd.shapes.size(), wd.materials.size(), sc.emitters.size());
    return 0;
}

// Integrator::save's writer (utils.h:95-156) on a raw float32 framebuffer.
int cmdExr(int argc, char** argv) {
    if (argc < 6) return 2;
    const int W = atoi(argv[3]), H = atoi(argv[4]);
    std::unique_ptr<v3f[]> rgb(new v3f[size_t(W) * H]);
    FILE* f = fopen(argv[2], "rb");
    if (!f) return 1;
    const size_t n = fread(rgb.get(), sizeof(float), size_t(W) * H * 3, f);
    fclose(f);
    if (n != size_t(W) * H * 3) return 1;
    return saveEXR(rgb, argv[5], W, H) ? 0 : 1;
}

// loadTOML (main.cpp:22-116) -> the Config fields the BDPT path reads, as JSON.
int cmdToml(int argc, char** argv) {
    Config cfg;
    bool rt;
    try {
        rt = loadTOML(cfg, argv[2]);
    } catch (std::exception const& e) {
        printf("{\"error\": true}\n");
        return 0;
    }
    const auto& c = cfg.camera;
    std::string hex;  // objfile bytes as hex (no JSON escaping questions)
    for (unsigned char ch : cfg.objFile.string()) {
        char b[3];
        snprintf(b, sizeof b, "%02x", ch);
        hex += b;
    }
    printf("{\"error\": false, \"objfile_hex\": \"%s\", \"fov\": \"%a\", \"eye\": [\"%a\", \"%a\", \"%a\"], "
           "\"at\": [\"%a\", \"%a\", \"%a\"], \"up\": [\"%a\", \"%a\", \"%a\"], \"width\": %d, \"height\": %d, "
           "\"realtime\": %d, \"integrator\": %d",
           hex.c_str(), c.fov, c.o.x, c.o.y, c.o.z, c.at.x, c.at.y, c.at.z, c.up.x, c.up.y, c.up.z,
           cfg.width, cfg.height, rt ? 1 : 0, (int)cfg.integrator);
    if (!rt && (cfg.integrator == EBDPTIntegrator || cfg.integrator == EPathTracerIntegrator))
        printf(", \"rrDepth\": %d, \"rrProb\": \"%a\"", cfg.integratorSettings.pt.rrDepth, cfg.integratorSettings.pt.rrProb);
    if (!rt && cfg.integrator == EPathTracerIntegrator)
        printf(", \"isExplicit\": %d, \"maxDepth\": %d, \"emitterSamples\": %zu, \"bsdfSamples\": %zu",
               (int)cfg.integratorSettings.pt.isExplicit, cfg.integratorSettings.pt.maxDepth,
               cfg.integratorSettings.pt.emitterSamples, cfg.integratorSettings.pt.bsdfSamples);
    if (!rt && cfg.integrator == EDirectIntegrator)
        printf(", \"emitterSamples\": %zu, \"bsdfSamples\": %zu, \"samplingStrategy\": \"%s\"",
               cfg.integratorSettings.di.emitterSamples, cfg.integratorSettings.di.bsdfSamples,
               cfg.integratorSettings.di.samplingStrategy.c_str());
    if (!rt) printf(", \"spp\": %d", cfg.spp);
    printf("}\n");
    return 0;
}

std::vector<float> readF32(const std::string& path) {
    std::vector<float> v;
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return v;
    fseek(f, 0, SEEK_END);
    const long n = ftell(f) / 4;
    fseek(f, 0, SEEK_SET);
    v.resize((size_t)n);
    if (fread(v.data(), 4, (size_t)n, f) != (size_t)n) v.clear();
    fclose(f);
    return v;
}

inline int f2i(float x) {
    int i;
    memcpy(&i, &x, 4);
    return i;
}
inline float i2f(int i) {
    float x;
    memcpy(&x, &i, 4);
    return x;
}

// Per-function known-answer outputs of the reference's own functions on
// records read from a float32 file (test fixtures, tests/golden/make_kat_goldens.py):
//   bsdf      in (mat, wo[3], wi[3], u[2])  out (eval[3], pdf, sample f[3], wi[3], pdf, type, null)
//             BSDF::eval / pdf / sample (core.h:308-310) of scene material mat
//   fresnel   in (eta_i, eta_t, cos_i, cos_t)   out F    GlassBSDF::FresnelDielectric (glass.h:40-53)
//   tri       in (ray[8], v0 v1 v2)  out (hit, t, u, v)  rayTriangleIntersect (core.h:379-400)
//   intersect in ray[8]  out (hit, t, u, v, shapeID, primID, matID, p[3], frameNs.n[3], frameNg.n[3],
//             wo[3], -1, occluded)   AcceleratorBVH::intersect (accel.h:125-172) and the any-hit
//             query visibilityQuery makes (bvh.h:259-352, occlusion = true)
//   splat     in p[3]  out (x, y) as int bits   BDPTIntegrator::splatToImagePlane (bdpt.h:485-496)
int cmdKat(int argc, char** argv) {
    if (argc < 8) return 2;
    const std::string toml = argv[2], kind = argv[5];
    const int W = atoi(argv[3]), H = atoi(argv[4]);
    Setup s;
    setup(s, toml, W, H, 1, 0);
    const std::vector<float> in = readF32(argv[6]);
    std::vector<float> out;
    const Scene& sc = *s.scene;
    if (kind == "bsdf") {
        for (size_t r = 0; r + 9 <= in.size(); r += 9) {
            const int mat = f2i(in[r]);
            const BSDF* b = sc.bsdfs[mat].get();
            float o[14] = {0};
            if (!b) {
                o[13] = 1.f;  // illum 5: the reference keeps a null BSDF
            } else {
                SurfaceInteraction si;
                si.wo = v3f(in[r + 1], in[r + 2], in[r + 3]);
                si.wi = v3f(in[r + 4], in[r + 5], in[r + 6]);
                si.matID = mat;
                const v3f f = b->eval(si);
                const float pdf = b->pdf(si);
                SurfaceInteraction so = si;
                float spdf = 0.f;
                const v3f sf = b->sample(so, v2f(in[r + 7], in[r + 8]), &spdf);
                const float vals[13] = {f.x, f.y, f.z, pdf, sf.x, sf.y, sf.z, so.wi.x, so.wi.y, so.wi.z, spdf,
                                        i2f((int)b->getType()), 0.f};
                memcpy(o, vals, sizeof(vals));
            }
            out.insert(out.end(), o, o + 14);
        }
    } else if (kind == "fresnel") {
        const GlassBSDF* g = nullptr;
        for (const auto& b : sc.bsdfs)
            if (!g && b) g = dynamic_cast<const GlassBSDF*>(b.get());
        if (!g) { fprintf(stderr, "no glass material\n"); return 2; }
        for (size_t r = 0; r + 4 <= in.size(); r += 4) out.push_back(g->FresnelDielectric(in[r], in[r + 1], in[r + 2], in[r + 3]));
    } else if (kind == "tri") {
        for (size_t r = 0; r + 17 <= in.size(); r += 17) {
            const Ray ray(v3f(in[r], in[r + 1], in[r + 2]), v3f(in[r + 3], in[r + 4], in[r + 5]), in[r + 6], in[r + 7]);
            float t = 0.f, u = 0.f, v = 0.f;
            const bool hit = rayTriangleIntersect(ray, v3f(in[r + 8], in[r + 9], in[r + 10]),
                                                  v3f(in[r + 11], in[r + 12], in[r + 13]),
                                                  v3f(in[r + 14], in[r + 15], in[r + 16]), t, u, v);
            const float o[4] = {hit ? 1.f : 0.f, t, u, v};
            out.insert(out.end(), o, o + 4);
        }
    } else if (kind == "intersect") {
        for (size_t r = 0; r + 8 <= in.size(); r += 8) {
            const Ray ray(v3f(in[r], in[r + 1], in[r + 2]), v3f(in[r + 3], in[r + 4], in[r + 5]), in[r + 6], in[r + 7]);
            SurfaceInteraction si;
            const bool hit = sc.bvh->intersect(ray, si);
            IntersectionInfo ii = IntersectionInfo();
            const bool occ = sc.bvh->bvh->getIntersection(ray, &ii, true);
            float o[21] = {0};
            o[0] = hit ? 1.f : 0.f;
            o[1] = si.t;
            if (hit) {
                o[2] = si.u, o[3] = si.v;
                o[4] = i2f((int)si.shapeID), o[5] = i2f((int)si.primID), o[6] = i2f(si.matID);
                o[7] = si.p.x, o[8] = si.p.y, o[9] = si.p.z;
                o[10] = si.frameNs.n.x, o[11] = si.frameNs.n.y, o[12] = si.frameNs.n.z;
                o[13] = si.frameNg.n.x, o[14] = si.frameNg.n.y, o[15] = si.frameNg.n.z;
                o[16] = si.wo.x, o[17] = si.wo.y, o[18] = si.wo.z;
            }
            o[19] = i2f(-1);
            o[20] = occ ? 1.f : 0.f;
            out.insert(out.end(), o, o + 21);
        }
    } else if (kind == "splat") {
        const BDPTIntegrator* bi = dynamic_cast<const BDPTIntegrator*>(s.integ.get());
        if (!bi) { fprintf(stderr, "splat needs a bdpt scene\n"); return 2; }
        for (size_t r = 0; r + 3 <= in.size(); r += 3) {
            int x = 0, y = 0;
            bi->splatToImagePlane(v3f(in[r], in[r + 1], in[r + 2]), x, y);
            out.push_back(i2f(x));
            out.push_back(i2f(y));
        }
    } else {
        fprintf(stderr, "unknown kat kind\n");
        return 2;
    }
    writeBin(argv[7], out.data(), out.size() * 4);
    printf("{\"records\": %zu}\n", out.size());
    return 0;
}

// Integrator::render(const Ray&, Sampler&) (integrator.h:31) with an arbitrary
// sampler state: records of (ray[8], std::mt19937 state as 625 words = what
// libstdc++'s operator<< writes: _M_x[624], _M_p). Out per record: Li[3],
// the state after the call (625 words), then the image's non-zero pixels
// after the call (camera splats; rgb cleared first): count, then up to 16
// (pixel, r, g, b) in pixel order.
int cmdSampleState(int argc, char** argv) {
    if (argc < 10) return 2;
    const std::string toml = argv[2];
    const int W = atoi(argv[3]), H = atoi(argv[4]), spp = atoi(argv[5]), rr = atoi(argv[6]);
    Setup s;
    setup(s, toml, W, H, spp, rr);
    const std::vector<float> in = readF32(argv[7]);
    const size_t rec = 8 + 625;
    std::vector<float> out;
    for (size_t r = 0; r + rec <= in.size(); r += rec) {
        const Ray ray(v3f(in[r], in[r + 1], in[r + 2]), v3f(in[r + 3], in[r + 4], in[r + 5]), in[r + 6], in[r + 7]);
        std::ostringstream os;
        for (int k = 0; k < 625; k++) {
            uint32_t w;
            memcpy(&w, &in[r + 8 + k], 4);
            os << w << ' ';
        }
        Sampler sampler(0);
        std::istringstream is(os.str());
        is >> sampler.g;
        s.integ->rgb->clear();
        const v3f Li = s.integ->render(ray, sampler);
        out.push_back(Li.x), out.push_back(Li.y), out.push_back(Li.z);
        std::ostringstream so;
        so << sampler.g;
        std::istringstream si(so.str());
        for (int k = 0; k < 625; k++) {
            unsigned long long w = 0;
            si >> w;
            uint32_t w32 = (uint32_t)w;
            float f;
            memcpy(&f, &w32, 4);
            out.push_back(f);
        }
        std::vector<float> sp;
        int n = 0;
        for (int p = 0; p < W * H; p++) {
            const v3f v = s.integ->rgb->data[p];
            if (v.x != 0.f || v.y != 0.f || v.z != 0.f) {
                if (n < 16) sp.push_back(i2f(p)), sp.push_back(v.x), sp.push_back(v.y), sp.push_back(v.z);
                n++;
            }
        }
        out.push_back(i2f(n));
        sp.resize(64, 0.f);
        out.insert(out.end(), sp.begin(), sp.end());
    }
    writeBin(argv[8], out.data(), out.size() * 4);
    printf("{\"records\": %zu}\n", out.size() / (3 + 625 + 1 + 64));
    (void)argv[9];
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: ref_bdpt render|sample|dump <scene.toml> ...\n");
        return 2;
    }
    std::string cmd = argv[1];
    if (cmd == "render" && argc >= 6) return cmdRender(argc, argv);
    if (cmd == "sample") return cmdSample(argc, argv);
    if (cmd == "dump" && argc >= 6) return cmdDump(argc, argv);
    if (cmd == "exr") return cmdExr(argc, argv);
    if (cmd == "toml") return cmdToml(argc, argv);
    if (cmd == "kat") return cmdKat(argc, argv);
    if (cmd == "sample_state") return cmdSampleState(argc, argv);
    fprintf(stderr, "bad command\n");
    return 2;
}
