// Checks INTEGRATION.md's reference-side binding through the reference's own types.
//
// TEST INFRASTRUCTURE ONLY. Compiled (oracle/ref/Makefile, target `adapter`)
// with the reference's sources plus the adapter header and registration edits
// that make_adapter.py extracts verbatim from INTEGRATION.md, linked against the
// product library lib/libbdpt_amd.so. Outputs go to oracle/_ref/adapter/.
//
// Modes:
//   adapter_check layout <scene.toml>
//       Scene::load (renderer.cpp:235-315), then GpuBDPTIntegrator::uploadScene
//       (bdpt_scene_create from the Scene) against bdpt_scene_load_obj of the same
//       OBJ: every device array (bdpt_scene_export_layout) must be equal bit for
//       bit. No GPU needed.
//   adapter_check frame <scene.toml> W H SPP out.f32
//       loadTOML (with the `type = "bdpt_gpu"` edit) -> Renderer::init (the factory
//       edit) -> Renderer::render (the offline-branch edit: renderFrame on the GPU)
//       -> the framebuffer as float32; then Renderer::cleanUp (EXR next to the TOML).
//   adapter_check samples <scene.toml> W H SPP N STRIDE
//       For N camera samples (pixel q*STRIDE mod W*H, sample q mod SPP, seeded as
//       the goldens are): GpuBDPTIntegrator::render(ray, sampler) against the
//       reference BDPTIntegrator::render(ray, sampler) on the same Scene and the same
//       Sampler state. Li bit for bit, the std::mt19937 state after the call equal,
//       and the camera splats (both rgb buffers, cleared before each sample) bit for
//       bit. Prints a JSON summary; exit status 1 on any mismatch.
#define main tinyrender_reference_main
#include "main.cpp"  // the edited copy (oracle/_ref/adapter/src/main.cpp): loadTOML, g_FrameBufferLocks
#undef main

#include <integrators/bdpt.h>
#include <integrators/bdpt_gpu.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

using namespace TinyRender;

namespace {

int layout(const std::string& toml) {
    Config cfg;
    std::cout.setstate(std::ios::failbit);
    loadTOML(cfg, toml);
    Scene scene(cfg);
    const bool ok = scene.load(false);
    std::cout.clear();
    if (!ok) return fprintf(stderr, "scene load failed\n"), 2;
    GpuBDPTIntegrator g(scene);
    g.m_gpu = new GpuBDPTIntegrator::Gpu();
    g.uploadScene();  // bdpt_scene_create from the reference's Scene
    fs::path obj(cfg.objFile);
    if (!obj.is_absolute()) obj = (cfg.tomlFile.parent_path() / obj).make_preferred();  // renderer.cpp:240-241
    bdpt_scene* fromObj = nullptr;
    if (bdpt_scene_load_obj(obj.string().c_str(), &fromObj) != BDPT_OK)
        return fprintf(stderr, "load_obj: %s\n", bdpt_last_error()), 2;
    int bad = 0;
    long long total = 0;
    printf("{\"arrays\": [");
    for (int a = 0; a < BDPT_LAYOUT_ARRAYS; a++) {
        int64_t na = 0, nb = 0;
        bdpt_scene_export_layout(g.m_gpu->scene, a, nullptr, &na);
        bdpt_scene_export_layout(fromObj, a, nullptr, &nb);
        std::vector<unsigned char> A((size_t)na), B((size_t)nb);
        bdpt_scene_export_layout(g.m_gpu->scene, a, A.data(), &na);
        bdpt_scene_export_layout(fromObj, a, B.data(), &nb);
        const bool same = na == nb && (na == 0 || std::memcmp(A.data(), B.data(), (size_t)na) == 0);
        bad += !same;
        total += na;
        printf("%s{\"id\": %d, \"bytes\": %lld, \"equal\": %s}", a ? ", " : "", a, (long long)na, same ? "true" : "false");
    }
    bdpt_scene_info ia, ib;
    bdpt_scene_get_info(g.m_gpu->scene, &ia);
    bdpt_scene_get_info(fromObj, &ib);
    const bool infoSame = std::memcmp(&ia, &ib, sizeof(ia)) == 0;
    bad += !infoSame;
    printf("], \"bytes\": %lld, \"info_equal\": %s, \"triangles\": %lld, \"mismatches\": %d}\n", total,
           infoSame ? "true" : "false", (long long)ia.triangles, bad);
    bdpt_scene_free(fromObj);
    g.release();
    return bad ? 1 : 0;
}

int frame(const std::string& toml, int W, int H, int spp, const std::string& out) {
    Config config;
    loadTOML(config, toml);
    if (config.integrator != EBDPTGpuIntegrator) return fprintf(stderr, "the scene file must say type = \"bdpt_gpu\"\n"), 2;
    config.width = W, config.height = H, config.spp = spp;
    Renderer renderer(config);
    if (!renderer.init(false, true)) return fprintf(stderr, "Renderer::init failed\n"), 2;
    g_FrameBufferLocks.reset(new std::mutex[(size_t)W * H]);
    renderer.render();
    FILE* f = fopen(out.c_str(), "wb");
    fwrite(&renderer.integrator->rgb->data[0], sizeof(float), (size_t)W * H * 3, f);
    fclose(f);
    renderer.cleanUp();
    printf("{\"integrator\": \"%s\", \"width\": %d, \"height\": %d, \"spp\": %d}\n",
           dynamic_cast<GpuBDPTIntegrator*>(renderer.integrator.get()) ? "GpuBDPTIntegrator" : "other", W, H, spp);
    return 0;
}

// renderer.cpp:140-153 and :165-195 (the camera ray of one sample), as the goldens' driver builds it.
Ray cameraRay(const Config& cfg, int W, int H, int spp, int pixel, Sampler& sampler) {
    const float near = 1.f, far = 1000.f;
    const glm::mat4 cameraToWorld = glm::inverse(glm::lookAt(cfg.camera.o, cfg.camera.at, cfg.camera.up));
    const float invWidth = 1.f / W, invHeight = 1.f / H;
    const float angle = std::tanf(deg2rad * cfg.camera.fov * 0.5f);
    const float aspectRatio = (float)W / H;
    const int j = pixel % W, i = pixel / W;
    const float y = (1.f - ((float)i + 0.5f) * invHeight) * 2.f - 1.f;
    const float x = (((float)j + 0.5f) * invWidth) * 2.f - 1.f;
    v4f imagePlanePoint;
    if (spp == 1) {
        imagePlanePoint = v4f(x * angle * aspectRatio, y * angle, -near, 0);
    } else {
        p2f randomSample = sampler.next2D();
        randomSample -= 0.5f;
        randomSample.x = randomSample.x * invWidth;
        randomSample.y = randomSample.y * invHeight;
        imagePlanePoint = v4f((x + randomSample.x) * angle * aspectRatio, (y + randomSample.y) * angle, -near, 0);
    }
    v3f rayDir = cameraToWorld * imagePlanePoint;
    rayDir = glm::normalize(rayDir);
    return Ray(cfg.camera.o, rayDir, near, far);
}

inline bool sameBits(float a, float b) { return std::memcmp(&a, &b, 4) == 0; }

int samples(const std::string& toml, int W, int H, int spp, int n, int stride) {
    Config config;
    loadTOML(config, toml);
    if (config.integrator != EBDPTGpuIntegrator) return fprintf(stderr, "the scene file must say type = \"bdpt_gpu\"\n"), 2;
    config.width = W, config.height = H, config.spp = spp;
    std::cout.setstate(std::ios::failbit);
    Renderer renderer(config);
    const bool ok = renderer.init(false, true);
    BDPTIntegrator ref(renderer.scene);  // the CPU integrator on the same Scene
    ref.init();
    std::cout.clear();
    if (!ok) return fprintf(stderr, "Renderer::init failed\n"), 2;
    g_FrameBufferLocks.reset(new std::mutex[(size_t)W * H]);
    Integrator& gpu = *renderer.integrator;
    long long liBad = 0, stBad = 0, spBad = 0, nonzero = 0, splatPixels = 0;
    for (int q = 0; q < n; q++) {
        const int pixel = (int)(((long long)q * stride) % ((long long)W * H)), k = q % spp;
        Sampler s((int)(260450963u + (unsigned)pixel * (unsigned)spp + (unsigned)k));
        const Ray ray = cameraRay(config, W, H, spp, pixel, s);
        Sampler a = s, b = s;
        gpu.rgb->clear();
        ref.rgb->clear();
        const v3f lg = gpu.render(ray, a);
        const v3f lr = ref.render(ray, b);
        liBad += !(sameBits(lg.x, lr.x) && sameBits(lg.y, lr.y) && sameBits(lg.z, lr.z));
        stBad += !(a.g == b.g);
        nonzero += lr.x != 0.f || lr.y != 0.f || lr.z != 0.f;
        bool sp = true;
        for (int p = 0; p < W * H; p++) {
            const v3f u = gpu.rgb->data[p], v = ref.rgb->data[p];
            sp = sp && sameBits(u.x, v.x) && sameBits(u.y, v.y) && sameBits(u.z, v.z);
            splatPixels += v.x != 0.f || v.y != 0.f || v.z != 0.f;
        }
        spBad += !sp;
    }
    static_cast<GpuBDPTIntegrator&>(gpu).release();
    printf("{\"samples\": %d, \"li_mismatch\": %lld, \"state_mismatch\": %lld, \"splat_mismatch\": %lld, "
           "\"nonzero_li\": %lld, \"splat_pixels\": %lld}\n",
           n, liBad, stBad, spBad, nonzero, splatPixels);
    return (liBad || stBad || spBad) ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "";
    if (mode == "layout" && argc == 3) return layout(argv[2]);
    if (mode == "frame" && argc == 7) return frame(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), argv[6]);
    if (mode == "samples" && argc == 8)
        return samples(argv[2], atoi(argv[3]), atoi(argv[4]), atoi(argv[5]), atoi(argv[6]), atoi(argv[7]));
    fprintf(stderr, "usage: adapter_check layout TOML | frame TOML W H SPP OUT | samples TOML W H SPP N STRIDE\n");
    return 2;
}
