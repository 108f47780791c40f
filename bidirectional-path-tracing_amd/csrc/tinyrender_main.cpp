// tinyrender_amd — the reference's command line (src/main.cpp:121-181,
// `tinyrender <scene.toml> [nogui]`) for the BDPT path on an MI355X:
// loadTOML -> Scene::load -> Integrator::init -> the timed render
// (main.cpp:146-152, "Render took: ... seconds.") -> Integrator::save, which
// writes the EXR next to the TOML (integrator.cpp:26-30).
//
// Offline `type = "bdpt"` (the hot path), `type = "path"` and `type = "direct"`
// (the reference's PathTracerIntegrator and DirectIntegrator on the same
// substrate) are accepted; the other
// integrators and the realtime render passes are rejected with an error.
// Optional overrides (not in the reference): --width W --height H --spp N
// --rr D --device K --out FILE.exr --seed S, and --gpus N / --devices a,b,...
// to render on several devices (row shards + one RCCL sum-reduce, bdpt_multi_*).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bdpt_amd.h"

namespace {

int die(const char* what) {
    std::fprintf(stderr, "%s: %s\n", what, bdpt_last_error());
    return EXIT_FAILURE;
}

// fs::path::replace_extension("exr") on the TOML path (integrator.cpp:28).
std::string exr_path_of(const std::string& toml) {
    const size_t slash = toml.find_last_of('/');
    const size_t dot = toml.find_last_of('.');
    const size_t name = slash == std::string::npos ? 0 : slash + 1;
    // a leading dot names the file (".toml"), it is not an extension
    if (dot == std::string::npos || dot <= name || (dot == name && toml.size() > name)) return toml + ".exr";
    return toml.substr(0, dot) + ".exr";
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "Syntax: %s <scene.toml> [nogui] [--width W --height H --spp N --rr D --device K "
                             "--out FILE.exr --seed S --gpus N --devices a,b,...]\n", argv[0]);
        return EXIT_FAILURE;
    }
    const std::string toml = argv[1];
    int W = -1, H = -1, spp = -1, rr = -1, device = 0;
    long long seed = -1;
    std::string out;
    std::vector<int32_t> devices;  // non-empty: the multi-device render
    for (int i = 2; i < argc; i++) {
        const std::string a = argv[i];
        auto next = [&](const char* flag) -> const char* {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", flag);
                std::exit(EXIT_FAILURE);
            }
            return argv[++i];
        };
        if (a == "nogui") continue;  // there is no GUI on this path
        else if (a == "--width") W = std::atoi(next("--width"));
        else if (a == "--height") H = std::atoi(next("--height"));
        else if (a == "--spp") spp = std::atoi(next("--spp"));
        else if (a == "--rr") rr = std::atoi(next("--rr"));
        else if (a == "--device") device = std::atoi(next("--device"));
        else if (a == "--seed") seed = std::atoll(next("--seed"));
        else if (a == "--out") out = next("--out");
        else if (a == "--gpus") {
            const int n = std::atoi(next("--gpus"));
            devices.clear();
            for (int k = 0; k < n; k++) devices.push_back(k);
        } else if (a == "--devices") {
            devices.clear();
            for (const char* q = next("--devices"); *q;) {
                devices.push_back(static_cast<int32_t>(std::strtol(q, const_cast<char**>(&q), 10)));
                if (*q == ',') q++;
                else if (*q) break;
            }
        }
        else {
            std::fprintf(stderr, "unknown argument %s\n", a.c_str());
            return EXIT_FAILURE;
        }
    }

    bdpt_config cfg;
    if (bdpt_config_load_toml(toml.c_str(), &cfg) != BDPT_OK) {
        std::fprintf(stderr, "Error while parsing scene file: %s\n", bdpt_last_error());  // main.cpp:128-131
        return EXIT_FAILURE;
    }
    if (cfg.realtime) {
        std::fprintf(stderr, "realtime render passes are not part of the MI355X BDPT path\n");
        return EXIT_FAILURE;
    }
    std::printf("%s\n", cfg.integrator);  // main.cpp:72
    const bool path = std::strcmp(cfg.integrator, "path") == 0;
    const bool direct = std::strcmp(cfg.integrator, "direct") == 0;
    if (!path && !direct && std::strcmp(cfg.integrator, "bdpt") != 0) {
        std::fprintf(stderr, "integrator type \"%s\" is not part of the MI355X BDPT path\n", cfg.integrator);
        return EXIT_FAILURE;
    }
    if (W > 0) cfg.width = W;
    if (H > 0) cfg.height = H;
    if (spp > 0) cfg.spp = spp;
    if (rr > 0) cfg.rr_depth = rr;

    bdpt_scene* scene = nullptr;
    if (bdpt_scene_load_obj(cfg.obj_file, &scene) != BDPT_OK) return die("Scene::load");
    bdpt_ctx* ctx = nullptr;
    bdpt_multi* multi = nullptr;
    if (!devices.empty()) {
        if (bdpt_multi_create(scene, static_cast<int32_t>(devices.size()), devices.data(), &multi) != BDPT_OK)
            return die("bdpt_multi_create");
    } else if (bdpt_ctx_create(scene, device, &ctx) != BDPT_OK) {
        return die("bdpt_ctx_create");
    }

    bdpt_frame_params p;
    std::memset(&p, 0, sizeof(p));
    p.camera = cfg.camera;
    p.width = cfg.width;
    p.height = cfg.height;
    p.spp = cfg.spp;
    p.rr_depth = cfg.rr_depth;
    p.strategy = BDPT_STRATEGY_BDPT;
    p.seed_base = seed >= 0 ? static_cast<uint32_t>(seed) : 260450963u;  // renderer.cpp:155
    p.row_offset = 0;
    p.row_stride = 1;
    std::vector<float> rgb(static_cast<size_t>(cfg.width) * cfg.height * 3, 0.f);  // Integrator::init: rgb->clear()

    const auto t0 = std::chrono::high_resolution_clock::now();
    if (path) {
        if (rr > 0) cfg.path.rr_depth = rr;
        p.rr_depth = 1;  // unused by the path tracer
        const int rc = multi ? bdpt_multi_render_host(multi, &p, &cfg.path, nullptr, rgb.data())
                             : bdpt_render_path_host(ctx, &p, &cfg.path, rgb.data());
        if (rc != BDPT_OK) return die("render (path)");
    } else if (direct) {
        p.rr_depth = 1;  // unused by the direct integrator
        const int rc = multi ? bdpt_multi_render_host(multi, &p, nullptr, &cfg.direct, rgb.data())
                             : bdpt_render_direct_host(ctx, &p, &cfg.direct, rgb.data());
        if (rc != BDPT_OK) {
            if (cfg.direct.sampling_strategy == 0) {  // direct.h:460-461
                std::printf("Error: wrong strategy\n");
                return EXIT_FAILURE;
            }
            return die("render (direct)");
        }
    } else if ((multi ? bdpt_multi_render_host(multi, &p, nullptr, nullptr, rgb.data())
                      : bdpt_render_host(ctx, &p, rgb.data())) != BDPT_OK) {
        return die("render (bdpt)");
    }
    const auto t1 = std::chrono::high_resolution_clock::now();
    std::printf("Render took: %g seconds.\n", std::chrono::duration<double>(t1 - t0).count());
    if (multi) {
        bdpt_multi_stats st;
        bdpt_multi_get_stats(multi, &st);
        std::printf("%d devices (%s): render %.3f ms, reduce %.3f ms\n", st.devices, st.rccl ? "RCCL reduce" : "local sum",
                    st.render_ms, st.reduce_ms);
    }

    const std::string exr = out.empty() ? exr_path_of(toml) : out;
    if (bdpt_save_exr(rgb.data(), cfg.width, cfg.height, exr.c_str()) != BDPT_OK) return die("saveEXR");
    std::printf("\nSaved EXR image to %s\n", exr.c_str());  // utils.h:149
    if (multi) bdpt_multi_destroy(multi);
    if (ctx) bdpt_ctx_destroy(ctx);
    bdpt_scene_free(scene);
    return EXIT_SUCCESS;
}
