// Multi-device frame rendering in one host process: the reference's offline
// loop (renderer.cpp:130-214) fanned out over its worker threads by
// parallel_for (src/core/parallelfor.h:25-65) becomes one context, one stream
// and one full-frame buffer per HIP device. Device i renders the interleaved
// row shard i, i + N, i + 2N, ... (every camera sample of those rows; light
// subpaths splat anywhere, so every device accumulates a whole frame), and one
// RCCL sum-reduce over xGMI (ncclReduce to device 0, communicators from
// ncclCommInitAll) is the path's only exchange. The launches are asynchronous,
// so all devices render concurrently from a single host thread.
//
// RCCL is resolved at first use with dlopen (librccl.so.1 of the ROCm image):
// processes that never render on several devices do not load it. A device list
// that names one device more than once (a single-GPU rehearsal of the
// decomposition) cannot form an RCCL communicator; those buffers are summed on
// the root device by a copy and an element-wise add kernel instead.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "bdpt_amd.h"

namespace bdpt {
int set_error(int code, const std::string& msg);

// dst[i] += src[i] (the repeated-device reduce on the root).
__global__ __launch_bounds__(256) void fb_add_kernel(float* __restrict__ dst, const float* __restrict__ src, size_t n) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * 256)
        dst[i] += src[i];
}
static hipError_t launch_fb_add(float* dst, const float* src, size_t n, hipStream_t st) {
    const unsigned blocks = static_cast<unsigned>(std::min<size_t>((n + 255) / 256, 4096));
    hipLaunchKernelGGL(fb_add_kernel, dim3(blocks), dim3(256), 0, st, dst, src, n);
    return hipGetLastError();
}
}  // namespace bdpt

namespace {

#define MHIP(expr)                                                                                              \
    do {                                                                                                        \
        hipError_t e_ = (expr);                                                                                 \
        if (e_ != hipSuccess) return bdpt::set_error(BDPT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Rccl {
    bool tried = false;
    void* so = nullptr;
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string why;
};

Rccl& rccl() {
    static Rccl r;
    if (r.tried) return r;
    r.tried = true;
    r.so = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!r.so) r.so = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!r.so) {
        const char* e = dlerror();
        r.why = std::string("librccl not loadable: ") + (e ? e : "?");
        return r;
    }
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(r.so, "ncclCommInitAll"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(r.so, "ncclCommDestroy"));
    r.reduce = reinterpret_cast<decltype(r.reduce)>(dlsym(r.so, "ncclReduce"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(r.so, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(r.so, "ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.so, "ncclGetErrorString"));
    if (!r.comm_init_all || !r.comm_destroy || !r.reduce || !r.group_start || !r.group_end || !r.error_string) {
        r.why = "librccl lacks an entry point";
        r.comm_init_all = nullptr;
    }
    return r;
}

int nccl_fail(ncclResult_t res, const char* what) {
    return bdpt::set_error(BDPT_ERR_HIP, std::string(what) + ": " + rccl().error_string(res));
}

}  // namespace

struct bdpt_multi {
    std::vector<int32_t> devices;
    std::vector<bdpt_ctx*> ctx;
    std::vector<hipStream_t> stream;
    std::vector<float*> fb;       // per-device full frame (device i's own memory)
    std::vector<ncclComm_t> comm;  // empty: no RCCL (a repeated device)
    float* stage = nullptr;        // repeated-device reduce: root-device staging buffer
    size_t fb_floats = 0;
    hipEvent_t t0 = nullptr, t1 = nullptr, t2 = nullptr;  // root device: render start, renders done, reduce done
    bdpt_multi_stats stats{};
};

static int multi_buffers(bdpt_multi* m, size_t n) {
    if (n <= m->fb_floats) return BDPT_OK;
    for (size_t i = 0; i < m->devices.size(); i++) {
        MHIP(hipSetDevice(m->devices[i]));
        if (m->fb[i]) MHIP(hipFree(m->fb[i]));
        m->fb[i] = nullptr;
        MHIP(hipMalloc(&m->fb[i], n * sizeof(float)));
    }
    if (m->comm.empty() && m->devices.size() > 1) {
        MHIP(hipSetDevice(m->devices[0]));
        if (m->stage) MHIP(hipFree(m->stage));
        m->stage = nullptr;
        MHIP(hipMalloc(&m->stage, n * sizeof(float)));
    }
    m->fb_floats = n;
    return BDPT_OK;
}

extern "C" {

int bdpt_multi_create(const bdpt_scene* scene, int32_t ndevices, const int32_t* devices, bdpt_multi** out) {
    if (!scene || !out || ndevices < 1 || ndevices > BDPT_MAX_DEVICES || !devices)
        return bdpt::set_error(BDPT_ERR_INVALID, "bad argument (1 <= ndevices <= BDPT_MAX_DEVICES)");
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return bdpt::set_error(BDPT_ERR_NO_DEVICE, "no HIP device");
    for (int i = 0; i < ndevices; i++)
        if (devices[i] < 0 || devices[i] >= count) return bdpt::set_error(BDPT_ERR_INVALID, "bad device index");
    bdpt_multi* m = new bdpt_multi;
    m->devices.assign(devices, devices + ndevices);
    m->ctx.assign(ndevices, nullptr);
    m->stream.assign(ndevices, nullptr);
    m->fb.assign(ndevices, nullptr);
    int rc = BDPT_OK;
    for (int i = 0; i < ndevices && rc == BDPT_OK; i++) {
        rc = bdpt_ctx_create(scene, devices[i], &m->ctx[i]);
        if (rc == BDPT_OK && hipSetDevice(devices[i]) != hipSuccess) rc = bdpt::set_error(BDPT_ERR_HIP, "hipSetDevice");
        if (rc == BDPT_OK && hipStreamCreateWithFlags(&m->stream[i], hipStreamNonBlocking) != hipSuccess)
            rc = bdpt::set_error(BDPT_ERR_HIP, "hipStreamCreate");
    }
    std::vector<int32_t> sorted(m->devices);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    if (rc == BDPT_OK && distinct) {  // RCCL even for N = 1 (a one-rank reduce)
        Rccl& r = rccl();
        if (!r.comm_init_all) {
            rc = bdpt::set_error(BDPT_ERR_UNSUPPORTED, r.why);
        } else {
            m->comm.assign(ndevices, nullptr);
            const ncclResult_t res = r.comm_init_all(m->comm.data(), ndevices, m->devices.data());
            if (res != ncclSuccess) {
                m->comm.clear();
                rc = nccl_fail(res, "ncclCommInitAll");
            }
        }
    }
    if (rc == BDPT_OK && hipSetDevice(devices[0]) == hipSuccess) {
        if (hipEventCreate(&m->t0) != hipSuccess || hipEventCreate(&m->t1) != hipSuccess ||
            hipEventCreate(&m->t2) != hipSuccess)
            rc = bdpt::set_error(BDPT_ERR_HIP, "hipEventCreate");
    }
    if (rc != BDPT_OK) {
        const std::string msg = bdpt_last_error();
        bdpt_multi_destroy(m);
        return bdpt::set_error(rc, msg);
    }
    m->stats.devices = ndevices;
    m->stats.rccl = m->comm.empty() ? 0 : 1;
    *out = m;
    return BDPT_OK;
}

int bdpt_multi_destroy(bdpt_multi* m) {
    if (!m) return BDPT_OK;
    for (size_t i = 0; i < m->devices.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        if (m->stream[i]) (void)hipStreamSynchronize(m->stream[i]);
    }
    for (ncclComm_t c : m->comm)
        if (c) rccl().comm_destroy(c);
    for (size_t i = 0; i < m->devices.size(); i++) {
        (void)hipSetDevice(m->devices[i]);
        if (m->fb[i]) (void)hipFree(m->fb[i]);
        if (m->stream[i]) (void)hipStreamDestroy(m->stream[i]);
        if (m->ctx[i]) bdpt_ctx_destroy(m->ctx[i]);
    }
    if (!m->devices.empty()) {
        (void)hipSetDevice(m->devices[0]);
        if (m->stage) (void)hipFree(m->stage);
        if (m->t0) (void)hipEventDestroy(m->t0);
        if (m->t1) (void)hipEventDestroy(m->t1);
        if (m->t2) (void)hipEventDestroy(m->t2);
    }
    delete m;
    return BDPT_OK;
}

int bdpt_multi_render_host(bdpt_multi* m, const bdpt_frame_params* params, const bdpt_path_params* path,
                           const bdpt_direct_params* direct, float* fb_host) {
    if (!m || !params || !fb_host) return bdpt::set_error(BDPT_ERR_INVALID, "null argument");
    if (path && direct) return bdpt::set_error(BDPT_ERR_INVALID, "one integrator per call");
    if (params->width <= 0 || params->height <= 0 || params->spp <= 0)
        return bdpt::set_error(BDPT_ERR_INVALID, "width/height/spp must be > 0");
    if (params->row_offset != 0 || params->row_stride != 1)
        return bdpt::set_error(BDPT_ERR_INVALID, "the multi-device render shards the whole image itself");
    const int N = static_cast<int>(m->devices.size());
    const size_t n = static_cast<size_t>(params->width) * params->height * 3;
    int rc;
    if ((rc = multi_buffers(m, n))) return rc;
    const auto wall0 = std::chrono::steady_clock::now();
    // root accumulates onto the caller's frame (the bdpt_render_host convention)
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipEventRecord(m->t0, m->stream[0]));
    MHIP(hipMemcpyAsync(m->fb[0], fb_host, n * sizeof(float), hipMemcpyHostToDevice, m->stream[0]));
    for (int i = 1; i < N; i++) {
        MHIP(hipSetDevice(m->devices[i]));
        MHIP(hipMemsetAsync(m->fb[i], 0, n * sizeof(float), m->stream[i]));
    }
    for (int i = 0; i < N; i++) {  // bdpt::dist.row_shard: device i renders rows i, i + N, ...
        bdpt_frame_params p = *params;
        p.row_offset = i;
        p.row_stride = N;
        if (path) rc = bdpt_render_path(m->ctx[i], &p, path, m->fb[i], m->stream[i]);
        else if (direct) rc = bdpt_render_direct(m->ctx[i], &p, direct, m->fb[i], m->stream[i]);
        else rc = bdpt_render(m->ctx[i], &p, m->fb[i], m->stream[i]);
        if (rc) return rc;
    }
    // renders done on every device: the root's t1 waits for the others' streams
    for (int i = 1; i < N; i++) {
        hipEvent_t ev;
        MHIP(hipSetDevice(m->devices[i]));
        MHIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        MHIP(hipEventRecord(ev, m->stream[i]));
        MHIP(hipSetDevice(m->devices[0]));
        MHIP(hipStreamWaitEvent(m->stream[0], ev, 0));
        MHIP(hipEventDestroy(ev));
    }
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipEventRecord(m->t1, m->stream[0]));
    if (!m->comm.empty()) {
        Rccl& r = rccl();
        ncclResult_t res = r.group_start();
        for (int i = 0; i < N && res == ncclSuccess; i++) {
            MHIP(hipSetDevice(m->devices[i]));
            res = r.reduce(m->fb[i], i == 0 ? m->fb[0] : nullptr, n, ncclFloat, ncclSum, 0, m->comm[i], m->stream[i]);
        }
        const ncclResult_t end = r.group_end();
        if (res != ncclSuccess) return nccl_fail(res, "ncclReduce");
        if (end != ncclSuccess) return nccl_fail(end, "ncclGroupEnd");
    } else {
        for (int i = 1; i < N; i++) {  // repeated device: copy + add on the root
            MHIP(hipSetDevice(m->devices[0]));
            MHIP(hipMemcpyPeerAsync(m->stage, m->devices[0], m->fb[i], m->devices[i], n * sizeof(float),
                                    m->stream[0]));
            MHIP(bdpt::launch_fb_add(m->fb[0], m->stage, n, m->stream[0]));
        }
    }
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipEventRecord(m->t2, m->stream[0]));
    MHIP(hipMemcpyAsync(fb_host, m->fb[0], n * sizeof(float), hipMemcpyDeviceToHost, m->stream[0]));
    for (int i = 0; i < N; i++) {
        MHIP(hipSetDevice(m->devices[i]));
        MHIP(hipStreamSynchronize(m->stream[i]));
    }
    float render_ms = 0.f, reduce_ms = 0.f;
    MHIP(hipSetDevice(m->devices[0]));
    MHIP(hipEventElapsedTime(&render_ms, m->t0, m->t1));
    MHIP(hipEventElapsedTime(&reduce_ms, m->t1, m->t2));
    m->stats.render_ms = render_ms;
    m->stats.reduce_ms = reduce_ms;
    m->stats.wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
    m->stats.samples = 0;
    m->stats.capped_samples = 0;
    m->stats.schedule_errors = 0;
    for (int i = 0; i < N; i++) {
        bdpt_stats s;
        if ((rc = bdpt_get_stats(m->ctx[i], &s))) return rc;
        m->stats.kernel_ms[i] = s.kernel_ms;
        m->stats.device_samples[i] = s.samples;
        m->stats.samples += s.samples;
        m->stats.capped_samples += s.capped_samples;
        m->stats.schedule_errors += s.schedule_errors;
    }
    // as bdpt_render_host: MT19937 draws past the generated ring (or a continuation
    // walk out of stack) on any device mean the frame was rendered from wrong numbers
    if (m->stats.schedule_errors)
        return bdpt::set_error(BDPT_ERR_HIP, std::to_string(m->stats.schedule_errors) +
                                                 " schedule errors over the devices (MT19937 draws past the "
                                                 "generated ring, or a continuation walk out of stack)");
    // as bdpt_render_host: a Russian-roulette frame in which some sample met the
    // light-vertex store or the bounce guard is not the reference's image
    if (params->russian_roulette && !path && !direct && m->stats.capped_samples)
        return bdpt::set_error(BDPT_ERR_UNSUPPORTED, std::to_string(m->stats.capped_samples) +
                                                         " samples met the Russian-roulette bounds (light-vertex store / "
                                                         "bounce guard); the image is not the reference's");
    return BDPT_OK;
}

int bdpt_multi_get_stats(bdpt_multi* m, bdpt_multi_stats* out) {
    if (!m || !out) return bdpt::set_error(BDPT_ERR_INVALID, "null argument");
    *out = m->stats;
    return BDPT_OK;
}

}  // extern "C"
