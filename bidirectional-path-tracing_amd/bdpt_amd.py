"""Python host binding of the MI355X BDPT library (lib/libbdpt_amd.so).

Mirrors the reference's plugin surface for the BDPT path
(JackMinn/Bidirectional-Path-Tracing):

  Scene(obj_path)                      Scene::load          src/core/renderer.cpp:235-315
  BDPTIntegrator(scene, config)        BDPTIntegrator ctor  src/integrators/bdpt.h:38-43
    .init()                            Integrator::init     src/core/integrator.cpp:16-20 (allocates rgb)
    .render(ray, sampler) -> Li        Integrator::render   bdpt.h:219-241 (one camera sample)
    .render_frame(...)                 Renderer::render offline loop renderer.cpp:130-214
    .rgb                               Integrator::rgb      (W x H x 3 float32, accumulated)
  Sampler(seed)                        Sampler              src/core/math.h:63-76 (seed + draw count)
  Ray(o, d, min_t, max_t)              Ray                  src/core/core.h:117-122
  load_toml(path) -> SceneConfig       loadTOML             src/main.cpp:22-116
  PathTracerIntegrator(scene, config, PathSettings)
                                       PathTracerIntegrator src/integrators/path.h (TOML type = "path")
  save_exr(rgb, W, H, path)            Integrator::save     integrator.cpp:26-30 -> saveEXR utils.h:95-156

Everything renders on the GPU through the C-ABI of include/bdpt_amd.h; there
is no CPU fallback (a missing library or device raises).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BDPT_AMD_LIB selects an alternative in-tree build (kernel-variant experiments).
LIB_PATH = os.environ.get("BDPT_AMD_LIB") or os.path.join(HERE, "lib", "libbdpt_amd.so")

STRATEGY_BDPT, STRATEGY_LIGHT_TRACING, STRATEGY_PATH_TRACING = 0, 1, 2
RR_NONE, RR_LUMINANCE = 0, 1  # bdpt_frame_params.russian_roulette (BDPT_RR_*)
FLAG_COUNT, FLAG_FULL_TRAVERSAL = 1, 2
REFERENCE_SEED = 260450963  # renderer.cpp:155
COUNTER_NAMES = ["closest_rays", "shadow_rays", "interior_visits", "tri_tests", "light_verts",
                 "light_vert_reads", "splats", "rng_draws", "trav_lane_iters", "trav_wave_iters",
                 "shade_lane_actions", "shade_wave_actions", "trav_clocks", "shade_clocks", "loop_clocks",
                 "slab_fallbacks", "stack_gt8", "stack_gt12", "stack_gt16", "pop_culled",
                 "clk_resolve", "clk_start_eye", "clk_eye_vertex", "clk_emitter_sample", "clk_start_light",
                 "clk_nee", "clk_light_vertex", "clk_connect", "clk_continue", "clk_light_next", "clk_eye_next",
                 "clk_finish"]


class BdptError(RuntimeError):
    pass


class _Camera(ctypes.Structure):
    _fields_ = [("eye", ctypes.c_float * 3), ("at", ctypes.c_float * 3), ("up", ctypes.c_float * 3),
                ("fov", ctypes.c_float)]


class _FrameParams(ctypes.Structure):
    _fields_ = [("camera", _Camera), ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("spp", ctypes.c_int32),
                ("rr_depth", ctypes.c_int32), ("strategy", ctypes.c_int32), ("seed_base", ctypes.c_uint32),
                ("row_offset", ctypes.c_int32), ("row_stride", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("russian_roulette", ctypes.c_int32)]


class _SceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int64) for n in
                ("triangles", "bvh_nodes", "shapes", "materials", "emitters", "bvh_max_depth", "device_bytes",
                 "bvh_leaves", "wide_nodes", "wide_depth", "wide_max_stack", "wide_leaves", "triangle_tree")]


class _PathParams(ctypes.Structure):  # bdpt_path_params
    _fields_ = [("is_explicit", ctypes.c_int32), ("max_depth", ctypes.c_int32), ("rr_depth", ctypes.c_int32),
                ("rr_prob", ctypes.c_float), ("emitter_samples", ctypes.c_int32), ("bsdf_samples", ctypes.c_int32)]


class _DirectParams(ctypes.Structure):  # bdpt_direct_params
    _fields_ = [("sampling_strategy", ctypes.c_int32), ("emitter_samples", ctypes.c_int32),
                ("bsdf_samples", ctypes.c_int32)]


class _Config(ctypes.Structure):  # bdpt_config
    _fields_ = [("toml_file", ctypes.c_char * 4096), ("obj_file_raw", ctypes.c_char * 4096),
                ("obj_file", ctypes.c_char * 4096), ("camera", _Camera), ("width", ctypes.c_int32),
                ("height", ctypes.c_int32), ("realtime", ctypes.c_int32), ("integrator", ctypes.c_char * 32),
                ("rr_depth", ctypes.c_int32), ("rr_prob", ctypes.c_float), ("spp", ctypes.c_int32),
                ("path", _PathParams), ("direct", _DirectParams), ("sampling_strategy", ctypes.c_char * 32)]


class _Splat(ctypes.Structure):  # bdpt_splat
    _fields_ = [("pixel", ctypes.c_int32), ("rgb", ctypes.c_float * 3)]


# bdpt_hit (AcceleratorBVH::intersect's SurfaceInteraction fields)
HIT_DTYPE = np.dtype([("hit", np.int32), ("t", np.float32), ("u", np.float32), ("v", np.float32),
                      ("shape_id", np.int32), ("prim_id", np.int32), ("mat_id", np.int32), ("p", np.float32, 3),
                      ("ns", np.float32, 3), ("ng", np.float32, 3), ("wo", np.float32, 3), ("tri", np.int32)])


def _af32(a, cols):
    return np.ascontiguousarray(np.asarray(a, np.float32).reshape(-1, cols))


def _ai32(a):
    return np.ascontiguousarray(np.asarray(a, np.int32).reshape(-1))


MAX_DEVICES = 16  # BDPT_MAX_DEVICES


class _MultiStats(ctypes.Structure):  # bdpt_multi_stats
    _fields_ = [("devices", ctypes.c_int32), ("rccl", ctypes.c_int32), ("wall_ms", ctypes.c_double),
                ("render_ms", ctypes.c_double), ("reduce_ms", ctypes.c_double), ("samples", ctypes.c_int64),
                ("kernel_ms", ctypes.c_double * MAX_DEVICES), ("device_samples", ctypes.c_int64 * MAX_DEVICES),
                ("capped_samples", ctypes.c_int64), ("schedule_errors", ctypes.c_int64)]


class _MaterialDesc(ctypes.Structure):  # bdpt_material_desc
    _fields_ = [("illum", ctypes.c_int32), ("kd", ctypes.c_float * 3), ("ks", ctypes.c_float * 3),
                ("ke", ctypes.c_float * 3), ("tf", ctypes.c_float * 3), ("ns", ctypes.c_float), ("ni", ctypes.c_float),
                ("scale", ctypes.c_float), ("spec_weight", ctypes.c_float), ("has_texture", ctypes.c_int32)]


class _EmitterDesc(ctypes.Structure):  # bdpt_emitter_desc
    _fields_ = [("shape", ctypes.c_int32), ("area", ctypes.c_float), ("radiance", ctypes.c_float * 3),
                ("ncdf", ctypes.c_int32), ("cdf", ctypes.c_void_p)]


class _BvhNodeDesc(ctypes.Structure):  # bdpt_bvh_node_desc
    _fields_ = [("bmin", ctypes.c_float * 3), ("bmax", ctypes.c_float * 3), ("start", ctypes.c_uint32),
                ("nprims", ctypes.c_uint32), ("right_offset", ctypes.c_uint32)]


class _SceneDesc(ctypes.Structure):  # bdpt_scene_desc
    _fields_ = [("triangles", ctypes.c_int64), ("positions", ctypes.c_void_p), ("normals", ctypes.c_void_p),
                ("tri_shape", ctypes.c_void_p), ("tri_prim", ctypes.c_void_p), ("tri_mat", ctypes.c_void_p),
                ("shapes", ctypes.c_int32), ("materials", ctypes.c_int32), ("material", ctypes.c_void_p),
                ("emitters", ctypes.c_int32), ("emitter", ctypes.c_void_p), ("bvh_nodes", ctypes.c_int64),
                ("bvh", ctypes.c_void_p), ("bvh_order", ctypes.c_void_p)]


# BsdfKind (bdpt_types.h) -> the MTL illum that selects it (renderer.cpp:258-271)
KIND_ILLUM = {0: 5, 1: 7, 2: 3, 3: 6, 4: 8, 5: 2}
LAYOUT_ARRAYS = ("tri", "shade", "nodes", "wnodes", "wtri", "lbox", "bsdfs", "emitters", "emit_tri", "emit_cdf",
                 "shape_emitter", "roots", "bsdfs_ingested")  # bdpt_scene_export_layout ids 0..12


@dataclass
class SceneDesc:
    """bdpt_scene_desc as numpy arrays: the Scene a caller already holds in memory
    (core.h:352-358) - triangles in (shape, face) order, materials with their
    constructed constants, emitters with their CDFs, the flat Fast-BVH and the
    BVH's object order."""
    positions: np.ndarray   # float32 (n, 9)
    normals: np.ndarray     # float32 (n, 9)
    tri_shape: np.ndarray   # int32 (n,)
    tri_prim: np.ndarray
    tri_mat: np.ndarray
    shapes: int
    materials: list         # dicts: illum kd ks ke tf ns ni scale spec_weight has_texture
    emitters: list          # dicts: shape area radiance cdf
    bvh: np.ndarray         # structured (bmin f4[3], bmax f4[3], start u4, nprims u4, right_offset u4)
    bvh_order: np.ndarray   # int32 (n,)


BVH_NODE_DTYPE = np.dtype([("bmin", "<f4", 3), ("bmax", "<f4", 3), ("start", "<u4"), ("nprims", "<u4"),
                           ("right_offset", "<u4")])


class _Stats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("samples", ctypes.c_int64), ("launches", ctypes.c_int64),
                ("counters", ctypes.c_int64 * len(COUNTER_NAMES)),  # BDPT_NUM_COUNTERS
                ("capped_samples", ctypes.c_int64), ("span_ms", ctypes.c_double), ("tail_ms", ctypes.c_double),
                ("max_light_depth", ctypes.c_int64), ("max_eye_depth", ctypes.c_int64),
                ("max_queries", ctypes.c_int64), ("schedule_errors", ctypes.c_int64), ("sched", ctypes.c_int64 * 4),
                ("parked_samples", ctypes.c_int64), ("rr_long_walks_max", ctypes.c_int64),
                ("rr_express_iters", ctypes.c_int64 * 3)]


# Sources that make up the frame kernels' code objects: their hash stamps the
# profiles (PMC passes) so bench.py only reuses a measurement of the same kernel.
KERNEL_SOURCES = ("csrc/bdpt_kernels.hip", "csrc/bdpt_kernels_split.hip", "csrc/bdpt_path.hpp", "csrc/bdpt_device.hpp", "csrc/device_math.hpp",
                  "csrc/bdpt_types.h", "Makefile")


def kernel_build_hash() -> str:
    """sha256[:16] over the frame kernel's sources and build flags."""
    import hashlib

    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(HERE, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def build(force: bool = False) -> str:
    """Compiles lib/libbdpt_amd.so in-tree with hipcc for gfx950."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE, "-j4"], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BdptError(f"{LIB_PATH} is missing: run build() (hipcc --offload-arch=gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, f32p = ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_float)
        L.bdpt_last_error.restype = ctypes.c_char_p
        L.bdpt_version.restype = ctypes.c_char_p
        L.bdpt_last_kernel.restype = ctypes.c_char_p
        L.bdpt_last_kernel.argtypes = [ctypes.c_void_p]
        L.bdpt_set_row_order.argtypes = [vp, vp, i32]
        L.bdpt_get_row_costs.argtypes = [vp, vp, i32]
        L.bdpt_scene_load_obj.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
        L.bdpt_scene_free.argtypes = [vp]
        L.bdpt_scene_get_info.argtypes = [vp, ctypes.POINTER(_SceneInfo)]
        L.bdpt_scene_export.argtypes = [vp, vp, vp, vp, vp]
        L.bdpt_scene_export_traversal.argtypes = [vp, vp, vp, vp, vp]
        L.bdpt_intersect_from.argtypes = [vp, ctypes.c_int64, vp, vp, vp, i32, vp]
        L.bdpt_scene_create.argtypes = [ctypes.POINTER(_SceneDesc), ctypes.POINTER(vp)]
        L.bdpt_scene_export_layout.argtypes = [vp, i32, vp, ctypes.POINTER(ctypes.c_int64)]
        L.bdpt_camera_constants.argtypes = [ctypes.POINTER(_Camera), i32, i32, f32p]
        L.bdpt_device_count.argtypes = [ctypes.POINTER(i32)]
        L.bdpt_ctx_create.argtypes = [vp, i32, ctypes.POINTER(vp)]
        L.bdpt_ctx_destroy.argtypes = [vp]
        L.bdpt_render.argtypes = [vp, ctypes.POINTER(_FrameParams), vp, vp]
        L.bdpt_render_host.argtypes = [vp, ctypes.POINTER(_FrameParams), vp]
        L.bdpt_render_sample.argtypes = [vp, ctypes.POINTER(_FrameParams), f32p, ctypes.c_uint32,
                                         ctypes.POINTER(i32), f32p, vp]
        L.bdpt_sampler_state.argtypes = [ctypes.c_uint32, ctypes.c_int64, vp]
        L.bdpt_render_sample_mt.argtypes = [vp, ctypes.POINTER(_FrameParams), f32p, vp, f32p,
                                            ctypes.POINTER(_Splat), i32, ctypes.POINTER(i32)]
        L.bdpt_render_path_sample_mt.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_PathParams), f32p,
                                                 vp, f32p]
        L.bdpt_render_direct_sample_mt.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_DirectParams),
                                                   f32p, vp, f32p]
        i64 = ctypes.c_int64
        L.bdpt_bsdf_eval.argtypes = [vp, i64, vp, vp, vp, vp]
        L.bdpt_bsdf_pdf.argtypes = [vp, i64, vp, vp, vp, vp]
        L.bdpt_bsdf_sample.argtypes = [vp, i64, vp, vp, vp, vp, vp, vp]
        L.bdpt_bsdf_type.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(i32)]
        L.bdpt_intersect.argtypes = [vp, i64, vp, i32, vp]
        L.bdpt_splat_to_image_plane.argtypes = [vp, ctypes.POINTER(_FrameParams), i64, vp, vp]
        L.bdpt_debug_fresnel.argtypes = [i32, i64, vp, vp]
        L.bdpt_debug_triangle.argtypes = [i32, i64, vp, vp, vp]
        L.bdpt_get_stats.argtypes = [vp, ctypes.POINTER(_Stats)]
        L.bdpt_multi_create.argtypes = [vp, i32, vp, ctypes.POINTER(vp)]
        L.bdpt_multi_destroy.argtypes = [vp]
        L.bdpt_multi_render_host.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_PathParams),
                                             ctypes.POINTER(_DirectParams), vp]
        L.bdpt_multi_get_stats.argtypes = [vp, ctypes.POINTER(_MultiStats)]
        L.bdpt_synchronize.argtypes = [vp]
        L.bdpt_config_load_toml.argtypes = [ctypes.c_char_p, ctypes.POINTER(_Config)]
        L.bdpt_render_path.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_PathParams), vp, vp]
        L.bdpt_render_path_host.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_PathParams), vp]
        for fn, pt in (("bdpt_render_path_sample", _PathParams), ("bdpt_render_direct_sample", _DirectParams)):
            getattr(L, fn).argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(pt), f32p, ctypes.c_uint32,
                                       ctypes.POINTER(i32), f32p]
        L.bdpt_render_direct.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_DirectParams), vp, vp]
        L.bdpt_render_direct_host.argtypes = [vp, ctypes.POINTER(_FrameParams), ctypes.POINTER(_DirectParams), vp]
        L.bdpt_direct_strategy.restype = i32
        L.bdpt_direct_strategy.argtypes = [ctypes.c_char_p]
        L.bdpt_debug_math.argtypes = [i32, i32, vp, vp, vp, ctypes.c_int64]
        L.bdpt_encode_exr.argtypes = [vp, i32, i32, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        L.bdpt_save_exr.argtypes = [vp, i32, i32, ctypes.c_char_p]
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        raise BdptError(f"bdpt error {rc}: {lib().bdpt_last_error().decode()}")


def device_count() -> int:
    n = ctypes.c_int32(0)
    _check(lib().bdpt_device_count(ctypes.byref(n)))
    return n.value


@dataclass
class Camera:
    eye: tuple = (0.0, 0.8, 3.8)
    at: tuple = (0.0, 0.8, 0.0)
    up: tuple = (0.0, 1.0, 0.0)
    fov: float = 30.0

    def c(self) -> _Camera:
        c = _Camera()
        c.eye[:], c.at[:], c.up[:] = list(map(float, self.eye)), list(map(float, self.at)), list(map(float, self.up))
        c.fov = float(self.fov)
        return c


@dataclass
class Config:
    """The subset of the reference's Config (core.h:195-248) the BDPT path reads."""
    camera: Camera = field(default_factory=Camera)
    width: int = 768   # main.cpp:41-42 defaults
    height: int = 576
    spp: int = 1       # main.cpp:112
    rr_depth: int = 5  # main.cpp:105
    rr_prob: float = 0.0  # read but unused by bdpt.h (its rrProbability is luminance-based, bdpt.h:127-129)
    strategy: int = STRATEGY_BDPT
    russian_roulette: int = 0  # RR_NONE: NO_RR = 1 as shipped (bdpt.h:18); RR_LUMINANCE: its NO_RR = 0 branch
    seed_base: int = REFERENCE_SEED


@dataclass
class PathSettings:
    """PathTracerIntegrator settings ([renderer] of a type = "path" scene, main.cpp:96-101)."""
    explicit: bool = True
    max_depth: int = -1
    rr_depth: int = 5
    rr_prob: float = 0.95
    emitter_samples: int = 1
    bsdf_samples: int = 0

    def c(self) -> _PathParams:
        p = _PathParams()
        p.is_explicit, p.max_depth, p.rr_depth = int(self.explicit), self.max_depth, self.rr_depth
        p.rr_prob, p.emitter_samples, p.bsdf_samples = self.rr_prob, self.emitter_samples, self.bsdf_samples
        return p


# DirectIntegrator::render's samplingStrategy strings (direct.h:450-461) -> BDPT_DIRECT_*
DIRECT_STRATEGIES = {"area": 1, "solidAngle": 2, "cosineHemisphere": 3, "bsdf": 4, "mis": 5}


@dataclass
class DirectSettings:
    """DirectIntegrator settings ([renderer] of a type = "direct" scene, main.cpp:88-92)."""
    sampling_strategy: str = "emitter"  # the reference's default, which its render() rejects
    emitter_samples: int = 1
    bsdf_samples: int = 1

    def c(self) -> _DirectParams:
        d = _DirectParams()
        d.sampling_strategy = DIRECT_STRATEGIES.get(self.sampling_strategy, 0)
        d.emitter_samples, d.bsdf_samples = self.emitter_samples, self.bsdf_samples
        return d


@dataclass
class SceneConfig:
    """loadTOML's result (main.cpp:22-116): the scene file settings, plus the
    objfile resolved as Scene::load does (renderer.cpp:236-241)."""
    toml_file: str
    obj_file: str
    obj_file_raw: str
    config: Config
    realtime: bool
    integrator: str
    path: PathSettings = field(default_factory=PathSettings)
    direct: DirectSettings = field(default_factory=DirectSettings)


def load_toml(path: str) -> SceneConfig:
    c = _Config()
    _check(lib().bdpt_config_load_toml(path.encode(), ctypes.byref(c)))
    cam = Camera(eye=tuple(c.camera.eye), at=tuple(c.camera.at), up=tuple(c.camera.up), fov=c.camera.fov)
    cfg = Config(camera=cam, width=c.width, height=c.height, spp=c.spp, rr_depth=c.rr_depth, rr_prob=c.rr_prob)
    pp = c.path
    path = PathSettings(explicit=bool(pp.is_explicit), max_depth=pp.max_depth, rr_depth=pp.rr_depth,
                        rr_prob=pp.rr_prob, emitter_samples=pp.emitter_samples, bsdf_samples=pp.bsdf_samples)
    direct = DirectSettings(sampling_strategy=c.sampling_strategy.decode(), emitter_samples=c.direct.emitter_samples,
                            bsdf_samples=c.direct.bsdf_samples)
    return SceneConfig(toml_file=c.toml_file.decode(), obj_file=c.obj_file.decode(),
                       obj_file_raw=c.obj_file_raw.decode(), config=cfg, realtime=bool(c.realtime),
                       integrator=c.integrator.decode(), path=path, direct=direct)


def encode_exr(rgb: np.ndarray, width: int, height: int) -> bytes:
    """saveEXR's bytes (utils.h:95-156): half-float B, G, R planes, uncompressed."""
    fb = np.ascontiguousarray(rgb, dtype=np.float32).reshape(-1)
    if fb.size != width * height * 3:
        raise BdptError(f"framebuffer has {fb.size} floats, expected {width * height * 3}")
    n = ctypes.c_int64(0)
    _check(lib().bdpt_encode_exr(fb.ctypes.data, width, height, None, 0, ctypes.byref(n)))
    out = np.zeros(n.value, np.uint8)
    _check(lib().bdpt_encode_exr(fb.ctypes.data, width, height, out.ctypes.data, n.value, ctypes.byref(n)))
    return out.tobytes()


def save_exr(rgb: np.ndarray, width: int, height: int, path: str) -> None:
    """Integrator::save (integrator.cpp:26-30)."""
    fb = np.ascontiguousarray(rgb, dtype=np.float32).reshape(-1)
    if fb.size != width * height * 3:
        raise BdptError(f"framebuffer has {fb.size} floats, expected {width * height * 3}")
    _check(lib().bdpt_save_exr(fb.ctypes.data, width, height, path.encode()))


@dataclass
class Ray:
    o: tuple
    d: tuple
    min_t: float = 1e-8
    max_t: float = 3.402823466e38


MT19937_WORDS = 625  # BDPT_MT19937_WORDS: _M_x[624], _M_p (libstdc++'s operator<< order)


def _mt_twist(x: np.ndarray) -> None:
    """mersenne_twister_engine::_M_gen_rand (libstdc++ random.tcc) on x[0:624] in place."""
    up, lo, a = np.uint32(0x80000000), np.uint32(0x7FFFFFFF), np.uint32(0x9908B0DF)
    for k in range(624):
        y = (x[k] & up) | (x[(k + 1) % 624] & lo)
        x[k] = x[(k + 397) % 624] ^ (y >> np.uint32(1)) ^ (a if y & np.uint32(1) else np.uint32(0))


class Sampler:
    """The reference's Sampler (src/core/math.h:63-76): a std::mt19937 and a
    uniform_real_distribution<float>. `state` is the engine as libstdc++ streams
    it (_M_x[624], then the position _M_p); the single-sample renders take and
    advance it exactly as the reference does."""

    def __init__(self, seed: int):
        rs = np.random.RandomState(int(seed) & 0xFFFFFFFF)  # init_genrand == std::mt19937(seed)
        key, pos = rs.get_state()[1:3]
        self.state = np.concatenate([key.astype(np.uint32), [np.uint32(pos)]]).astype(np.uint32)

    @staticmethod
    def from_state(state) -> "Sampler":
        s = Sampler(0)
        st = np.ascontiguousarray(state, np.uint32).reshape(-1)
        if st.size != MT19937_WORDS or st[-1] > 624:
            raise ValueError("a std::mt19937 state is 624 words and a position <= 624")
        s.state = st.copy()
        return s

    @staticmethod
    def for_sample(pixel: int, spp: int, k: int, base: int = REFERENCE_SEED) -> "Sampler":
        return Sampler((base + pixel * spp + k) & 0xFFFFFFFF)

    def next_u32(self) -> int:
        x = self.state
        if x[624] >= 624:
            _mt_twist(x)
            x[624] = 0
        y = int(x[int(x[624])])
        x[624] += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def next(self) -> float:
        """Sampler::next: generate_canonical<float, 24> (random.tcc:3348-3380)."""
        f = np.float32(self.next_u32()) / np.float32(4294967296.0)
        return float(f) if f < 1.0 else float(np.float32(0.99999994))

    def next2D(self) -> tuple:
        x = self.next()
        return x, self.next()


class Scene:
    def __init__(self, obj_path: str):
        h = ctypes.c_void_p()
        _check(lib().bdpt_scene_load_obj(obj_path.encode(), ctypes.byref(h)))
        self._h = h
        self.path = obj_path

    @classmethod
    def from_desc(cls, d: SceneDesc) -> "Scene":
        """bdpt_scene_create: the scene handed over from arrays the caller holds."""
        keep = []

        def arr(a, dt, shape=None):
            a = np.ascontiguousarray(np.asarray(a, dt))
            if shape is not None:
                a = a.reshape(shape)
            keep.append(a)
            return a.ctypes.data

        n = int(np.asarray(d.tri_shape).size)
        mats = (_MaterialDesc * max(len(d.materials), 1))()
        for k, m in enumerate(d.materials):
            mats[k].illum = int(m["illum"])
            for f in ("kd", "ks", "ke", "tf"):
                getattr(mats[k], f)[:] = [float(x) for x in m[f]]
            mats[k].ns, mats[k].ni = float(m["ns"]), float(m["ni"])
            mats[k].scale, mats[k].spec_weight = float(m.get("scale", 1.0)), float(m.get("spec_weight", 0.0))
            mats[k].has_texture = int(m.get("has_texture", 0))
        ems = (_EmitterDesc * max(len(d.emitters), 1))()
        for k, e in enumerate(d.emitters):
            ems[k].shape, ems[k].area = int(e["shape"]), float(e["area"])
            ems[k].radiance[:] = [float(x) for x in e["radiance"]]
            ems[k].ncdf = int(np.asarray(e["cdf"]).size)
            ems[k].cdf = arr(e["cdf"], np.float32)
        c = _SceneDesc()
        c.triangles = n
        c.positions, c.normals = arr(d.positions, np.float32), arr(d.normals, np.float32)
        c.tri_shape, c.tri_prim, c.tri_mat = arr(d.tri_shape, np.int32), arr(d.tri_prim, np.int32), arr(d.tri_mat,
                                                                                                           np.int32)
        c.shapes, c.materials, c.material = int(d.shapes), len(d.materials), ctypes.addressof(mats)
        c.emitters, c.emitter = len(d.emitters), ctypes.addressof(ems)
        bvh = np.ascontiguousarray(np.asarray(d.bvh, BVH_NODE_DTYPE))
        keep.append(bvh)
        c.bvh_nodes, c.bvh = int(bvh.size), bvh.ctypes.data
        c.bvh_order = arr(d.bvh_order, np.int32)
        h = ctypes.c_void_p()
        _check(lib().bdpt_scene_create(ctypes.byref(c), ctypes.byref(h)))
        self = cls.__new__(cls)
        self._h, self.path = h, None
        return self

    def export_layout(self, array) -> bytes:
        """bdpt_scene_export_layout: one of the device arrays (LAYOUT_ARRAYS) as bytes."""
        i = LAYOUT_ARRAYS.index(array) if isinstance(array, str) else int(array)
        n = ctypes.c_int64(0)
        _check(lib().bdpt_scene_export_layout(self._h, i, None, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(max(n.value, 1))
        _check(lib().bdpt_scene_export_layout(self._h, i, buf, ctypes.byref(n)))
        return buf.raw[:n.value]

    def to_desc(self) -> SceneDesc:
        """The descriptor of this scene, rebuilt from its exports (BVH leaf order back
        to (shape, face) order; materials and emitters from the ingested records)."""
        inf = self.info()
        tf, ti, nf, nu = self.export()
        perm = np.lexsort((ti[:, 1], ti[:, 0]))  # (shape, prim) order
        order = np.empty_like(perm)
        order[perm] = np.arange(perm.size)
        rec = np.frombuffer(self.export_layout("bsdfs_ingested"), np.uint32).reshape(-1, 18)
        recf = rec.view(np.float32)
        mats = [dict(illum=KIND_ILLUM[int(r[0])], kd=f[2:5], ks=f[5:8], tf=f[8:11], ke=f[11:14], ns=f[14], ni=f[15],
                     scale=f[16], spec_weight=f[17]) for r, f in zip(rec, recf)]
        em = np.frombuffer(self.export_layout("emitters"), np.int32).reshape(-1, 12)
        cdf = np.frombuffer(self.export_layout("emit_cdf"), np.float32)
        ems = [dict(shape=int(e[0]), area=e.view(np.float32)[4], radiance=e.view(np.float32)[5:8],
                    cdf=cdf[e[3]:e[3] + e[1] + 1]) for e in em]
        bvh = np.zeros(nf.shape[0], BVH_NODE_DTYPE)
        bvh["bmin"], bvh["bmax"] = nf[:, :3], nf[:, 3:]
        bvh["start"], bvh["nprims"], bvh["right_offset"] = nu[:, 0], nu[:, 1], nu[:, 2]
        return SceneDesc(positions=tf[perm, :9], normals=tf[perm, 9:], tri_shape=ti[perm, 0], tri_prim=ti[perm, 1],
                         tri_mat=ti[perm, 2], shapes=inf["shapes"], materials=mats, emitters=ems, bvh=bvh,
                         bvh_order=order.astype(np.int32))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.bdpt_scene_free(self._h)
            self._h = None

    def info(self) -> dict:
        i = _SceneInfo()
        _check(lib().bdpt_scene_get_info(self._h, ctypes.byref(i)))
        return {n: getattr(i, n) for n, _ in _SceneInfo._fields_}

    def bsdf_type(self, mat: int) -> tuple:
        """(BSDF::getType() flags, kind) of material `mat` (core.h:311; kind 1 diffuse,
        2 mirror, 3 glass, 4 mixture, 5 phong, 0 null)."""
        t, k = ctypes.c_uint32(0), ctypes.c_int32(0)
        _check(lib().bdpt_bsdf_type(self._h, mat, ctypes.byref(t), ctypes.byref(k)))
        return t.value, k.value

    def export(self):
        """(tri_f32[n,18], tri_i32[n,3], node_f32[m,6], node_u32[m,3]) in the reference's dump layout."""
        inf = self.info()
        n, m = inf["triangles"], inf["bvh_nodes"]
        tf, ti = np.zeros((n, 18), np.float32), np.zeros((n, 3), np.int32)
        nf, nu = np.zeros((m, 6), np.float32), np.zeros((m, 3), np.uint32)
        _check(lib().bdpt_scene_export(self._h, tf.ctypes.data, ti.ctypes.data, nf.ctypes.data, nu.ctypes.data))
        return tf, ti, nf, nu

    def export_traversal(self):
        """(wnodes[k,8,4], wtri[n,3,4], lbox[l,2,4], root_link): the traversal tree
        (wide_bvh.hpp); the link / index / leaf-id words are uint32 bit patterns."""
        inf = self.info()
        wn = np.zeros((inf["wide_nodes"], 8, 4), np.float32)
        wt = np.zeros((inf["triangles"], 3, 4), np.float32)
        lb = np.zeros((inf["bvh_leaves"], 2, 4), np.float32)
        root = ctypes.c_uint32()
        _check(lib().bdpt_scene_export_traversal(self._h, wn.ctypes.data, wt.ctypes.data, lb.ctypes.data,
                                                 ctypes.byref(root)))
        return wn, wt, lb, int(root.value)


def camera_constants(cam: Camera, width: int, height: int) -> np.ndarray:
    out = np.zeros(72, np.float32)
    c = cam.c()
    _check(lib().bdpt_camera_constants(ctypes.byref(c), width, height,
                                       out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return out


class BDPTIntegrator:
    """GPU BDPT integrator with the reference's Integrator interface."""

    def __init__(self, scene: Scene, config: Config, device: int = 0):
        self.scene = scene
        self.config = config
        self.device = device
        h = ctypes.c_void_p()
        _check(lib().bdpt_ctx_create(scene._h, device, ctypes.byref(h)))
        self._h = h
        self.rgb = None

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.bdpt_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def init(self) -> bool:
        self.rgb = np.zeros((self.config.height, self.config.width, 3), np.float32)
        return True

    def params(self, row_offset: int = 0, row_stride: int = 1, flags: int = 0) -> _FrameParams:
        c = self.config
        p = _FrameParams()
        p.camera = c.camera.c()
        p.width, p.height, p.spp, p.rr_depth = c.width, c.height, c.spp, c.rr_depth
        p.strategy, p.seed_base = c.strategy, c.seed_base & 0xFFFFFFFF
        p.row_offset, p.row_stride, p.flags = row_offset, row_stride, flags
        p.russian_roulette = c.russian_roulette
        return p

    def render(self, ray: Ray, sampler: Sampler) -> np.ndarray:
        """Integrator::render(const Ray&, Sampler&) (bdpt.h:219-241): Li of one
        camera sample; its light-path splats are added to self.rgb in order; the
        sampler's std::mt19937 state advances as the reference advances it."""
        if self.rgb is None:
            self.init()
        Li, splats = self.render_sample(ray, sampler)
        rgb = self.rgb.reshape(-1, 3)
        for px, v in splats:
            rgb[px] += v
        return Li

    def render_sample(self, ray: Ray, sampler: Sampler):
        """bdpt_render_sample_mt: (Li, [(pixel, rgb float32[3]), ...]) of one sample."""
        r = (ctypes.c_float * 8)(*ray.o, *ray.d, ray.min_t, ray.max_t)
        cap = max(self.config.rr_depth, 1)
        sp = (_Splat * cap)()
        n = ctypes.c_int32(0)
        Li = (ctypes.c_float * 3)()
        p = self.params()
        st = np.ascontiguousarray(sampler.state, np.uint32)
        rc = lib().bdpt_render_sample_mt(self._h, ctypes.byref(p), r, st.ctypes.data, Li, sp, cap, ctypes.byref(n))
        if rc == -1 and n.value > cap:  # Russian roulette: more splats than rr_depth; the state is untouched
            cap = n.value
            sp = (_Splat * cap)()
            rc = lib().bdpt_render_sample_mt(self._h, ctypes.byref(p), r, st.ctypes.data, Li, sp, cap, ctypes.byref(n))
        _check(rc)
        sampler.state = st
        return np.array(Li[:], np.float32), [(sp[k].pixel, np.array(sp[k].rgb[:], np.float32)) for k in range(n.value)]

    # ---- the BSDF plugin contract and the path's building blocks (per-function entry points)
    def bsdf_eval(self, mat, wo, wi) -> np.ndarray:
        """BSDF::eval (core.h:308) of scene materials mat[k] on local directions: f * cos(wi), (n, 3)."""
        m, o, i = _ai32(mat), _af32(wo, 3), _af32(wi, 3)
        out = np.zeros((m.size, 3), np.float32)
        _check(lib().bdpt_bsdf_eval(self._h, m.size, m.ctypes.data, o.ctypes.data, i.ctypes.data, out.ctypes.data))
        return out

    def bsdf_pdf(self, mat, wo, wi) -> np.ndarray:
        """BSDF::pdf (core.h:309): the solid-angle pdf of wi, (n,)."""
        m, o, i = _ai32(mat), _af32(wo, 3), _af32(wi, 3)
        out = np.zeros(m.size, np.float32)
        _check(lib().bdpt_bsdf_pdf(self._h, m.size, m.ctypes.data, o.ctypes.data, i.ctypes.data, out.ctypes.data))
        return out

    def bsdf_sample(self, mat, wo, u):
        """BSDF::sample (core.h:310): (f * cos, wi, pdf) for samples u (n, 2)."""
        m, o, uu = _ai32(mat), _af32(wo, 3), _af32(u, 2)
        f, wi, pdf = np.zeros((m.size, 3), np.float32), np.zeros((m.size, 3), np.float32), np.zeros(m.size, np.float32)
        _check(lib().bdpt_bsdf_sample(self._h, m.size, m.ctypes.data, o.ctypes.data, uu.ctypes.data, f.ctypes.data,
                                      wi.ctypes.data, pdf.ctypes.data))
        return f, wi, pdf

    def intersect(self, rays, occlusion: bool = False, origin_normals=None, origin_tris=None) -> np.ndarray:
        """AcceleratorBVH::intersect (accel.h:125-172) or the occlusion query of
        visibilityQuery (bvh.h:259-352) on rays (n, 8): a structured bdpt_hit array.
        origin_normals (n, 3): the surfaces the rays leave (the path's interpolated
        shading normals), origin_tris (n,): their triangles (bdpt_hit.tri order, -1:
        none), for the frames' near-cull rule (bdpt_intersect_from); None: no near cull."""
        r = _af32(rays, 8)
        out = np.zeros(r.shape[0], HIT_DTYPE)
        if origin_normals is None:
            _check(lib().bdpt_intersect(self._h, r.shape[0], r.ctypes.data, 1 if occlusion else 0, out.ctypes.data))
        else:
            nr = _af32(origin_normals, 3)
            ot = None if origin_tris is None else np.ascontiguousarray(origin_tris, np.int32).reshape(-1)
            if ot is not None and ot.shape[0] != r.shape[0]:
                raise ValueError("origin_tris needs one entry per ray")
            _check(lib().bdpt_intersect_from(self._h, r.shape[0], r.ctypes.data, nr.ctypes.data,
                                             None if ot is None else ot.ctypes.data, 1 if occlusion else 0,
                                             out.ctypes.data))
        return out

    def splat_to_image_plane(self, points) -> np.ndarray:
        """BDPTIntegrator::splatToImagePlane (bdpt.h:485-496) of points (n, 3): int32 (n, 2)."""
        q = _af32(points, 3)
        out = np.zeros((q.shape[0], 2), np.int32)
        p = self.params()
        _check(lib().bdpt_splat_to_image_plane(self._h, ctypes.byref(p), q.shape[0], q.ctypes.data, out.ctypes.data))
        return out

    def render_frame(self, row_offset: int = 0, row_stride: int = 1, flags: int = 0) -> np.ndarray:
        """All pixels x spp of the (sharded) image into self.rgb (host copy)."""
        if self.rgb is None:
            self.init()
        p = self.params(row_offset, row_stride, flags)
        _check(lib().bdpt_render_host(self._h, ctypes.byref(p), self.rgb.ctypes.data))
        return self.rgb

    def render_device(self, fb_ptr: int, stream_ptr: int = 0, row_offset: int = 0, row_stride: int = 1,
                      flags: int = 0) -> None:
        """Asynchronous render into a device framebuffer (e.g. a torch tensor's data_ptr())."""
        p = self.params(row_offset, row_stride, flags)
        _check(lib().bdpt_render(self._h, ctypes.byref(p), ctypes.c_void_p(fb_ptr), ctypes.c_void_p(stream_ptr)))

    def stats(self) -> dict:
        s = _Stats()
        _check(lib().bdpt_get_stats(self._h, ctypes.byref(s)))
        return dict(kernel_ms=s.kernel_ms, samples=s.samples, launches=s.launches,
                    counters=dict(zip(COUNTER_NAMES, list(s.counters))), capped_samples=s.capped_samples,
                    span_ms=s.span_ms, tail_ms=s.tail_ms, max_light_depth=s.max_light_depth,
                    max_eye_depth=s.max_eye_depth, max_queries=s.max_queries, schedule_errors=s.schedule_errors, parked_samples=s.parked_samples,
                    rr_long_walks_max=s.rr_long_walks_max, rr_express_iters=list(s.rr_express_iters),
                    sched=dict(zip(("step_tasks", "shade_steps", "steps_ge32", "steps_ge64"), list(s.sched))),
                    kernel=(lib().bdpt_last_kernel(self._h) or b"").decode())

    def synchronize(self) -> None:
        _check(lib().bdpt_synchronize(self._h))

    def set_row_order(self, order) -> None:
        """Claim order of the shard's local rows for later renders (bdpt_set_row_order);
        None or [] restores top to bottom. Changes no sample, only which run last."""
        a = np.ascontiguousarray(np.asarray([] if order is None else order, dtype=np.int32))
        _check(lib().bdpt_set_row_order(self._h, a.ctypes.data if a.size else None, int(a.size)))

    def row_costs(self, nrows: int) -> np.ndarray:
        """Queries per local row of the last FLAG_COUNT render (bdpt_get_row_costs)."""
        out = np.zeros(nrows, np.int64)
        _check(lib().bdpt_get_row_costs(self._h, out.ctypes.data, int(nrows)))
        return out

    def save(self, path: str) -> None:
        """Integrator::save: self.rgb as the reference's EXR."""
        save_exr(self.rgb, self.config.width, self.config.height, path)


def cost_row_order(costs) -> np.ndarray:
    """Local rows by descending cost (ties top to bottom): the costly rows are claimed
    first, so the samples still in flight when a shard's work runs out are cheap ones."""
    c = np.asarray(costs)
    return np.lexsort((np.arange(c.size), -c)).astype(np.int32)


class PathTracerIntegrator(BDPTIntegrator):
    """The reference's PathTracerIntegrator (src/integrators/path.h) on the same
    GPU substrate: render(ray, sampler), render_frame and render_device as for BDPT."""

    def __init__(self, scene: Scene, config: Config, path: PathSettings | None = None, device: int = 0):
        super().__init__(scene, config, device)
        self.path = path or PathSettings()

    def render(self, ray: Ray, sampler: Sampler) -> np.ndarray:
        """PathTracerIntegrator::render(const Ray&, Sampler&) (path.h:235-245): Li of
        one sample; the sampler's std::mt19937 state advances."""
        r = (ctypes.c_float * 8)(*ray.o, *ray.d, ray.min_t, ray.max_t)
        Li = (ctypes.c_float * 3)()
        p, pp = self.params(), self.path.c()
        st = np.ascontiguousarray(sampler.state, np.uint32)
        _check(lib().bdpt_render_path_sample_mt(self._h, ctypes.byref(p), ctypes.byref(pp), r, st.ctypes.data, Li))
        sampler.state = st
        return np.array(Li[:], np.float32)

    def render_frame(self, row_offset: int = 0, row_stride: int = 1, flags: int = 0) -> np.ndarray:
        if self.rgb is None:
            self.init()
        p, pp = self.params(row_offset, row_stride, flags), self.path.c()
        _check(lib().bdpt_render_path_host(self._h, ctypes.byref(p), ctypes.byref(pp), self.rgb.ctypes.data))
        return self.rgb

    def render_device(self, fb_ptr: int, stream_ptr: int = 0, row_offset: int = 0, row_stride: int = 1,
                      flags: int = 0) -> None:
        """Asynchronous; call check_levels() after the stream is synchronised: a
        sample that outgrew the 512-level recursion stack makes the frame differ
        from the reference's (render_frame checks this itself)."""
        p, pp = self.params(row_offset, row_stride, flags), self.path.c()
        _check(lib().bdpt_render_path(self._h, ctypes.byref(p), ctypes.byref(pp), ctypes.c_void_p(fb_ptr),
                                      ctypes.c_void_p(stream_ptr)))

    def check_levels(self) -> None:
        """Raises BdptError if a sample of the last render_device call outgrew the
        level stack (bdpt_get_stats counters[1] of bdpt_render_path)."""
        n = self.stats()["counters"]["shadow_rays"]
        if n:
            raise BdptError(f"{n} path samples outgrew the 512-level recursion stack")


class DirectIntegrator(BDPTIntegrator):
    """The reference's DirectIntegrator (src/integrators/direct.h) on the same GPU
    substrate: one bounce of direct light by area, solid-angle, cosine-hemisphere,
    BSDF or MIS sampling, with the emitters as the spheres the reference makes of
    them (renderer.cpp:349-358)."""

    def __init__(self, scene: Scene, config: Config, direct: DirectSettings | None = None, device: int = 0):
        super().__init__(scene, config, device)
        self.direct = direct or DirectSettings(sampling_strategy="mis")

    def render(self, ray: Ray, sampler: Sampler) -> np.ndarray:
        """DirectIntegrator::render(const Ray&, Sampler&) (direct.h:449-462): Li of one
        sample; the sampler's std::mt19937 state advances."""
        r = (ctypes.c_float * 8)(*ray.o, *ray.d, ray.min_t, ray.max_t)
        Li = (ctypes.c_float * 3)()
        p, d = self.params(), self.direct.c()
        st = np.ascontiguousarray(sampler.state, np.uint32)
        _check(lib().bdpt_render_direct_sample_mt(self._h, ctypes.byref(p), ctypes.byref(d), r, st.ctypes.data, Li))
        sampler.state = st
        return np.array(Li[:], np.float32)

    def render_frame(self, row_offset: int = 0, row_stride: int = 1, flags: int = 0) -> np.ndarray:
        if self.rgb is None:
            self.init()
        p, d = self.params(row_offset, row_stride, flags), self.direct.c()
        _check(lib().bdpt_render_direct_host(self._h, ctypes.byref(p), ctypes.byref(d), self.rgb.ctypes.data))
        return self.rgb

    def render_device(self, fb_ptr: int, stream_ptr: int = 0, row_offset: int = 0, row_stride: int = 1,
                      flags: int = 0) -> None:
        p, d = self.params(row_offset, row_stride, flags), self.direct.c()
        _check(lib().bdpt_render_direct(self._h, ctypes.byref(p), ctypes.byref(d), ctypes.c_void_p(fb_ptr),
                                        ctypes.c_void_p(stream_ptr)))


class MultiDeviceRenderer:
    """One process, several HIP devices (bdpt_multi_*): the reference's parallel_for
    over host threads (parallelfor.h:25-65) as one context and stream per device,
    interleaved row shards, and one RCCL sum-reduce of the frames to devices[0].
    A repeated device (e.g. [0, 0]) rehearses the decomposition on one GPU with a
    local sum instead of RCCL."""

    def __init__(self, scene: Scene, config: Config, devices=(0,), path: PathSettings | None = None,
                 direct: DirectSettings | None = None):
        self.scene, self.config, self.devices = scene, config, list(devices)
        self.path, self.direct = path, direct
        dev = (ctypes.c_int32 * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _check(lib().bdpt_multi_create(scene._h, len(self.devices), dev, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.bdpt_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def render_frame(self) -> np.ndarray:
        c = self.config
        p = _FrameParams()
        p.camera = c.camera.c()
        p.width, p.height, p.spp = c.width, c.height, c.spp
        p.rr_depth = 1 if (self.path or self.direct) else c.rr_depth  # rrDepth is the BDPT setting
        p.strategy, p.seed_base = c.strategy, c.seed_base & 0xFFFFFFFF
        p.row_offset, p.row_stride, p.flags = 0, 1, 0
        rgb = np.zeros((c.height, c.width, 3), np.float32)
        pp = ctypes.byref(self.path.c()) if self.path else None
        dp = ctypes.byref(self.direct.c()) if self.direct else None
        _check(lib().bdpt_multi_render_host(self._h, ctypes.byref(p), pp, dp, rgb.ctypes.data))
        return rgb

    def stats(self) -> dict:
        s = _MultiStats()
        _check(lib().bdpt_multi_get_stats(self._h, ctypes.byref(s)))
        n = s.devices
        return dict(devices=n, rccl=bool(s.rccl), wall_ms=s.wall_ms, render_ms=s.render_ms, reduce_ms=s.reduce_ms,
                    samples=s.samples, kernel_ms=list(s.kernel_ms)[:n], device_samples=list(s.device_samples)[:n],
                    capped_samples=s.capped_samples, schedule_errors=s.schedule_errors)


def debug_math(fn: str, x: np.ndarray, y: np.ndarray | None = None, device: int = 0) -> np.ndarray:
    """The device sinf / cosf / powf (glibc restatements) on float32 inputs:
    fn in {"sinf", "cosf", "powf", "sincos_s", "sincos_c"}."""
    code = {"sinf": 0, "cosf": 1, "powf": 2, "sincos_s": 3, "sincos_c": 4}[fn]
    x = np.ascontiguousarray(x, np.float32)
    yy = None if y is None else np.ascontiguousarray(y, np.float32)
    out = np.empty_like(x)
    _check(lib().bdpt_debug_math(device, code, x.ctypes.data, None if yy is None else yy.ctypes.data,
                                 out.ctypes.data, x.size))
    return out


def debug_fresnel(inp, device: int = 0) -> np.ndarray:
    """GlassBSDF::FresnelDielectric (glass.h:40-53) on (n, 4) = (eta_i, eta_t, cos_i, cos_t)."""
    x = _af32(inp, 4)
    out = np.zeros(x.shape[0], np.float32)
    _check(lib().bdpt_debug_fresnel(device, x.shape[0], x.ctypes.data, out.ctypes.data))
    return out


def debug_triangle(rays, verts, device: int = 0) -> np.ndarray:
    """rayTriangleIntersect (core.h:379-400): (n, 4) = (hit, t, u, v) for rays (n, 8), verts (n, 9)."""
    r, v = _af32(rays, 8), _af32(verts, 9)
    out = np.zeros((r.shape[0], 4), np.float32)
    _check(lib().bdpt_debug_triangle(device, r.shape[0], r.ctypes.data, v.ctypes.data, out.ctypes.data))
    return out
